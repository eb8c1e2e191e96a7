# Fused path on the GPU: fused/keygen/parity tests, then a same-process A/B against variant
# libraries. Usage on the GPU box: bash tools/fz4_check.sh <tag> <libs>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-fz4}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fused.py tests/test_gpu_keygen.py tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.txt | head -20; exit 1; }
timeout -k 10 200 python3 tools/ab_fused.py --libs $2 --reps 4 > $O/ab.txt 2>&1; cat $O/ab.txt

# The whole GPU test suite, then a same-process A/B of the eval (and fused) paths against variant
# libraries. Usage on the GPU box: bash tools/ev_check.sh <tag> <libs>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ev}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/tests.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.txt | head -30; exit 1; }
timeout -k 10 200 python3 tools/ab_fused.py --libs $2 --reps 4 --eval > $O/ab.txt 2>&1; cat $O/ab.txt

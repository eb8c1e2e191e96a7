set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/fz2; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fused.py tests/test_gpu_keygen.py -x -v --timeout 240 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 $O/tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python3 tools/ab_fused.py --libs zk-odst_amd/variants/libb2f_v1.so,zk-odst_amd/variants/libb2f_pf2.so --reps 4 > $O/ab.txt 2>&1; cat $O/ab.txt
timeout -k 10 120 python3 tools/eval_phases.py --fused 155 > $O/phases.txt 2>&1; cat $O/phases.txt

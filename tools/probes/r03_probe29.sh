# Eval fast pass with three register sets at 2 waves per SIMD: the eval parity
# tests, then one-process A/B of the eval against HEAD.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_evalfast.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $OUT/eval_tests.txt 2>&1; rc=$?
tail -2 $OUT/eval_tests.txt
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
timeout -k 10 500 python3 tools/ab_fused.py --libs "zk-odst_amd/variants/libb2f_head.so,zk-odst_amd/libb2f_diag.so" --modes 27 --eval --reps 4 > $OUT/ab_eval_xyz.txt 2>&1; ok
echo done

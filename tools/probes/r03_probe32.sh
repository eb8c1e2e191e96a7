# Edge tile stores: one instruction per column for both regions (per-lane offsets in one
# resource) instead of one per region: fused GPU tests, then one-process A/B against HEAD.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fused.py tests/test_gpu_keygen.py tests/test_gpu_hasher.py -x -v --timeout 300 --timeout-method thread > $OUT/fused_tests.txt 2>&1; rc=$?
tail -2 $OUT/fused_tests.txt
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
timeout -k 10 500 python3 tools/ab_fused.py --libs "zk-odst_amd/variants/libb2f_head.so,zk-odst_amd/libb2f_diag.so" --modes 27 --reps 4 > $OUT/ab_edge_store.txt 2>&1; ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o p --output-format csv -- python3 $R/tools/ab_fused.py --libs "zk-odst_amd/variants/libb2f_head.so" --modes 27 --reps 2 > /dev/null 2>&1; ok
echo done

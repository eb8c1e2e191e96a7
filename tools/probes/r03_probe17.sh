# Fused half-round stores at 3 workgroups per CU: split around the lookup checks (6 / 3 columns
# first) and cache policies (non-temporal, sc0), one process, interleaved.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fused.py -x -q --timeout 200 --timeout-method thread > $OUT/fused_tests.txt 2>&1; ok
V=zk-odst_amd/variants
timeout -k 10 500 python3 tools/ab_fused.py --libs "zk-odst_amd/libb2f_diag.so,$V/libb2f_sp6.so,$V/libb2f_sp3.so,$V/libb2f_nt.so,$V/libb2f_sc0.so" --modes 27 --fill --reps 4 > $OUT/ab_split_policy.txt 2>&1; ok
echo done

# Staging columns with the tail rows in front (one LDS stride, no per-column select): every GPU
# test, then one-process A/B against the TL-area form and the pre-line-ownership form, and the
# workgroups-per-CU sweep of the new form.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; ok
V=zk-odst_amd/variants
timeout -k 10 400 python3 tools/ab_fused.py --libs "$V/libb2f_tl.so,$V/libb2f_pre.so,zk-odst_amd/libb2f_diag.so@B2F_FUSED_PERCU=3,zk-odst_amd/libb2f_diag.so@B2F_FUSED_PERCU=1" --modes 27 --fill --reps 4 > $OUT/ab_stride.txt 2>&1; ok
echo done

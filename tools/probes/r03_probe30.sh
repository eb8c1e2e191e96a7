# Edge tiles in the half-round launch's last workgroups: every GPU test, then one-process A/B of
# the edge workgroup count (0 = HEAD's separate edge launch) against HEAD.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -2 $OUT/gpu_tests.txt
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
D=zk-odst_amd/libb2f_diag.so
timeout -k 10 600 python3 tools/ab_fused.py --libs "zk-odst_amd/variants/libb2f_head.so,$D@B2F_FUSED_EDGE_BLOCKS=0,$D@B2F_FUSED_EDGE_BLOCKS=48,$D@B2F_FUSED_EDGE_BLOCKS=64,$D@B2F_FUSED_EDGE_BLOCKS=96" --modes 27 --reps 4 > $OUT/ab_edge_blocks.txt 2>&1; ok
echo done

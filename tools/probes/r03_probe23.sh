# The half-round launch walking whole instances (state carried tile to tile, lite record): every
# GPU test, then one-process A/B against HEAD's tile-dealt launch.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
tail -3 $OUT/gpu_tests.txt
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
timeout -k 10 500 python3 tools/ab_fused.py --libs "zk-odst_amd/variants/libb2f_head.so,zk-odst_amd/libb2f_diag.so" --modes 27,2 --fill --reps 4 > $OUT/ab_seq.txt 2>&1; ok
echo done

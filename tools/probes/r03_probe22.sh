# Half-round launch dealt in bands of consecutive tiles per wave visit (4, 24 = one 12-round
# instance per visit) vs single tiles.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
V=zk-odst_amd/variants
timeout -k 10 500 python3 tools/ab_fused.py --libs "zk-odst_amd/libb2f_diag.so,$V/libb2f_band4.so,$V/libb2f_band24.so" --modes 27,2 --fill --reps 4 > $OUT/ab_band.txt 2>&1; ok
echo done

# Eval fast pass: non-temporal cell loads, 48-tile bands (one process, interleaved).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
V=zk-odst_amd/variants
timeout -k 10 500 python3 tools/ab_fused.py --libs "zk-odst_amd/libb2f_diag.so,$V/libb2f_evnt.so,$V/libb2f_band48.so" --modes 27 --eval --reps 4 > $OUT/ab_eval.txt 2>&1; ok
echo done

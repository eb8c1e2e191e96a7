# Eval fast pass check-group costs (diagnostics build): modes 0 (staging only), 1 (lookups),
# 8 (gates), 16 (copies), 27 (all) -- the fast pass alone, one process.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
D=zk-odst_amd/libb2f_diag.so
timeout -k 10 500 python3 tools/ab_fused.py --libs "$D@B2F_DIAG_EVALFAST=0,$D@B2F_DIAG_EVALFAST=1,$D@B2F_DIAG_EVALFAST=8,$D@B2F_DIAG_EVALFAST=16,$D@B2F_DIAG_EVALFAST=27" --modes 27 --eval --reps 3 > $OUT/ab_evalfast_modes.txt 2>&1; ok
echo done

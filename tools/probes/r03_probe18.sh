# Non-temporal half-round stores: every GPU test, PERCU sweep against HEAD's write-back build,
# then the round evidence (bench line, rocprof stats, PMC traffic).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; ok
D=zk-odst_amd/libb2f_diag.so
timeout -k 10 500 python3 tools/ab_fused.py --libs "zk-odst_amd/variants/libb2f_wb.so,$D@B2F_FUSED_PERCU=2,$D@B2F_FUSED_PERCU=3,$D@B2F_FUSED_PERCU=4" --modes 27 --fill --reps 4 > $OUT/ab_nt_percu.txt 2>&1; ok
bash tools/round_profile.sh $TAG/round > $OUT/round.log 2>&1; ok
echo done

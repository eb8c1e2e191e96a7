# Final evidence of the round at HEAD: host probe, every GPU test, smoke, bench, the N = 2
# rehearsals (gpu_check.sh), then the round profile (bench, rocprof stats, PMC traffic).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
bash tools/gpu_check.sh $TAG/check > $OUT/check.log 2>&1 || { echo "gpu_check rc=$?"; tail -5 $OUT/check.log; exit 1; }
bash tools/round_profile.sh $TAG/round > $OUT/round.log 2>&1 || { echo "round rc=$?"; exit 2; }
echo done

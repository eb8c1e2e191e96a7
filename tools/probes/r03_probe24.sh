# Round evidence at HEAD (instance-walking half-round launch): bench line, rocprof stats, PMC
# traffic (round_profile.sh), smoke.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 120 python3 -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.txt 2>&1 || { echo "smoke rc=$?"; exit 1; }
bash tools/round_profile.sh $TAG/round > $OUT/round.log 2>&1 || { echo "round rc=$?"; exit 2; }
echo done

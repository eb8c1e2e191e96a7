# GPU tests, then the PMC of the fused kernel's modes 27/2/0 (tools/pmc_fused.sh) and the
# per-phase clocks (tools/fz_phases.sh). Usage on the box: bash tools/r03_check.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || exit 1
bash tools/pmc_fused.sh 27,2,0 > $OUT/pmc.log 2>&1 || exit 2
cp gpurun_out/pmcf/summary.txt $OUT/pmc_summary.txt
bash tools/fz_phases.sh $TAG/fzp > $OUT/phases.log 2>&1 || exit 3
echo done

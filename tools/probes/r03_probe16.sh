# PMC of the fused half-round kernel at HEAD (3 workgroups per CU): modes 27 (full), 2 (stores,
# no checks), 0 (assign only) beside the fill and eval; phase clocks of the same modes.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
bash tools/pmc_fused.sh 27,2,0 > $OUT/pmc_fused.log 2>&1; ok
cp gpurun_out/pmcf/summary.txt $OUT/pmc_summary.txt
bash tools/fz_phases.sh $TAG/fzp > $OUT/phases.log 2>&1; ok
timeout -k 10 300 python3 tools/ab_fused.py --libs "zk-odst_amd/libb2f_diag.so" --modes 27,2,0 --fill --reps 3 > $OUT/ab_modes.txt 2>&1; ok
echo done

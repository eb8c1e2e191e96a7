# Line-aligned fused kernel: where the time goes now (modes 27 / 2 / 0 and 1 workgroup per CU,
# in one process) and its PMC (instructions, LDS bank conflicts) beside the eval fast pass.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 300 python3 tools/ab_fused.py --libs "zk-odst_amd/libb2f_diag.so,zk-odst_amd/libb2f_diag.so@B2F_FUSED_PERCU=1" --modes 27,2,0 --fill --eval --reps 3 > $OUT/ab_modes.txt 2>&1; ok
timeout -k 10 700 bash tools/pmc_fused.sh 27,2,0 > $OUT/pmc_fused.log 2>&1; ok
cp -r gpurun_out/pmcf $OUT/ 2>/dev/null
echo done

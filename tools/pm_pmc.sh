# SQ / TCC counters of the permutation-columns kernels (three rocprofv3 --pmc passes of
# tools/bench_lookup.py, each its own run), summarised per kernel by tools/pmc_kernels.py.
# Usage on the GPU box: bash tools/pm_pmc.sh <tag> [lib]
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-pmpmc}
LIB=${2:+--lib $2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
B="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
C="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
D="FETCH_SIZE"
E="WRITE_SIZE"
for p in ${PASSES:-a b c d e}; do
  eval CN=\$$(echo $p | tr a-e A-E)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CN -d $OUT/pm_$p -o p --output-format csv -- python3 $R/tools/bench_perm.py --forms 3 --reps 1 $LIB > $OUT/pm_$p.log 2>&1 || { echo pm pmc $p failed; exit 3; }
done
cd $R
python3 tools/pmc_kernels.py "$OUT/pm_*" pm_,gp_ > $OUT/pm_pmc.txt
cat $OUT/pm_pmc.txt | cut -c1-400

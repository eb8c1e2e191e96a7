# PMC probe of the fused kernel's diagnostic modes beside the fill and eval (diagnostics).
# Usage on the GPU box: bash tools/pmc_fused.sh [modes]   (outputs under gpurun_out/pmcf/)
R=$GRAFT_REPO_ROOT
M=${1:-27,2,0}
OUT=$R/gpurun_out/pmcf
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
A="--reps 1 --fill-modes 3 --eval-modes 7 --fused-modes $M"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT/a -o p --output-format csv -- python3 $R/tools/ablate.py $A > $OUT/a.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM -d $OUT/b -o p --output-format csv -- python3 $R/tools/ablate.py $A > $OUT/b.log 2>&1
echo rc=$?
cd $R && python3 tools/pmc_summary.py gpurun_out/pmcf > gpurun_out/pmcf/summary.txt; cat gpurun_out/pmcf/summary.txt

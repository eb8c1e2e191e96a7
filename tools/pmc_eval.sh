R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmce
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT/a -o p --output-format csv -- python3 $R/tools/ablate.py --reps 1 --fill-modes 3 --eval-modes 7,1,2,4 > $OUT/a.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d $OUT/b -o p --output-format csv -- python3 $R/tools/ablate.py --reps 1 --fill-modes 3 --eval-modes 7,1,2,4 > $OUT/b.log 2>&1
echo rc=$?

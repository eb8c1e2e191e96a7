# SQ counters of the eval fast pass (eval_hr_kernel / eval_edge_kernel, the split path's product
# eval) in two rocprofv3 --pmc passes of a small bench.py --path split run, summarised per kernel
# by tools/pmc_kernels.py (the LDS-side counters that bound a staging ring).
# Usage on the GPU box: bash tools/pmc_evalfast.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-evfpmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
B="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES"
ARGS="--path split --steps 2 --warmup 1 --no-cpu --export-rows 0 --aux-steps 1 --floor-reps 0 --lookup-circuits 0 --perm-k 0 --hasher-messages 0 --config4 0 --witness-gather 0"
for p in a b; do
  eval CN=\$$(echo $p | tr ab AB)
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $CN -d $OUT/ev_$p -o p --output-format csv -- python3 $R/bench.py $ARGS > $OUT/ev_$p.log 2>&1 || { echo evalfast pmc $p failed; exit 3; }
done
cd $R
python3 tools/pmc_kernels.py "$OUT/ev_*" eval_hr,eval_edge > $OUT/evalfast_pmc.txt
cut -c1-400 $OUT/evalfast_pmc.txt

# The fused pass against the split fill on ONE box: the interleaved
# fill_eval / fill min ratio (tools/ab_fused.py --fill), then the s_memtime phase clocks of the
# fused half-round kernel (B2F_DIAG_FUSED=155) and of the fill kernel (B2F_DIAG_FILL=11).
# Usage on the GPU box: bash tools/fz_vs_fill.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-fzf}; mkdir -p $O
timeout -k 10 300 python3 tools/ab_fused.py --fill --reps 5 > $O/ab.txt 2>&1 || exit 1
timeout -k 10 120 python3 tools/eval_phases.py --fused 155 > $O/phases_fused.txt 2>&1 || exit 2
timeout -k 10 120 python3 tools/eval_phases.py --fill > $O/phases_fill.txt 2>&1 || exit 3
grep -hv amdgpu.ids $O/ab.txt $O/phases_fused.txt $O/phases_fill.txt

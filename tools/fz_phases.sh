# Phase clocks of the fused half-round kernel (diagnostics build): full, stores only, assign only.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-fzp}; mkdir -p $O
for m in 155 130 128; do
  timeout -k 10 120 python3 tools/eval_phases.py --fused $m >> $O/phases.txt 2>&1 || exit 1
done
cat $O/phases.txt

# Same-process A/B of fused variants (diagnostics builds under zk-odst_amd/variants/), with the
# per-check-group ablation modes. Usage on the GPU box: bash tools/fz3_check.sh <tag> <libs> [modes]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-fz3}; mkdir -p $O
timeout -k 10 300 python3 tools/ab_fused.py --libs $2 --modes ${3:-27} --reps 3 > $O/ab.txt 2>&1; rc=$?
cat $O/ab.txt; exit $rc

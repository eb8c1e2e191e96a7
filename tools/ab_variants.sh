# A/B timing of library variants on one box (diagnostics): bash tools/ab_variants.sh v1 v2 ...
# (zk-odst_amd/variants/libb2f_<v>.so built beforehand; ablate.py args via AB_ARGS)
set -o pipefail
ARGS=${AB_ARGS:---reps 3 --fill-modes 3 --eval-modes 7 --fused-modes 27}
for v in "$@"; do
  timeout -k 10 150 python tools/ablate.py --lib $GRAFT_REPO_ROOT/zk-odst_amd/variants/libb2f_$v.so $ARGS > gpurun_out/ab_$v.txt 2>&1 || exit 1
done

set -o pipefail
for rep in 1 2; do
for v in f1 f6; do
 for w in 8 5 4; do
  B2F_FILL_WGS=$w timeout -k 10 100 python tools/ablate.py --lib $GRAFT_REPO_ROOT/zk-odst_amd/variants/libb2f_$v.so --reps 2 --fill-modes 3 --eval-modes 7 > gpurun_out/fab_${v}_$w.txt 2>&1 || exit 1
 done
done
done

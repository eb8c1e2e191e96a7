# Box characterization in one process per tool: fill floor (DIAG_FILL=2) vs the fill, eval load
# floor, fused modes 27/2/0; then the fused launch at 2/3/4 workgroups per CU and the two-tiles-
# ahead word prefetch (B2F_HR_PF2), interleaved (tools/ab_fused.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 300 python3 tools/ablate.py --reps 3 --fill-modes 3,2 --eval-modes 7,1 --fused-modes 27,2,0 > $OUT/ablate.txt 2>&1; ok
D=zk-odst_amd/libb2f_diag.so
V=zk-odst_amd/variants/libb2f_pf2.so
timeout -k 10 400 python3 tools/ab_fused.py --reps 3 --libs "$D@B2F_FUSED_PERCU=2,$D@B2F_FUSED_PERCU=3,$D@B2F_FUSED_PERCU=4,$V@B2F_FUSED_PERCU=2,$V@B2F_FUSED_PERCU=3" > $OUT/ab_percu.txt 2>&1; ok

timeout -k 10 400 python3 -u tools/hasher_race.py 4 > $OUT/hasher_race.txt 2>&1; ok
echo done

# Line ownership on / off in one process (same code: the variant forces kc = tc = 0), against the
# pre-ownership revision, at 2 and 3 workgroups per CU.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
V=zk-odst_amd/variants
D=zk-odst_amd/libb2f_diag.so
timeout -k 10 500 python3 tools/ab_fused.py --libs "$D,$D@B2F_FUSED_PERCU=3,$V/libb2f_noown.so,$V/libb2f_noown.so@B2F_FUSED_PERCU=3,$V/libb2f_pre.so,$V/libb2f_pre.so@B2F_FUSED_PERCU=3" --modes 27,2 --fill --reps 4 > $OUT/ab_own.txt 2>&1; ok
echo done

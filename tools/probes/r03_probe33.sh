# Edge launch: workgroups per CU (1/2/3) and store policy (write-back vs non-temporal), one process.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
D=zk-odst_amd/libb2f_diag.so
timeout -k 10 600 python3 tools/ab_fused.py --libs "$D@B2F_EDGE_PERCU=1,$D@B2F_EDGE_PERCU=2,$D@B2F_EDGE_PERCU=3,zk-odst_amd/variants/libb2f_edgewb.so" --modes 27 --reps 4 > $OUT/ab_edge_percu.txt 2>&1; ok
echo done

# Session restart: every GPU test at HEAD, then one-process A/B of the half-round launch's
# workgroups per CU (HEAD at 2/3/4, the pre-line-ownership revision at 2/3), then the bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; ok
V=zk-odst_amd/variants
D=zk-odst_amd/libb2f_diag.so
timeout -k 10 500 python3 tools/ab_fused.py --libs "$D@B2F_FUSED_PERCU=2,$D@B2F_FUSED_PERCU=3,$D@B2F_FUSED_PERCU=4,$V/libb2f_pre.so@B2F_FUSED_PERCU=2,$V/libb2f_pre.so@B2F_FUSED_PERCU=3" --modes 27,2 --fill --reps 4 > $OUT/ab_percu.txt 2>&1; ok
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err; ok

SKIP_TESTS=1 bash tools/prover_check.sh $TAG/pc; ok
echo done

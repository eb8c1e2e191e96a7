# Every GPU test (3 workgroups per CU by default, lookup count/block_down changes); eval fast
# pass workgroups per CU A/B; lookup A/B vs HEAD; lookup/perm per-kernel profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; ok
tail -2 $OUT/gpu_tests.txt
D=zk-odst_amd/libb2f_diag.so
timeout -k 10 400 python3 tools/ab_fused.py --libs "$D@B2F_EVAL_PERCU=2,$D@B2F_EVAL_PERCU=3,$D@B2F_EVAL_PERCU=4" --modes 27 --eval --fill --reps 3 > $OUT/ab_eval_percu.txt 2>&1; ok
V=zk-odst_amd/variants
for rep in 1 2; do
for L in $V/libb2f_lkold.so zk-odst_amd/libb2f.so; do
  timeout -k 10 120 python3 tools/bench_lookup.py --form 3 --lib $L >> $OUT/ab_lookup.jsonl 2>/dev/null; ok
done
done
SKIP_TESTS=1 bash tools/prover_check.sh $TAG/pc; ok
echo done

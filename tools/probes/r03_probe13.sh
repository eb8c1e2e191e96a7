# Lookup columns: the index + factor/chunk kernels vs HEAD's per-row permute (same process
# order, same box), unroll variants; then every lookup GPU test and the product's profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lookup.py -x -v --timeout 120 --timeout-method thread > $OUT/lookup_tests.txt 2>&1; ok
V=zk-odst_amd/variants
for rep in 1 2; do
for L in $V/libb2f_lkold.so zk-odst_amd/libb2f.so $V/libb2f_lku4.so $V/libb2f_lku8.so; do
  timeout -k 10 120 python3 tools/bench_lookup.py --form 3 --lib $L >> $OUT/ab_lookup.jsonl 2>/dev/null; ok
done
done
SKIP_TESTS=1 bash tools/prover_check.sh $TAG/pc; ok
echo done

# Lookup columns + Fp export on the GPU: parity tests, then throughput per form and a
# per-kernel rocprof summary. Usage on the GPU box: bash tools/lk_check.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-lk}
mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lookup.py tests/test_gpu_parity.py -k "lookup or fp_export" -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
tail -4 $O/tests.txt
[ $rc -eq 0 ] || exit 1
for f in 1 0 3 2; do
  timeout -k 10 120 python3 tools/bench_lookup.py --form $f >> $O/bench.jsonl 2>&1 || exit 2
done
cat $O/bench.jsonl
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o lk --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_lookup.py --form 3 > /dev/null 2>&1 || exit 3
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/$O/kernel_stats.csv \;
cut -d, -f1-4 $GRAFT_REPO_ROOT/$O/kernel_stats.csv | head -14

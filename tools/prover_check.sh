# Prover-column kernels on the GPU: lookup/permutation/spread-table/export parity tests, then
# throughput and a per-kernel rocprof summary. Usage on the GPU box: bash tools/prover_check.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pc}
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lookup.py tests/test_gpu_perm.py tests/test_gpu_parity.py -k "lookup or perm or spread or fp_export" -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
  tail -4 $O/tests.txt
  [ $rc -eq 0 ] || exit 1
fi
for f in 1 3; do
  timeout -k 10 120 python3 tools/bench_lookup.py --form $f >> $O/bench_lookup.jsonl 2>&1 || exit 2
done
timeout -k 10 200 python3 tools/bench_perm.py >> $O/bench_perm.jsonl 2>&1 || exit 3
grep -h '^{' $O/bench_lookup.jsonl $O/bench_perm.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_lk -o lk --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_lookup.py --form 3 > /dev/null 2>&1 || exit 4
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_pm -o pm --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_perm.py --forms 3 > /dev/null 2>&1 || exit 5
find $GRAFT_REPO_ROOT/$O/prof_lk -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/$O/lookup_kernel_stats.csv \;
find $GRAFT_REPO_ROOT/$O/prof_pm -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/$O/perm_kernel_stats.csv \;
echo done

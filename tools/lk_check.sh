# Lookup columns + Fp export on the GPU: parity tests, then throughput per form and a
# per-kernel rocprof summary. Usage on the GPU box: bash tools/lk_check.sh <tag>
#   SKIP_TESTS=1  skip the parity tests;  AB="name1 name2"  also time variant libraries
#   zk-odst_amd/variants/libb2f_<name>.so (tools/build_variant.sh), interleaved with the product
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-lk}
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lookup.py tests/test_gpu_parity.py -k "lookup or fp_export" -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
  tail -4 $O/tests.txt
  [ $rc -eq 0 ] || exit 1
fi
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/bench_lookup.py --form 1 >> $O/bench.jsonl 2>&1 || exit 2
  for v in $AB; do
    timeout -k 10 120 python3 tools/bench_lookup.py --form 1 --lib zk-odst_amd/variants/libb2f_$v.so >> $O/bench.jsonl 2>&1 || exit 2
  done
done
timeout -k 10 120 python3 tools/bench_lookup.py --form 3 >> $O/bench.jsonl 2>&1 || exit 2
cat $O/bench.jsonl
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o lk --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_lookup.py --form 1 > /dev/null 2>&1 || exit 3
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/$O/kernel_stats.csv \;
python3 $GRAFT_REPO_ROOT/tools/kstats.py $GRAFT_REPO_ROOT/$O/kernel_stats.csv 1

# Permutation columns on the GPU: parity tests, then the per-proof z call and the keygen sigma
# call per form, interleaved with variant libraries (AB="name ..." -> zk-odst_amd/variants/
# libb2f_<name>.so), and a per-kernel rocprof summary. Usage: bash tools/pm_check.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pm}
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_perm.py -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1; rc=$?
  tail -3 $O/tests.txt
  [ $rc -eq 0 ] || exit 1
fi
for rep in 1 2; do
  timeout -k 10 200 python3 tools/bench_perm.py --forms 3 >> $O/bench.jsonl 2>&1 || exit 2
  for v in $AB; do
    timeout -k 10 200 python3 tools/bench_perm.py --forms 3 --lib zk-odst_amd/variants/libb2f_$v.so >> $O/bench.jsonl 2>&1 || exit 2
  done
done
grep -v amdgpu.ids $O/bench.jsonl
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o pm --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_perm.py --forms 3 > /dev/null 2>&1 || exit 3
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/$O/kernel_stats.csv \;
python3 $GRAFT_REPO_ROOT/tools/kstats.py $GRAFT_REPO_ROOT/$O/kernel_stats.csv 5

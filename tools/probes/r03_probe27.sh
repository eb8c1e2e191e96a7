# Lookup permute with wave-cooperative run searches: the lookup parity tests, then A/B against
# HEAD's per-row searches and the per-kernel profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lookup.py -x -v --timeout 200 --timeout-method thread > $OUT/lookup_tests.txt 2>&1; rc=$?
tail -2 $OUT/lookup_tests.txt
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
V=zk-odst_amd/variants
for rep in 1 2; do
for L in $V/libb2f_lkold.so zk-odst_amd/libb2f.so; do
  timeout -k 10 120 python3 tools/bench_lookup.py --form 3 --lib $L >> $OUT/ab_lookup.jsonl 2>/dev/null; ok
done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o lk --output-format csv -- python3 $R/tools/bench_lookup.py --form 3 > /dev/null 2>&1; ok
echo done

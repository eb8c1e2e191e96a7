# Lookup columns A/B: HEAD's per-row permute vs the index + factor/chunk kernels at unroll
# 1/2/4/16; rocprof per-kernel of the HEAD form.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
V=zk-odst_amd/variants
for rep in 1 2; do
for L in $V/libb2f_lkold.so zk-odst_amd/libb2f.so $V/libb2f_lku1.so $V/libb2f_lku2.so $V/libb2f_lku4.so; do
  timeout -k 10 120 python3 tools/bench_lookup.py --form 3 --lib $L >> $OUT/ab_lookup.jsonl 2>/dev/null; ok
done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_old -o lk --output-format csv -- python3 $R/tools/bench_lookup.py --form 3 --lib $R/$V/libb2f_lkold.so > /dev/null 2>&1; ok
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_u1 -o lk --output-format csv -- python3 $R/tools/bench_lookup.py --form 3 --lib $R/$V/libb2f_lku1.so > /dev/null 2>&1; ok
echo done

# Permutation factors with chunk_len 3 unrolled: the permutation parity tests, then A/B against HEAD.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_perm.py -x -v --timeout 200 --timeout-method thread > $OUT/perm_tests.txt 2>&1; rc=$?
tail -2 $OUT/perm_tests.txt
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit 1; }
for rep in 1 2; do
for L in zk-odst_amd/variants/libb2f_head.so zk-odst_amd/libb2f.so; do
  echo "lib $L" >> $OUT/ab_perm.jsonl
  timeout -k 10 200 python3 tools/bench_perm.py --forms 3 --lib $L >> $OUT/ab_perm.jsonl 2>/dev/null; ok
done
done
echo done

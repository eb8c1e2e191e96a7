# Lookup / permutation parity + bench with the reworked grand product; the store probe with the
# mixed-policy boundary-line variant.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lookup.py tests/test_gpu_perm.py -x -v --timeout 120 --timeout-method thread > $OUT/prover_tests.txt 2>&1; ok
for f in 1 3; do timeout -k 10 120 python3 tools/bench_lookup.py --form $f >> $OUT/lookup.jsonl 2>> $OUT/lookup.err; ok; done
timeout -k 10 120 python3 tools/bench_perm.py >> $OUT/perm.jsonl 2>> $OUT/perm.err; ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/lkprof -o p --output-format csv -- python3 $R/tools/bench_lookup.py --form 3 > $OUT/lkprof.log 2>&1; ok
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/pmprof -o p --output-format csv -- python3 $R/tools/bench_perm.py > $OUT/pmprof.log 2>&1; ok
cd $R
timeout -k 10 300 ./tools/store_probe 262144 a > $OUT/store_probe_align.jsonl 2>&1; ok
echo done

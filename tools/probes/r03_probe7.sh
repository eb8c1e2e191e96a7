# Lookup / permutation parity and timings after D moved onto the block totals; one bench.py line.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lookup.py tests/test_gpu_perm.py -x -v --timeout 120 --timeout-method thread > $OUT/prover_tests.txt 2>&1; ok
timeout -k 10 120 python3 tools/bench_lookup.py --form 3 >> $OUT/lookup.jsonl 2>> $OUT/lookup.err; ok
timeout -k 10 120 python3 tools/bench_perm.py >> $OUT/perm.jsonl 2>> $OUT/perm.err; ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/pmprof -o p --output-format csv -- python3 $R/tools/bench_perm.py > $OUT/pmprof.log 2>&1; ok
cd $R
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err; ok
echo done

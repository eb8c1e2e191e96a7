# Round-6 check (diagnostics; outputs under gpurun_out/<tag>/): the lookup with its table pass and
# sort on a third stream (tests, A/B against the sort-on-main variant, one call's timeline) and
# the export's column-stride / allocation-order question.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06e}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
V=zk-odst_amd/variants
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lookup.py tests/test_gpu_checks.py tests/test_gpu_perm.py -x -v --timeout 120 --timeout-method thread -m gpu > $OUT/tests.txt 2>&1 || exit 1
for rep in 1 2 3; do
  for lib in "" $V/libb2f_lksort0.so; do
    timeout -k 10 120 python3 tools/bench_lookup.py ${lib:+--lib $lib} >> $OUT/lookup_ab.jsonl 2>> $OUT/lookup_ab.err || exit 2
  done
done
timeout -k 10 300 python3 tools/bench_export.py --pads 0,1024,0,1024,64 --reps 4 > $OUT/export_alloc.txt 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/lkprof -o p --output-format csv -- python3 $R/tools/bench_lookup.py --reps 2 > $OUT/lkprof.log 2>&1 || exit 4
echo done

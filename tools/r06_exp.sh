# Round-6 A/B experiments in one GPU call (diagnostics; outputs under gpurun_out/<tag>/):
# eval fast-pass variants, export column-stride pads, lookup bounding variants, rocprof stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06b}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
V=zk-odst_amd/variants
timeout -k 10 400 python3 tools/ab_fused.py --libs $V/libb2f_r5head.so,$V/libb2f_evilv.so,$V/libb2f_evilv12.so,$V/libb2f_evilv48.so --eval --reps 5 > $OUT/ab_eval_ilv.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_export.py --pads 0,64,1024,4096 --reps 4 > $OUT/export_pads.txt 2>&1 || exit 2
for rep in 1 2 3; do
  for lib in "" $V/libb2f_lknowait.so $V/libb2f_lknoscan.so $V/libb2f_lkzt128.so; do
    timeout -k 10 120 python3 tools/bench_lookup.py ${lib:+--lib $lib} >> $OUT/lookup_bound.jsonl 2>> $OUT/lookup_bound.err || exit 3
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o p --output-format csv -- python3 $R/tools/ab_fused.py --eval --reps 3 > $OUT/prof.log 2>&1 || exit 4
echo done

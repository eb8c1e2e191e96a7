# One GPU call producing the round's evidence: the default bench line, a rocprofv3
# --kernel-trace --stats run of the same command, the PMC traffic passes (fused/fill/eval) and
# a FETCH_SIZE pass on the eval floor variants (eval_kernel<1>, load_stream_kernel) and the eval
# fast pass, diagnostics library.
# Usage on the GPU box: bash tools/round_profile.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-round}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o p --output-format csv -- python3 $R/bench.py --no-cpu --hasher-messages 0 > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit 2
cd $R && bash tools/pmc_traffic.sh > $OUT/traffic.log 2>&1 || exit 3
cp profiles/pmc_traffic.json $OUT/ 2>/dev/null
cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/evalfloor -o p --output-format csv -- python3 $R/tools/ablate.py --reps 2 --fill-modes 3 --eval-modes 1,7,32 > $OUT/evalfloor.log 2>&1 || exit 4
cd $R && python3 tools/pmc_fetch_by_kernel.py $OUT/evalfloor eval_kernel eval_hr_kernel load_stream_kernel > $OUT/evalfloor_fetch.json || exit 5
# bench again so its roofline.traffic picks up the PMC numbers just measured
timeout -k 10 400 python3 bench.py --cpu-seconds 5 > $OUT/bench_final.json 2> $OUT/bench_final.err || exit 6
echo done

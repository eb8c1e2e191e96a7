# HBM traffic per launch of fill/eval (FETCH_SIZE and WRITE_SIZE in separate passes, as
# MI355X_MICROARCH.md prescribes), summarised by tools/pmc_traffic.py into
# profiles/pmc_traffic.json. Usage on the GPU box: bash tools/pmc_traffic.sh [batch] [rounds]
R=$GRAFT_REPO_ROOT
B=${1:-262144}
RD=${2:-12}
OUT=$R/gpurun_out/traffic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $OUT/fetch -o p --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --export-rows 0 --aux-steps 1 --floor-reps 0 --lookup-circuits 0 --hasher-messages 0 --batch $B --rounds $RD > $OUT/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $OUT/write -o p --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --export-rows 0 --aux-steps 1 --floor-reps 0 --lookup-circuits 0 --hasher-messages 0 --batch $B --rounds $RD > $OUT/write.log 2>&1 && \
cd $R && python3 tools/pmc_traffic.py $OUT/fetch $OUT/write ${B}_${RD} profiles/pmc_traffic.json

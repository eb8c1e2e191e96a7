# Round evidence after the perm product count and the extras watchdog: every GPU test, smoke,
# bench, the N = 2 rehearsals (gpu_check.sh), then the watchdog firing inside the config-4 leg.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
bash tools/gpu_check.sh $TAG/check > $OUT/check.log 2>&1 || { echo "gpu_check rc=$?"; exit 1; }
B2F_BENCH_REHEARSE=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --batch 16384 --config4 32768 \
  --config4-world 2 --steps 3 --warmup 1 --extras-timeout 3 > $OUT/rehearse_watchdog.json 2> $OUT/rehearse_watchdog.err
echo "watchdog rehearsal rc=$?"
echo done

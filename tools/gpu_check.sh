# One GPU call: host probe, the GPU test suite, smoke, the default bench line, and a rehearsal
# of bench.py's N = 2 strong-scaling path (--global-batch, row-balanced mixed-rounds shards,
# witness gather) and of its config-4 leg, with both ranks on the one GPU over gloo.
# Usage on the GPU box: bash tools/gpu_check.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-check}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
{ nproc; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count())'
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; lscpu | head -20; free -g; } > $OUT/host.txt 2>&1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 120 python3 -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.txt 2>&1 || exit 2
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 3
B2F_BENCH_REHEARSE=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --global-batch 65536 --mix \
  --steps 3 --warmup 1 > $OUT/rehearse_n2.json 2> $OUT/rehearse_n2.err || exit 4
# bench.py's config-4 leg (weak headline, then a sharded batch + its full witness gather) at
# N = 2 with a small batch, then the same with the gather's memory check forced to skip
B2F_BENCH_REHEARSE=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --batch 16384 --config4 32768 \
  --config4-world 2 --steps 3 --warmup 1 > $OUT/rehearse_config4.json 2> $OUT/rehearse_config4.err || exit 5
B2F_BENCH_REHEARSE=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --batch 16384 --config4 32768 \
  --config4-world 2 --gather-cap-gb 1 --steps 3 --warmup 1 > $OUT/rehearse_config4_skip.json 2> $OUT/rehearse_config4_skip.err || exit 6
# bench.py --gpus 2 with no launcher: it spawns the two ranks itself
B2F_BENCH_REHEARSE=1 timeout -k 10 300 python3 bench.py --gpus 2 --batch 16384 --steps 3 --warmup 1 \
  > $OUT/rehearse_spawn_n2.json 2> $OUT/rehearse_spawn_n2.err || exit 7
echo done

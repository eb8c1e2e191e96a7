# The round's final evidence in one GPU call: the GPU test suite, smoke, the round profile (bench
# line, rocprofv3 kernel stats of the same command, PMC traffic stamped with these sources, the
# eval floor's FETCH_SIZE, the bench line again with the traffic), and bench.py --gpus 2 spawning
# its own two ranks (rehearsed on one GPU over gloo).
# Usage on the GPU box: bash tools/final_check.sh <tag>   (outputs under gpurun_out/<tag>/)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-final}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
{ nproc; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count())'
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; free -g; } > $OUT/host.txt 2>&1
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || exit 1
timeout -k 10 120 python3 -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.txt 2>&1 || exit 2
bash tools/round_profile.sh $TAG || exit 3
cd $R && B2F_BENCH_REHEARSE=1 timeout -k 10 300 python3 bench.py --gpus 2 --batch 16384 --steps 3 --warmup 1 \
  > $OUT/rehearse_spawn_n2.json 2> $OUT/rehearse_spawn_n2.err || exit 4
echo done

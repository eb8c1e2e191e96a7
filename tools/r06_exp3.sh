# Round-6 check (diagnostics; outputs under gpurun_out/<tag>/): the GPU tests the eval / perm /
# export changes touch, and the eval kernels under rocprof beside round 5's library.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06d}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
V=zk-odst_amd/variants
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_perm.py tests/test_gpu_parity.py tests/test_gpu_evalfast.py tests/test_gpu_checks.py tests/test_gpu_fused.py::test_max_rounds_instance -x -v --timeout 120 --timeout-method thread -m gpu > $OUT/tests.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o p --output-format csv -- python3 $R/tools/ab_fused.py --eval --reps 3 --libs $V/libb2f_r5head.so > $OUT/prof.log 2>&1 || exit 4
echo done1
# Fp export: workgroups per CU per form at the padded stride, the pasta pair form (variant)
cd $R
for pc in 2 3 4 5; do
  B2F_EXPORT_PERCU=$pc timeout -k 10 200 python3 tools/bench_export.py --libs zk-odst_amd/libb2f_diag.so,$V/libb2f_xpair.so --pads 1024 --reps 4 2>/dev/null | sed "s/^{/{\"percu\": $pc, /" >> $OUT/export_percu.jsonl || exit 5
done
echo done2
# one lookup call's kernel timeline (tools/lk_timeline.py reads it)
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/lkprof -o p --output-format csv -- python3 $R/tools/bench_lookup.py --reps 2 > $OUT/lkprof.log 2>&1 || exit 6
echo done3

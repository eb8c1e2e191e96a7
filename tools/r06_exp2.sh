# Round-6 A/B experiments (diagnostics; outputs under gpurun_out/<tag>/): permutation with and
# without the grand-product scratch pad and the output column pad, the eval descriptor kernel
# under rocprof, and the GPU tests the changes touch.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06c}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
V=zk-odst_amd/variants
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_perm.py tests/test_gpu_parity.py tests/test_gpu_evalfast.py tests/test_gpu_checks.py -x -v --timeout 120 --timeout-method thread -m gpu > $OUT/tests.txt 2>&1 || exit 1
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/bench_perm.py --forms 3 >> $OUT/perm_pad.jsonl 2>> $OUT/perm_pad.err || exit 2
  timeout -k 10 120 python3 tools/bench_perm.py --forms 3 --pad 0 >> $OUT/perm_pad.jsonl 2>> $OUT/perm_pad.err || exit 2
  timeout -k 10 120 python3 tools/bench_perm.py --forms 3 --pad 0 --lib $V/libb2f_gppad0.so >> $OUT/perm_pad.jsonl 2>> $OUT/perm_pad.err || exit 2
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o p --output-format csv -- python3 $R/tools/ab_fused.py --eval --reps 3 --libs $V/libb2f_r5head.so > $OUT/prof.log 2>&1 || exit 4
echo done

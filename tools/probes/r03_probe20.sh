# Fp export A/B: next-tile prefetch, 256 / 1024-row tiles; export parity tests first.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "export or spread" -x -q --timeout 200 --timeout-method thread > $OUT/export_tests.txt 2>&1; ok
V=zk-odst_amd/variants
timeout -k 10 300 python3 tools/bench_export.py --libs "$V/libb2f_xpf.so,$V/libb2f_xt256.so,$V/libb2f_xt1k.so" > $OUT/ab_export.jsonl 2>&1; ok
echo done

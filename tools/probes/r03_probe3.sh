# Lookup parity + bench, hasher race diagnostics, fused A/B (round-2 end vs HEAD) with eval, PMC
# of the fused modes 27/2/3/10/18 (all / none / lookups / gates / copies).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r03}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
ok() { rc=$?; [ $rc -le 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lookup.py tests/test_gpu_perm.py tests/test_gpu_fused.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.txt 2>&1; ok
for f in 1 3; do timeout -k 10 120 python3 tools/bench_lookup.py --form $f >> $OUT/lookup.jsonl 2>> $OUT/lookup.err; ok; done
timeout -k 10 200 python3 tools/ab_fused.py --libs zk-odst_amd/variants/libb2f_r02end.so,zk-odst_amd/variants/libb2f_chk1.so,zk-odst_amd/variants/libb2f_split6.so,zk-odst_amd/variants/libb2f_split3.so --eval --reps 4 > $OUT/ab.txt 2>&1; ok
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/lkprof -o p --output-format csv -- python3 $R/tools/bench_lookup.py --form 3 > $OUT/lkprof.log 2>&1; ok
cd $R
timeout -k 10 300 python3 -u tools/hasher_race.py 3 > $OUT/hasher_race.txt 2>&1; ok
bash tools/pmc_fused.sh 27,2,3,10,18 > $OUT/pmc.log 2>&1; ok
cp gpurun_out/pmcf/summary.txt $OUT/pmc_summary.txt
echo done

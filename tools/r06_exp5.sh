# Round-6 probes (diagnostics; outputs under gpurun_out/<tag>/): the lookup's sort stream at high
# priority (A/B), and whether store rates depend on the allocation written (export, fused pass).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06f}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
V=zk-odst_amd/variants
for rep in 1 2 3; do
  for lib in "" $V/libb2f_lks3prio.so; do
    timeout -k 10 120 python3 tools/bench_lookup.py ${lib:+--lib $lib} >> $OUT/lookup_prio.jsonl 2>> $OUT/lookup_prio.err || exit 1
  done
done
timeout -k 10 300 python3 tools/placement_probe.py --n 6 > $OUT/placement_export.jsonl 2> $OUT/placement_export.err || exit 2
timeout -k 10 300 python3 tools/placement_probe.py --fused 3 --reps 3 > $OUT/placement_fused.jsonl 2> $OUT/placement_fused.err || exit 3
echo done

# Round-6 probe (diagnostics; outputs under gpurun_out/<tag>/): the Fp export per allocation,
# product vs the column-staggered variant (both forms).
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-r06g}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python3 tools/placement_probe.py --n 6 --libs zk-odst_amd/variants/libb2f_xstag.so > $OUT/placement_export_stagger.jsonl 2> $OUT/placement_export_stagger.err || exit 1
echo done

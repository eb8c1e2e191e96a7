# Build the diagnostics library of another git revision as an A/B variant, without #ifdef
# variants in the product sources: the revision's csrc/ + include/ are exported to a scratch
# tree and compiled there.
#   bash tools/build_rev.sh <rev> <name> ["<extra hipcc flags>"]  ->  zk-odst_amd/variants/libb2f_<name>.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; N=$2; F=${3:-}
T=$(mktemp -d /tmp/b2f_rev.XXXXXX)
mkdir -p $T/zk-odst_amd/csrc $T/include
for f in $(git -C $ROOT ls-tree --name-only $REV zk-odst_amd/csrc/); do git -C $ROOT show $REV:$f > $T/$f; done
git -C $ROOT show $REV:include/b2f.h > $T/include/b2f.h
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950 -DB2F_DIAG $F"
O="-mllvm -amdgpu-atomic-optimizer-strategy=None"
cd $T/zk-odst_amd
$H $O -c -o k.o csrc/b2f_kernels.hip &
$H $O -c -o f.o csrc/b2f_fused.hip &
$H -c -o e.o csrc/b2f_export.hip &
$H -c -o l.o csrc/b2f_lookup.hip &
$H -c -o p.o csrc/b2f_perm.hip &
wait
mkdir -p $ROOT/zk-odst_amd/variants
$H -shared -o $ROOT/zk-odst_amd/variants/libb2f_$N.so k.o f.o e.o l.o p.o
rm -rf $T
echo built zk-odst_amd/variants/libb2f_$N.so from $REV

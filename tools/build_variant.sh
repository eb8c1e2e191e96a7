# Build a diagnostics library variant with extra compile flags on every source (A/B runs):
#   bash tools/build_variant.sh <name> "<flags>"  ->  zk-odst_amd/variants/libb2f_<name>.so
set -e
cd "$(dirname "$0")/../zk-odst_amd"
N=$1; F=$2
D=variants/build_$N
mkdir -p $D variants
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950 -DB2F_DIAG $F"
O="-mllvm -amdgpu-atomic-optimizer-strategy=None"
$H $O -c -o $D/k.o csrc/b2f_kernels.hip &
$H $O -c -o $D/f.o csrc/b2f_fused.hip &
$H -c -o $D/e.o csrc/b2f_export.hip &
$H -c -o $D/l.o csrc/b2f_lookup.hip &
$H -c -o $D/p.o csrc/b2f_perm.hip &
wait
$H -shared -o variants/libb2f_$N.so $D/k.o $D/f.o $D/e.o $D/l.o $D/p.o
rm -rf $D
echo built variants/libb2f_$N.so

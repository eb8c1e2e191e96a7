# Build a diagnostics library variant with extra compile flags (A/B runs, tools/ab_variants.sh):
#   bash tools/build_variant.sh <name> "<flags>"  ->  zk-odst_amd/variants/libb2f_<name>.so
set -e
cd "$(dirname "$0")/../zk-odst_amd"
N=$1; F=$2
D=variants/build_$N
mkdir -p $D variants
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -fvisibility=hidden --offload-arch=gfx950 -DB2F_DIAG $F"
$H -mllvm -amdgpu-atomic-optimizer-strategy=None -c -o $D/k.o csrc/b2f_kernels.hip &
$H -mllvm -amdgpu-atomic-optimizer-strategy=None -c -o $D/f.o csrc/b2f_fused.hip &
wait
$H -shared -o variants/libb2f_$N.so $D/k.o $D/f.o build/b2f_export.o build/b2f_lookup.o build/b2f_perm.o
echo built variants/libb2f_$N.so

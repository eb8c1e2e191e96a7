// Field-multiply throughput probe (diagnostics): chains of Montgomery products per lane, many
// waves, timed with HIP events; prints ns per product per CU-second equivalents.
//   hipcc -O3 --offload-arch=gfx950 -o tools/mulbench tools/mulbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include "../zk-odst_amd/csrc/b2f_field.h"
using namespace b2f::field;

template <class F>
__device__ __forceinline__ Fe mulB(const Fe& a, const Fe& b) {
  uint32_t t[8];
#pragma unroll
  for (int j = 0; j < 8; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t bi = b.w[i];
    uint64_t x = (uint64_t)a.w[0] * bi + t[0];
    uint32_t A = (uint32_t)(x >> 32);
    const uint32_t t0 = (uint32_t)x;
    const uint32_t m = t0 * F::NP;
    uint64_t y = (uint64_t)m * F::P[0] + t0;
    uint32_t C = (uint32_t)(y >> 32);
#pragma unroll
    for (int j = 1; j < 8; j++) {
      unsigned co;
      uint32_t lo = __builtin_addc(t[j], A, 0u, &co);
      x = (uint64_t)a.w[j] * bi + (((uint64_t)co << 32) | lo);
      A = (uint32_t)(x >> 32);
      uint32_t lo2 = __builtin_addc((uint32_t)x, C, 0u, &co);
      y = (uint64_t)m * F::P[j] + (((uint64_t)co << 32) | lo2);
      C = (uint32_t)(y >> 32);
      t[j - 1] = (uint32_t)y;
    }
    t[7] = C + A;
  }
  Fe r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.w[j] = t[j];
  return reduce_once<F>(r);
}

template <class F, int V, int CH>
__global__ __launch_bounds__(256) void k(const Fe* in, Fe* out, int n) {
  Fe acc[CH];
#pragma unroll
  for (int c = 0; c < CH; c++) acc[c] = in[(threadIdx.x + c) & 255];
  const Fe b = in[256 + (blockIdx.x & 15)];
  for (int i = 0; i < n; i++)
#pragma unroll
    for (int c = 0; c < CH; c++) acc[c] = V == 0 ? mul<F>(acc[c], b) : mulB<F>(acc[c], b);
  Fe s = acc[0];
#pragma unroll
  for (int c = 1; c < CH; c++) s = add<F>(s, acc[c]);
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ void madk(uint64_t* out, int n) {  // raw v_mad_u64_u32 chains, 8 independent
  uint64_t a[8];
  for (int c = 0; c < 8; c++) a[c] = threadIdx.x + c;
  const uint32_t b = blockIdx.x | 1;
  for (int i = 0; i < n; i++)
#pragma unroll
    for (int c = 0; c < 8; c++) a[c] = (uint64_t)(uint32_t)a[c] * b + (a[c] >> 32);
  uint64_t s = 0;
  for (int c = 0; c < 8; c++) s ^= a[c];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <class K>
float timeit(K launch) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  launch();
  hipEventRecord(e0);
  launch();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  Fe* in;
  Fe* out;
  hipMalloc(&in, 512 * sizeof(Fe));
  hipMemset(in, 0x11, 512 * sizeof(Fe));
  const int blocks = 256 * 16, n = 64;
  hipMalloc(&out, (size_t)blocks * 256 * sizeof(Fe));
  double prods = (double)blocks * 256 * n;
#define RUN(F, V, CH)                                                                             \
  {                                                                                               \
    float ms = timeit([&] { hipLaunchKernelGGL((k<F, V, CH>), dim3(blocks), dim3(256), 0, 0, in, out, n); }); \
    printf("%-7s variant %d chains %d: %.3f ms, %.2f G products/s\n", #F, V, CH, ms, prods * CH / ms / 1e6); \
  }
  RUN(Pallas, 0, 1) RUN(Pallas, 0, 2) RUN(Pallas, 1, 1) RUN(Pallas, 1, 2)
  RUN(Bn254, 0, 1) RUN(Bn254, 0, 2) RUN(Bn254, 1, 1) RUN(Bn254, 1, 2)
  {
    float ms = timeit([&] { hipLaunchKernelGGL(madk, dim3(blocks), dim3(256), 0, 0, (uint64_t*)out, 1024); });
    printf("v_mad_u64_u32: %.3f ms, %.1f G mads/s (%.2f per CU per cycle at 2.4 GHz)\n", ms,
           (double)blocks * 256 * 1024 * 8 / ms / 1e6, (double)blocks * 256 * 1024 * 8 / ms / 1e6 / 256 / 2.4);
  }
  return 0;
}

// Field-multiply throughput probe (diagnostics): chains of Montgomery products per lane, many
// waves, timed with HIP events. Variant 0: field::mul (the product the kernels use), 1:
// field::mul_cios (the form it replaced); plus a bit-for-bit check of one against the other.
//   hipcc -O3 --offload-arch=gfx950 -o tools/mulbench tools/mulbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include "../zk-odst_amd/csrc/b2f_field.h"
using namespace b2f::field;

// product scanning with two word products per asm block (one compiler wait state per block
// instead of one per product): a probe of the wait states' cost
__device__ __forceinline__ void madd_vv_vs(uint64_t& acc, uint32_t& ov, uint32_t x0, uint32_t y0, uint32_t x1,
                                           uint32_t y1) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %4, %5, %0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(ov)
      : "v"(x0), "v"(y0), "v"(x1), "s"(y1)
      : "vcc");
}
template <class F>
__device__ __forceinline__ Fe mul2(const Fe& a, const Fe& b) {
  uint32_t m[8], r[8];
  uint64_t acc = 0;
  uint32_t ov = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
#pragma unroll
    for (int i = 0; i < k; i++) {
      if (F::P[k - i]) madd_vv_vs(acc, ov, a.w[i], b.w[k - i], m[i], F::P[k - i]);
      else acc_madd(acc, ov, a.w[i], b.w[k - i]);
    }
    acc_madd(acc, ov, a.w[k], b.w[0]);
    m[k] = (uint32_t)acc * F::NP;
    acc_maddc(acc, ov, m[k], F::P[0]);
    acc = (acc >> 32) | ((uint64_t)ov << 32);
    ov = 0;
  }
#pragma unroll
  for (int k = 8; k < 15; k++) {
#pragma unroll
    for (int i = k - 7; i < 8; i++) {
      if (F::P[k - i]) madd_vv_vs(acc, ov, a.w[i], b.w[k - i], m[i], F::P[k - i]);
      else acc_madd(acc, ov, a.w[i], b.w[k - i]);
    }
    r[k - 8] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)ov << 32);
    ov = 0;
  }
  r[7] = (uint32_t)acc;
  Fe o;
#pragma unroll
  for (int j = 0; j < 8; j++) o.w[j] = r[j];
  return reduce_once<F>(o);
}

// Two independent products interleaved inside each asm block (ILP in one wave): product A carries
// through vcc, product B through an SGPR pair the compiler picks
__device__ __forceinline__ void x2_madd2(uint64_t& aa, uint32_t& oa, uint64_t& ab, uint32_t& ob, uint32_t xa0,
                                         uint32_t ya0, uint32_t xa1, uint32_t xb0, uint32_t yb0, uint32_t xb1,
                                         uint32_t y1) {
  uint64_t cb;
  asm("v_mad_u64_u32 %0, vcc, %5, %6, %0\n\t"
      "v_mad_u64_u32 %1, %4, %8, %9, %1\n\t"
      "v_addc_co_u32_e32 %2, vcc, 0, %2, vcc\n\t"
      "v_addc_co_u32_e64 %3, %4, 0, %3, %4\n\t"
      "v_mad_u64_u32 %0, vcc, %7, %11, %0\n\t"
      "v_mad_u64_u32 %1, %4, %10, %11, %1\n\t"
      "v_addc_co_u32_e32 %2, vcc, 0, %2, vcc\n\t"
      "v_addc_co_u32_e64 %3, %4, 0, %3, %4"
      : "+v"(aa), "+v"(ab), "+v"(oa), "+v"(ob), "=&s"(cb)
      : "v"(xa0), "v"(ya0), "v"(xa1), "v"(xb0), "v"(yb0), "v"(xb1), "s"(y1)
      : "vcc");
}
__device__ __forceinline__ void x2_madd1(uint64_t& aa, uint32_t& oa, uint64_t& ab, uint32_t& ob, uint32_t xa,
                                         uint32_t ya, uint32_t xb, uint32_t yb) {
  uint64_t cb;
  asm("v_mad_u64_u32 %0, vcc, %5, %6, %0\n\t"
      "v_mad_u64_u32 %1, %4, %7, %8, %1\n\t"
      "v_addc_co_u32_e32 %2, vcc, 0, %2, vcc\n\t"
      "v_addc_co_u32_e64 %3, %4, 0, %3, %4"
      : "+v"(aa), "+v"(ab), "+v"(oa), "+v"(ob), "=&s"(cb)
      : "v"(xa), "v"(ya), "v"(xb), "v"(yb)
      : "vcc");
}
__device__ __forceinline__ void x2_maddc(uint64_t& aa, uint32_t& oa, uint64_t& ab, uint32_t& ob, uint32_t xa,
                                         uint32_t xb, uint32_t y) {  // y uniform
  uint64_t cb;
  asm("v_mad_u64_u32 %0, vcc, %5, %7, %0\n\t"
      "v_mad_u64_u32 %1, %4, %6, %7, %1\n\t"
      "v_addc_co_u32_e32 %2, vcc, 0, %2, vcc\n\t"
      "v_addc_co_u32_e64 %3, %4, 0, %3, %4"
      : "+v"(aa), "+v"(ab), "+v"(oa), "+v"(ob), "=&s"(cb)
      : "v"(xa), "v"(xb), "s"(y)
      : "vcc");
}
template <class F>
__device__ __forceinline__ void mul_x2(const Fe& a, const Fe& b, const Fe& c, const Fe& d, Fe& oa, Fe& oc) {
  uint32_t ma[8], mc[8], ra[8], rc[8];
  uint64_t A = 0, C = 0;
  uint32_t va = 0, vc = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
#pragma unroll
    for (int i = 0; i < k; i++) {
      if (F::P[k - i]) x2_madd2(A, va, C, vc, a.w[i], b.w[k - i], ma[i], c.w[i], d.w[k - i], mc[i], F::P[k - i]);
      else x2_madd1(A, va, C, vc, a.w[i], b.w[k - i], c.w[i], d.w[k - i]);
    }
    x2_madd1(A, va, C, vc, a.w[k], b.w[0], c.w[k], d.w[0]);
    ma[k] = (uint32_t)A * F::NP;
    mc[k] = (uint32_t)C * F::NP;
    x2_maddc(A, va, C, vc, ma[k], mc[k], F::P[0]);
    A = (A >> 32) | ((uint64_t)va << 32);
    C = (C >> 32) | ((uint64_t)vc << 32);
    va = vc = 0;
  }
#pragma unroll
  for (int k = 8; k < 15; k++) {
#pragma unroll
    for (int i = k - 7; i < 8; i++) {
      if (F::P[k - i]) x2_madd2(A, va, C, vc, a.w[i], b.w[k - i], ma[i], c.w[i], d.w[k - i], mc[i], F::P[k - i]);
      else x2_madd1(A, va, C, vc, a.w[i], b.w[k - i], c.w[i], d.w[k - i]);
    }
    ra[k - 8] = (uint32_t)A;
    rc[k - 8] = (uint32_t)C;
    A = (A >> 32) | ((uint64_t)va << 32);
    C = (C >> 32) | ((uint64_t)vc << 32);
    va = vc = 0;
  }
  ra[7] = (uint32_t)A;
  rc[7] = (uint32_t)C;
  Fe x, y;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    x.w[j] = ra[j];
    y.w[j] = rc[j];
  }
  oa = reduce_once<F>(x);
  oc = reduce_once<F>(y);
}

// mul (b2f_field.h, product scanning) vs mul_cios (the operand-scanning form it replaced) on
// pseudo-random operands below p (top word reduced mod p's top word) and on 0, 1, p - 1: count of
// differing products
template <class F>
__global__ void check(uint32_t* bad, int n) {
  uint32_t s = blockIdx.x * 256 + threadIdx.x + 1;
  auto rnd = [&]() { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; };
  for (int it = 0; it < n; it++) {
    Fe a, b;
    for (int i = 0; i < 8; i++) { a.w[i] = rnd(); b.w[i] = rnd(); }
    a.w[7] %= F::P[7];  // < p
    b.w[7] %= F::P[7];
    if (it == 0) {  // edge operands: p - 1 and 0 / 1
      for (int i = 0; i < 8; i++) a.w[i] = F::P[i];
      a.w[0] -= 1;
      for (int i = 0; i < 8; i++) b.w[i] = 0;
      b.w[0] = threadIdx.x & 1u;
      if (threadIdx.x & 2u) b = a;
    }
    const Fe x = mul_comba<F>(a, b), y = mul_cios<F>(a, b), z = mul2<F>(a, b), q = mul_asm<F>(a, b);
    Fe u, v;
    mul_x2<F>(a, b, b, a, u, v);
    uint32_t d = 0;
    for (int i = 0; i < 8; i++) d |= (x.w[i] ^ y.w[i]) | (z.w[i] ^ y.w[i]) | (u.w[i] ^ y.w[i]) | (v.w[i] ^ y.w[i]) | (q.w[i] ^ y.w[i]);
    if (d) atomicAdd(bad, 1u);
  }
}

template <class F, int V, int CH>
__global__ __launch_bounds__(256) void k(const Fe* in, Fe* out, int n) {
  Fe acc[CH];
#pragma unroll
  for (int c = 0; c < CH; c++) acc[c] = in[(threadIdx.x + c) & 255];
  const Fe b = in[256 + (blockIdx.x & 15)];
  for (int i = 0; i < n; i++) {
    if (V == 3) {
#pragma unroll
      for (int c = 0; c + 1 < CH; c += 2) mul_x2<F>(acc[c], b, acc[c + 1], b, acc[c], acc[c + 1]);
    } else {
#pragma unroll
      for (int c = 0; c < CH; c++)
        acc[c] = V == 0 ? mul_comba<F>(acc[c], b) : V == 1 ? mul_cios<F>(acc[c], b) : V == 4 ? mul_asm<F>(acc[c], b) : mul2<F>(acc[c], b);
    }
  }
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
  RUN(Pallas, 0, 1) RUN(Pallas, 0, 2) RUN(Pallas, 1, 1) RUN(Pallas, 1, 2) RUN(Pallas, 2, 1) RUN(Pallas, 2, 2)
  RUN(Bn254, 0, 1) RUN(Bn254, 0, 2) RUN(Bn254, 1, 1) RUN(Bn254, 1, 2) RUN(Bn254, 2, 1) RUN(Bn254, 2, 2)
  // the same kernels with their workgroups per CU capped by dynamic LDS (48 KiB: 3 per CU = 3 waves
  // per SIMD, as pm_chunk_kernel runs; 64 KiB: 2): does a second independent chain per lane (ILP)
  // recover what fewer waves lose?
#define RUNL(F, V, CH, KB)                                                                        \
  {                                                                                               \
    float ms = timeit([&] { hipLaunchKernelGGL((k<F, V, CH>), dim3(blocks), dim3(256), KB * 1024, 0, in, out, n); }); \
    printf("%-7s variant %d chains %d lds %2d KiB: %.3f ms, %.2f G products/s\n", #F, V, CH, KB, ms, prods * CH / ms / 1e6); \
  }
  RUNL(Pallas, 0, 1, 48) RUNL(Pallas, 0, 2, 48) RUNL(Pallas, 0, 1, 64) RUNL(Pallas, 0, 2, 64)
  RUNL(Bn254, 0, 1, 48) RUNL(Bn254, 0, 2, 48) RUNL(Bn254, 0, 1, 64) RUNL(Bn254, 0, 2, 64)
  // variant 3: the two chains of a lane through mul_x2 (interleaved in each asm block)
  RUN(Pallas, 3, 2) RUN(Bn254, 3, 2)
  // variant 4: mul_asm (b2f_mont_asm.h, one asm block per product)
  RUN(Pallas, 4, 1) RUN(Pallas, 4, 2) RUN(Bn254, 4, 1) RUN(Bn254, 4, 2)
  RUNL(Pallas, 4, 1, 48) RUNL(Pallas, 4, 1, 64) RUNL(Bn254, 4, 1, 48)
  RUN(Pallas, 0, 1) RUN(Bn254, 0, 1)
  RUNL(Pallas, 3, 2, 48) RUNL(Pallas, 3, 2, 64) RUNL(Bn254, 3, 2, 48) RUNL(Bn254, 3, 2, 64)
  {
    uint32_t* bad;
    hipMalloc(&bad, 8);
    hipMemset(bad, 0, 8);
    hipLaunchKernelGGL(check<Pallas>, dim3(1024), dim3(256), 0, 0, bad, 16);
    hipLaunchKernelGGL(check<Bn254>, dim3(1024), dim3(256), 0, 0, bad + 1, 16);
    uint32_t h[2];
    hipMemcpy(h, bad, 8, hipMemcpyDeviceToHost);
    printf("mul / mul2 / mul_x2 / mul_asm (product scanning) vs mul_cios mismatches over 4.2M products: pallas %u bn254 %u\n", h[0], h[1]);
  }
  {
    float ms = timeit([&] { hipLaunchKernelGGL(madk, dim3(blocks), dim3(256), 0, 0, (uint64_t*)out, 1024); });
    printf("v_mad_u64_u32: %.3f ms, %.1f G mads/s (%.2f per CU per cycle at 2.4 GHz)\n", ms,
           (double)blocks * 256 * 1024 * 8 / ms / 1e6, (double)blocks * 256 * 1024 * 8 / ms / 1e6 / 256 / 2.4);
  }
  return 0;
}

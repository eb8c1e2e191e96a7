// Load-pattern probe (diagnostics, round 6): how fast the chip reads 11 u32 columns of R rows
// when each wave reads C consecutive rows of every column per step (16 B per lane, C / 4 lanes
// per column, the eval fast pass's shape at C = 208) and the waves' chunks are
//   rr:   dealt round-robin (wave w takes chunks w, w + W, ...: the chip's waves sit on one
//         contiguous front of every column), or
//   band: walked in bands of B consecutive chunks (band b -> wave b mod W, as the eval fast
//         pass walks its 24-tile bands: W separate fronts per column).
// Each wave keeps one chunk in flight ahead of the one it sums, as the eval fast pass does.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/load_probe tools/load_probe.hip
// Run:   tools/load_probe [rows_log2 = 28]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                  \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int NCOL = 11;

struct Chunk {
  uint4 v[NCOL];
};

__device__ __forceinline__ Chunk load_chunk(const uint32_t* __restrict__ a, uint64_t rows, uint64_t r0,
                                            uint32_t q) {
  Chunk c;
#pragma unroll
  for (int k = 0; k < NCOL; k++) c.v[k] = *reinterpret_cast<const uint4*>(a + k * rows + r0 + 4 * q);
  return c;
}

// C rows per chunk, Q = C / 4 lanes per column (Q <= 64: lanes >= Q repeat lane 0's address)
template <int C, bool BAND>
__global__ void __launch_bounds__(256) probe(const uint32_t* __restrict__ a, uint64_t rows, uint32_t band,
                                            uint32_t* __restrict__ out) {
  constexpr uint32_t Q = C / 4;
  static_assert(Q <= 64, "one 16-byte load per lane and column");
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t W = (uint64_t)gridDim.x * 4;
  const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t q = lane < Q ? lane : 0u;
  const uint64_t n = rows / C;  // chunks
  // chunk sequence of this wave: rr: w, w + W, ...; band: band b = w, w + W, ..., chunks b*B .. b*B+B-1
  auto chunk_at = [&](uint64_t i) -> uint64_t {
    if (!BAND) return w + i * W;
    const uint64_t b = w + (i / band) * W;
    return b * band + i % band;
  };
  uint32_t acc = 0;
  uint64_t i = 0, t = chunk_at(0);
  Chunk cur = load_chunk(a, rows, (t < n ? t : 0) * C, q);
  while (t < n) {
    const uint64_t tn = chunk_at(i + 1);
    const Chunk nxt = load_chunk(a, rows, (tn < n ? tn : 0) * C, q);
#pragma unroll
    for (int k = 0; k < NCOL; k++) acc ^= cur.v[k].x ^ cur.v[k].y ^ cur.v[k].z ^ cur.v[k].w;
    cur = nxt;
    t = tn;  // chunk_at is increasing in i: past the end once, past it for good
    i++;
  }
  if (acc == 0x12345678u) out[0] = acc;  // keeps the loads
}

// the eval kernel's floor shape: a workgroup per 1,024-row tile (wave k reads rows 256k..256k+255
// of it: 4 KB of every column per workgroup), tiles dealt to workgroups in bands of B with the
// XCD-aware deal of eval_kernel (b2f_kernels.hip)
__global__ void __launch_bounds__(256) probe_wg(const uint32_t* __restrict__ a, uint64_t rows, uint32_t band,
                                               uint32_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t G = gridDim.x;
  const uint64_t b0 = (G % 8 == 0) ? (blockIdx.x % 8) * (G / 8) + blockIdx.x / 8 : blockIdx.x;
  const uint64_t n = rows / 1024;
  auto seq = [&](uint64_t k) { return (b0 + (k / band) * G) * band + k % band; };
  uint32_t acc = 0;
  uint64_t i = 0, t = seq(0);
  Chunk cur = load_chunk(a, rows, (t < n ? t : 0) * 1024 + 256 * wv, lane);
  while (t < n) {
    const uint64_t tn = seq(i + 1);
    const Chunk nxt = load_chunk(a, rows, (tn < n ? tn : 0) * 1024 + 256 * wv, lane);
#pragma unroll
    for (int k = 0; k < NCOL; k++) acc ^= cur.v[k].x ^ cur.v[k].y ^ cur.v[k].z ^ cur.v[k].w;
    cur = nxt;
    t = tn;
    i++;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

float run_wg(const uint32_t* a, uint64_t rows, uint32_t band, uint32_t* out, int wgs_per_cu, int cus) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 4; rep++) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(probe_wg, dim3(cus * wgs_per_cu), dim3(256), 0, 0, a, rows, band, out);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;
  }
  CHK(hipEventDestroy(e0));
  CHK(hipEventDestroy(e1));
  return best;
}

template <int C, bool BAND>
float run(const uint32_t* a, uint64_t rows, uint32_t band, uint32_t* out, int wgs_per_cu, int cus) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 4; rep++) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL((probe<C, BAND>), dim3(cus * wgs_per_cu), dim3(256), 0, 0, a, rows, band, out);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;
  }
  CHK(hipEventDestroy(e0));
  CHK(hipEventDestroy(e1));
  return best;
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 28;
  const uint64_t rows = 1ull << lg;
  int dev = 0, cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  uint32_t* a = nullptr;
  uint32_t* out = nullptr;
  CHK(hipMalloc(&a, NCOL * rows * 4));
  CHK(hipMalloc(&out, 64));
  CHK(hipMemset(a, 1, NCOL * rows * 4));
  const double gb = NCOL * rows * 4 / 1e9;
  printf("%d CUs, %d columns x 2^%d rows (%.2f GB)\n", cus, NCOL, lg, gb);
  for (int wpc = 1; wpc <= 3; wpc++) {
    float t;
    t = run<208, false>(a, rows, 0, out, wpc, cus);
    printf("wg/CU %d  C=208 rr        %7.3f ms  %6.0f GB/s\n", wpc, t, gb / t * 1e3);
    t = run<208, true>(a, rows, 24, out, wpc, cus);
    printf("wg/CU %d  C=208 band 24   %7.3f ms  %6.0f GB/s\n", wpc, t, gb / t * 1e3);
    t = run<256, false>(a, rows, 0, out, wpc, cus);
    printf("wg/CU %d  C=256 rr        %7.3f ms  %6.0f GB/s\n", wpc, t, gb / t * 1e3);
    t = run<256, true>(a, rows, 24, out, wpc, cus);
    printf("wg/CU %d  C=256 band 24   %7.3f ms  %6.0f GB/s\n", wpc, t, gb / t * 1e3);
    t = run<256, true>(a, rows, 4, out, wpc, cus);
    printf("wg/CU %d  C=256 band 4    %7.3f ms  %6.0f GB/s\n", wpc, t, gb / t * 1e3);
    t = run_wg(a, rows, 4, out, wpc, cus);
    printf("wg/CU %d  wg tile band 4 %7.3f ms  %6.0f GB/s\n", wpc, t, gb / t * 1e3);
    t = run_wg(a, rows, 1, out, wpc, cus);
    printf("wg/CU %d  wg tile rr     %7.3f ms  %6.0f GB/s\n", wpc, t, gb / t * 1e3);
  }
  CHK(hipFree(a));
  CHK(hipFree(out));
  return 0;
}

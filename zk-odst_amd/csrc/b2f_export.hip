// b2f_export.hip -- Fp export of the trace: u32 advice cells ->
// pallas::Base field elements as halo2's prover holds them, column by column in halo2's
// advice-column order (table16.rs:281-294).
//
// Field: pasta_curves 0.5.1 Fp (Cargo.lock:1334-1337), p = 2^254 + d with
//   d = 0x224698fc094cf91b992d30ed00000001 (126 bits).
// In-memory form of Fp is Montgomery with R = 2^256: mont(x) = x * 2^256 mod p.
// For a cell value x < 2^32 this needs no multiprecision reduction: 2^256 = 4 * 2^254 and
// 2^254 = -d (mod p), so x * 2^256 = -4 x d (mod p), and since 4 x d < 2^160 < p,
//   mont(x) = p - 4 x d = 2^254 - (4x - 1) d        (x != 0),   mont(0) = 0.
// That is one 34 x 126-bit product and a 256-bit negation per cell (the oracle computes the
// same values with a generic Montgomery multiply by R^2, oracle/b2f_oracle.c).
// Canonical form (PrimeField::to_repr, 32-byte little endian) is simply (x, 0, 0, 0), in
// either field.
// BN254 Fr (halo2curves 0.3.2 bn256::Fr, r < 2^254, no such short form of r): mont(x) =
// x * (2^256 mod r) mod r with a 32-bit quotient from a fixed-point reciprocal
// (field::from_u32: 16 word products; the generic Montgomery product by R^2 it replaced took
// 72 and made this kernel VALU-bound, 4.9 ms at 2^25 rows). Each lane forms one cell and swaps
// a half with its store partner (export_fp_kernel<3>), so every cell is formed once.
//
// HBM-bound: 4 B read, 32 B written per cell. A wave writes 64 x 16 B = 1 KiB contiguous per
// store instruction (lane l stores 16-byte chunk l of a 1 KiB span, i.e. half l & 1 of cell
// l >> 1 of the span's 32 cells), non-temporal.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/b2f.h"
#include "b2f_field.h"

namespace b2f {

hipError_t launch_export_fp(const uint32_t* d_advice, uint64_t total_rows, uint64_t row_begin,
                            uint64_t nrows, uint32_t form, uint64_t* d_out, uint64_t out_rows,
                            int cu_count, unsigned* tctr, hipStream_t s);
hipError_t launch_spread_table(uint64_t usable_rows, uint32_t form, uint64_t* d_out,
                               uint64_t out_rows, hipStream_t s);

namespace {

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

constexpr uint64_t kD0 = 0x992d30ed00000001ull;  // d, low limb
constexpr uint64_t kD1 = 0x224698fc094cf91bull;  // d, high limb
constexpr int EXPORT_BLOCK = 256;
constexpr int CELLS_PER_ITER = EXPORT_BLOCK / 2;  // 128 cells = 4 KiB of output per WG pass

__device__ __forceinline__ u64x2 bn254_half(uint32_t x, uint32_t half) {
  const field::Fe m = field::from_u32<field::Bn254>(x);
  uint32_t o[4];
#pragma unroll
  for (int i = 0; i < 4; i++) o[i] = half ? m.w[4 + i] : m.w[i];  // no dynamic index (scratch)
  return u64x2{(uint64_t)o[0] | ((uint64_t)o[1] << 32), (uint64_t)o[2] | ((uint64_t)o[3] << 32)};
}

// limbs (2*half, 2*half+1) of the field element for cell value x: canonical (either field),
// pasta Montgomery (the closed form above) or BN254 Montgomery (FORM 3)
template <int FORM>
__device__ __forceinline__ u64x2 fp_half(uint32_t x, uint32_t half) {
  if (FORM == 3) return bn254_half(x, half);
  u64x2 r;
  if (!(FORM & 1)) {  // canonical, either field
    r.x = half ? 0 : x;
    r.y = 0;
    return r;
  }
  if (x == 0) {
    r.x = 0;
    r.y = 0;
    return r;
  }
  // z = (4x - 1) * d  < 2^160: limbs z0, z1, z2
  uint64_t y = 4ull * x - 1;
  uint64_t z0 = y * kD0;
  uint64_t h0 = __umul64hi(y, kD0);
  uint64_t l1 = y * kD1;
  uint64_t z2 = __umul64hi(y, kD1);
  uint64_t z1 = h0 + l1;
  z2 += (z1 < h0);
  // v = 2^254 - z  (two's complement of z plus 2^254; z != 0 so the low borrow chain is
  // that of a negation: v0 = -z0, then borrow 1 out of limb 0 iff z0 != 0)
  uint64_t b0 = (z0 != 0);
  uint64_t v0 = 0 - z0;
  uint64_t v1 = 0 - z1 - b0;
  uint64_t b1 = (z1 != 0) | b0;  // borrow out of limb 1
  uint64_t v2 = 0 - z2 - b1;
  uint64_t b2 = (z2 != 0) | b1;
  uint64_t v3 = (1ull << 62) - b2;
  r.x = half ? v2 : v0;
  r.y = half ? v3 : v1;
  return r;
}

// Persistent workgroups over XT-row tiles dealt round-robin (the fill kernel's pattern: the
// whole chip writes one narrow band of each output column at a time). Per tile a workgroup
// reads the ten 2 KiB column slices (all loads issued first) and writes the ten 16 KiB output
// slices; every store instruction of a wave covers 1 KiB contiguous.
constexpr int XT = 512;
constexpr int XSUB = XT / CELLS_PER_ITER;  // 4 store passes per column per tile
constexpr int kAofH[10] = {5, 3, 4, 6, 7, 8, 9, 0, 1, 2};

#ifndef B2F_EXPORT_DYN
#define B2F_EXPORT_DYN 1  // 0 (variant): tiles dealt round-robin to the workgroups (round 5)
#endif
template <int FORM>
__global__ __launch_bounds__(EXPORT_BLOCK) void export_fp_kernel(
    const uint32_t* __restrict__ advice, uint64_t total_rows, uint64_t row_begin,
    uint64_t nrows, uint64_t* __restrict__ out, uint64_t out_rows, unsigned* __restrict__ tctr) {
  const uint32_t t = threadIdx.x;
  const uint32_t half = t & 1;
  const uint64_t n_tiles = (nrows + XT - 1) / XT;
#if B2F_EXPORT_DYN
  // tiles claimed from the launch's counter (a barrier per tile shares the claim), so the
  // workgroups finish within a tile of each other: 2.20 -> 1.87 ms pasta, 2.12 -> 1.81 BN254 at
  // 2^25 rows (profiles/r06k_placement_export_dyn.jsonl; 65,536 claims of 184 KB each)
  __shared__ uint32_t s_tile[2];
  uint32_t slot = 0;
  auto claim = [&]() -> uint64_t {
    if (t == 0) s_tile[slot] = atomicAdd(tctr, 1u);
    __syncthreads();
    const uint64_t v = __builtin_amdgcn_readfirstlane(s_tile[slot]);
    slot ^= 1u;
    return v;
  };
  for (uint64_t tile = claim(); tile < n_tiles; tile = claim()) {
#else
  (void)tctr;
  for (uint64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
#endif
    const uint64_t r0 = tile * XT;
    uint32_t x[10][XSUB];
#pragma unroll
    for (int h = 0; h < 10; h++)
#pragma unroll
      for (int i = 0; i < XSUB; i++) {
        uint64_t cell = r0 + i * CELLS_PER_ITER + (t >> 1);
        x[h][i] = cell < nrows ? advice[(uint64_t)kAofH[h] * total_rows + row_begin + cell] : 0u;
      }
#pragma unroll
    for (int h = 0; h < 10; h++) {
      u64x2* dst = reinterpret_cast<u64x2*>(out + (uint64_t)h * out_rows * 4);
      if (FORM == 3) {
        // BN254's per-cell product is the cost, and both lanes of a store pair need the same
        // cell: each lane forms one whole cell of two consecutive passes instead (even lane:
        // pass i's, odd lane: pass i + 1's), and the pair swaps the half the other one stores
#pragma unroll
        for (int i = 0; i < XSUB; i += 2) {
          // a bitwise select: `half ? x[h][i + 1] : x[h][i]` became a dynamic index (x in scratch)
          const uint32_t xa = x[h][i], xb = x[h][i + 1];
          const field::Fe m = field::from_u32<field::Bn254>(xa ^ ((xa ^ xb) & (0u - half)));
          uint32_t own[4], give[4];
#pragma unroll
          for (int w = 0; w < 4; w++) {
            own[w] = half ? m.w[4 + w] : m.w[w];   // the half this lane stores of its own cell
            give[w] = half ? m.w[w] : m.w[4 + w];  // the half its partner stores
          }
          uint32_t got[4];
#pragma unroll
          for (int w = 0; w < 4; w++)  // lane ^ 1: DPP quad_perm [1, 0, 3, 2]
            got[w] = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)give[w], 0xB1, 0xf, 0xf, false);
          const u64x2 mine = u64x2{(uint64_t)own[0] | ((uint64_t)own[1] << 32), (uint64_t)own[2] | ((uint64_t)own[3] << 32)};
          const u64x2 other = u64x2{(uint64_t)got[0] | ((uint64_t)got[1] << 32), (uint64_t)got[2] | ((uint64_t)got[3] << 32)};
          const uint64_t c0 = r0 + i * CELLS_PER_ITER + (t >> 1), c1 = c0 + CELLS_PER_ITER;
          if (c0 < nrows) __builtin_nontemporal_store(half ? other : mine, dst + 2 * c0 + half);
          if (c1 < nrows) __builtin_nontemporal_store(half ? mine : other, dst + 2 * c1 + half);
        }
        continue;
      }
#pragma unroll
      for (int i = 0; i < XSUB; i++) {
        uint64_t cell = r0 + i * CELLS_PER_ITER + (t >> 1);
        if (cell < nrows) __builtin_nontemporal_store(fp_half<FORM>(x[h][i], half), dst + 2 * cell + half);
      }
    }
  }
}

// The spread table as the prover's three table (fixed) columns tag, dense, spread
// (SpreadTableChip::load, spread_table.rs:470-508: row x < 2^16 holds (tag(x), x, spread(x)),
// spread_table.rs:574-600), then the layouter's fill_from_row default -- row 0's values,
// all zero -- up to the usable rows. Two lanes per element, as the export kernel.
__device__ __forceinline__ uint32_t sp16(uint32_t x) {
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x = (x | (x << 2)) & 0x33333333u;
  x = (x | (x << 1)) & 0x55555555u;
  return x;
}
__global__ __launch_bounds__(256) void spread_table_kernel(uint64_t usable_rows, uint32_t form,
                                                           uint64_t* __restrict__ out,
                                                           uint64_t out_rows) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;  // 2 lanes per row
  const uint64_t row = i >> 1;
  const uint32_t half = (uint32_t)(i & 1);
  if (row >= usable_rows) return;
  const uint32_t x = row < 65536u ? (uint32_t)row : 0u;
  const uint32_t v[3] = {x < 256u ? 0u : (x < 32768u ? 1u : 2u), x, sp16(x)};
#pragma unroll
  for (int c = 0; c < 3; c++) {
    u64x2* dst = reinterpret_cast<u64x2*>(out + (uint64_t)c * out_rows * 4);
    u64x2 e;
    if (form == B2F_FP_BN254_MONTGOMERY) {
      e = bn254_half(v[c], half);
    } else {
      e = form & 1u ? fp_half<1>(v[c], half) : fp_half<0>(v[c], half);
    }
    __builtin_nontemporal_store(e, dst + 2 * row + half);
  }
}

}  // namespace

hipError_t launch_spread_table(uint64_t usable_rows, uint32_t form, uint64_t* d_out,
                               uint64_t out_rows, hipStream_t s) {
  const uint64_t lanes = 2 * usable_rows;
  hipLaunchKernelGGL(spread_table_kernel, dim3((uint32_t)((lanes + 255) / 256)), dim3(256), 0, s,
                     usable_rows, form, d_out, out_rows);
  return hipGetLastError();
}

hipError_t launch_export_fp(const uint32_t* d_advice, uint64_t total_rows, uint64_t row_begin,
                            uint64_t nrows, uint32_t form, uint64_t* d_out, uint64_t out_rows,
                            int cu_count, unsigned* tctr, hipStream_t s) {
  // persistent grid, workgroups per CU by form (below; halo2 column h -> a_i by kAofH)
  uint64_t tiles = (nrows + XT - 1) / XT;
  // persistent workgroups per CU, per form (same-process A/B, profiles/r05g*_export_ab_*.txt:
  // pasta 3 vs 4 / 2 / 5: 2.47 vs 2.49 / 2.85 / 2.79 ms; BN254 2 vs 4 / 3 / 5: 2.38 vs 2.54 /
  // 2.50 / 2.53 at 2^25 rows): fewer concurrent tile streams write faster until the cells'
  // compute is no longer hidden (pasta's is a few instructions, BN254's a 32-bit quotient)
  int per_cu = form == B2F_FP_BN254_MONTGOMERY ? 2 : 3;
#ifdef B2F_DIAG  // diagnostics: B2F_EXPORT_PERCU overrides the workgroups per CU
  if (const char* v = getenv("B2F_EXPORT_PERCU")) {
    const int k = atoi(v);
    if (k >= 1 && k <= 8) per_cu = k;
  }
#endif
  uint64_t want = (uint64_t)cu_count * per_cu;
  uint32_t gx = (uint32_t)(tiles < want ? tiles : want);
  if (gx == 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(tctr, 0, sizeof(unsigned), s);
  if (e != hipSuccess) return e;
  if (form == B2F_FP_BN254_MONTGOMERY) {
    hipLaunchKernelGGL(export_fp_kernel<3>, dim3(gx), dim3(EXPORT_BLOCK), 0, s, d_advice,
                       total_rows, row_begin, nrows, d_out, out_rows, tctr);
  } else if (form & 1u) {
    hipLaunchKernelGGL(export_fp_kernel<1>, dim3(gx), dim3(EXPORT_BLOCK), 0, s, d_advice,
                       total_rows, row_begin, nrows, d_out, out_rows, tctr);
  } else {
    hipLaunchKernelGGL(export_fp_kernel<0>, dim3(gx), dim3(EXPORT_BLOCK), 0, s, d_advice,
                       total_rows, row_begin, nrows, d_out, out_rows, tctr);
  }
  return hipGetLastError();
}

}  // namespace b2f

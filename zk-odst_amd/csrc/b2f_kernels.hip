// b2f_kernels.hip -- gfx950 kernels of the BLAKE2f Table16 engine and the C ABI of
// include/b2f.h. Trace contract: docs/LAYOUT.md. Design notes: DESIGN.md.
//
// Kernels (one stream, in order):
//   record_kernel  thread per instance: the BLAKE2f compression itself (RFC 7693 / EIP-152,
//                  blake2f-circuit/src/README.md:1-97), writing the work vector at the start
//                  of every half-round (the only cross-step state the row expansion needs)
//                  and h'. O(KB) per instance.
//   fill_kernel    thread per quad (4 consecutive rows), persistent workgroups over
//                  contiguous row ranges: recomputes the quad's G steps from the half-round
//                  state, builds the 4 rows x 11 columns in registers and writes them as
//                  16-byte column stores (coalesced 1 KiB per wave per column). HBM-write
//                  bound: 44 B per row.
//   eval_kernel    thread per quad over 1024-row LDS tiles (+16 halo rows): lookup check on
//                  every row, the gates whose selector bit is set, and the copy constraints
//                  of the quad's operand cells; wavefront reductions, one atomic per counter
//                  per workgroup. HBM-read bound: 44 B per row.
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>
#include <vector>

#include "../../include/b2f.h"
#include "b2f_layout.h"

using namespace b2f;

namespace b2f {
hipError_t launch_export_fp(const uint32_t* d_advice, uint64_t total_rows, uint64_t row_begin,
                            uint64_t nrows, uint32_t form, uint64_t* d_out, uint64_t out_rows,
                            int cu_count, hipStream_t s);  // b2f_export.hip
}

namespace {

__constant__ uint64_t c_iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL,
                                 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                                 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

// SIGMA = table16.rs:32-44
__constant__ __attribute__((aligned(16))) uint8_t c_sigma[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

__constant__ __attribute__((aligned(16))) uint8_t c_gidx[8][4] = {{0, 4, 8, 12}, {1, 5, 9, 13}, {2, 6, 10, 14},
                                     {3, 7, 11, 15}, {0, 5, 10, 15}, {1, 6, 11, 12},
                                     {2, 7, 8, 13}, {3, 4, 9, 14}};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// c_gidx / c_sigma repacked for one scalar-friendly load per G
constexpr uint32_t kGidxWord[8] = {0x0c080400u, 0x0d090501u, 0x0e0a0602u, 0x0f0b0703u,
                                   0x0f0a0500u, 0x0c0b0601u, 0x0d080702u, 0x0e090403u};
__constant__ uint32_t c_gidx_word[8] = {0x0c080400u, 0x0d090501u, 0x0e0a0602u, 0x0f0b0703u,
                                        0x0f0a0500u, 0x0c0b0601u, 0x0d080702u, 0x0e090403u};
struct SigmaPairs {
  uint16_t v[10][8];  // SIGMA[r][2g] | SIGMA[r][2g+1] << 8
};
constexpr SigmaPairs make_sigma_pairs() {
  const uint8_t S[10][16] = {
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
      {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
      {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
      {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
      {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
      {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
      {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
      {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
      {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
      {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};
  SigmaPairs P{};
  for (int r = 0; r < 10; r++)
    for (int g = 0; g < 8; g++) P.v[r][g] = (uint16_t)(S[r][2 * g] | (S[r][2 * g + 1] << 8));
  return P;
}
__constant__ SigmaPairs c_sigma_pairs = make_sigma_pairs();
#define c_sigma_pair c_sigma_pairs.v

constexpr int BLOCK = 256;            // threads per workgroup = quads per tile
constexpr int TILE_ROWS = 4 * BLOCK;  // 1024
constexpr int HALO_ROWS = 16;         // blocks are at most 12 rows
constexpr int TSTRIDE = TILE_ROWS + HALO_ROWS;
constexpr int NCOL_T = 11;            // a_0..a_9 + fixed

__device__ __forceinline__ uint64_t rotr64(uint64_t x, uint32_t n) {
  return (x >> n) | (x << (64 - n));
}
__device__ __forceinline__ uint32_t limb(uint64_t w, uint32_t k) {
  return (uint32_t)(w >> (16 * k)) & 0xffffu;
}
// Interleave a zero above each of the 16 low bits (shift-and-mask form).
__device__ __forceinline__ uint32_t spread16(uint32_t x) {
  x = (x | (x << 8)) & 0x00ff00ffu;
  x = (x | (x << 4)) & 0x0f0f0f0fu;
  x = (x | (x << 2)) & 0x33333333u;
  x = (x | (x << 1)) & 0x55555555u;
  return x;
}
__device__ __forceinline__ uint32_t tag16(uint32_t x) {
  return x < 256u ? 0u : (x < 32768u ? 1u : 2u);
}

// Row offsets -> instance. Largest i in [0, n) with off[i] <= row.
__device__ __forceinline__ uint32_t find_instance(const uint64_t* off, uint32_t n, uint64_t row) {
  uint32_t lo = 0, hi = n;  // off[lo] <= row < off[hi] (when row < off[n])
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (off[mid] <= row) lo = mid; else hi = mid;
  }
  return lo;
}

// index of the first work-vector state of instance i in the record (2*rounds+1 per instance)
__device__ __forceinline__ uint64_t state_index(uint64_t off_i, uint64_t i) {
  return 2 * ((off_i - (uint64_t)FIXED_ROWS * i) / ROUND_ROWS) + i;
}

// ------------------------------------------------------------------------- record kernel

__global__ void __launch_bounds__(BLOCK) record_kernel(const b2f_input* __restrict__ in,
                                                      uint32_t n,
                                                      const uint64_t* __restrict__ off,
                                                      uint64_t total_rows,
                                                      uint64_t states_cap,
                                                      uint64_t* __restrict__ rec,
                                                      uint64_t* __restrict__ h_out,
                                                      int* __restrict__ status) {
  uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  const b2f_input* x = in + i;
  uint32_t rounds = x->rounds;
  uint64_t o0 = off[i], o1 = off[i + 1];
  if (rounds > B2F_MAX_ROUNDS) { atomicOr(status, 1 << B2F_ERR_ROUNDS); return; }
  uint64_t R = (uint64_t)FIXED_ROWS + (uint64_t)ROUND_ROWS * rounds;
  bool bad = (o1 - o0 != R) || o1 > total_rows || (i == 0 && o0 != 0) ||
             (o0 < (uint64_t)FIXED_ROWS * i) || ((o0 - (uint64_t)FIXED_ROWS * i) % ROUND_ROWS);
  uint64_t st = bad ? 0 : state_index(o0, i);
  if (!bad && st + 2ull * rounds + 1 > states_cap) bad = true;
  if (bad) { atomicOr(status, 1 << B2F_ERR_LAYOUT); return; }

  uint64_t v[16], h[8];
#pragma unroll
  for (int k = 0; k < 8; k++) { h[k] = x->h[k]; v[k] = h[k]; v[k + 8] = c_iv[k]; }
  v[12] ^= x->t[0];
  v[13] ^= x->t[1];
  if (x->f) v[14] = ~v[14];

  uint64_t* s = rec + st * 16;
  auto dump = [&](void) {
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
      ulonglong2 p; p.x = v[k]; p.y = v[k + 1];
      *reinterpret_cast<ulonglong2*>(s + k) = p;
    }
    s += 16;
  };
  dump();
#define B2F_G(a, b, c, d, xx, yy)                                     \
  do {                                                               \
    v[a] = v[a] + v[b] + (xx); v[d] = rotr64(v[d] ^ v[a], 32);       \
    v[c] = v[c] + v[d];        v[b] = rotr64(v[b] ^ v[c], 24);       \
    v[a] = v[a] + v[b] + (yy); v[d] = rotr64(v[d] ^ v[a], 16);       \
    v[c] = v[c] + v[d];        v[b] = rotr64(v[b] ^ v[c], 63);       \
  } while (0)
  for (uint32_t r = 0; r < rounds; r++) {
    const uint8_t* sg = c_sigma[r % 10];
    // SIGMA indexes m at run time: gather from the (cached) input record, not registers.
    uint64_t mm[16];
#pragma unroll
    for (int k = 0; k < 16; k++) mm[k] = x->m[sg[k]];
    B2F_G(0, 4, 8, 12, mm[0], mm[1]);
    B2F_G(1, 5, 9, 13, mm[2], mm[3]);
    B2F_G(2, 6, 10, 14, mm[4], mm[5]);
    B2F_G(3, 7, 11, 15, mm[6], mm[7]);
    dump();
    B2F_G(0, 5, 10, 15, mm[8], mm[9]);
    B2F_G(1, 6, 11, 12, mm[10], mm[11]);
    B2F_G(2, 7, 8, 13, mm[12], mm[13]);
    B2F_G(3, 4, 9, 14, mm[14], mm[15]);
    dump();
  }
#undef B2F_G
  if (h_out) {
#pragma unroll
    for (int k = 0; k < 8; k++) h_out[8 * (uint64_t)i + k] = h[k] ^ v[k] ^ v[k + 8];
  }
}

// --------------------------------------------------------------------------- fill kernel

struct Quad {
  uint32_t c[10][4];
  uint32_t fx[4];
};

__device__ __forceinline__ void zero(Quad& Q) {
#pragma unroll
  for (int c = 0; c < 10; c++)
#pragma unroll
    for (int j = 0; j < 4; j++) Q.c[c][j] = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) Q.fx[j] = 0;
}

__device__ __forceinline__ void lrow(Quad& Q, int j, uint32_t x) {
  Q.c[A0][j] = tag16(x);
  Q.c[A1][j] = x;
  Q.c[A2][j] = spread16(x);
}

// XOR block (rho is wiring only): rows 2k = L(z_k) + operand spreads, 2k+1 = L(o_k)
__device__ __forceinline__ void q_xor(Quad& Q, uint64_t X, uint64_t Y, uint32_t q, int sel) {
  uint64_t z = X ^ Y, o = X & Y;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    uint32_t k = 2 * q + h;
    lrow(Q, 2 * h, limb(z, k));
    Q.c[A3][2 * h] = spread16(limb(X, k));
    Q.c[A4][2 * h] = spread16(limb(Y, k));
    lrow(Q, 2 * h + 1, limb(o, k));
  }
  if (q == 0) Q.fx[0] = 1u << sel;
}

__device__ __forceinline__ void q_xor24(Quad& Q, uint64_t X, uint64_t Y, uint32_t q) {
  uint64_t z = X ^ Y, o = X & Y, w = rotr64(z, 24);
#pragma unroll
  for (int j = 0; j < 4; j++) {
    uint32_t R = 4 * q + j, k = R / 3, kind = R - 3 * k;
    uint32_t zk = limb(z, k);
    uint32_t val = kind == 0 ? (zk & 0xffu) : (kind == 1 ? (zk >> 8) : limb(o, k));
    lrow(Q, j, val);
    if (kind == 0) {
      uint32_t wk = limb(w, k);
      Q.c[A3][j] = spread16(limb(X, k));
      Q.c[A4][j] = spread16(limb(Y, k));
      Q.c[A7][j] = wk;
      Q.c[A8][j] = spread16(wk);
    }
  }
  if (q == 0) Q.fx[0] = (1u << S_B1) | (1u << S_EFGH);
}

__device__ __forceinline__ void q_xor63(Quad& Q, uint64_t X, uint64_t Y, uint32_t q) {
  uint64_t z = X ^ Y, o = X & Y, w = rotr64(z, 63);
#pragma unroll
  for (int h = 0; h < 2; h++) {
    uint32_t k = 2 * q + h;
    uint32_t zk = limb(z, k), wk = limb(w, k);
    lrow(Q, 2 * h, zk & 0x7fffu);
    Q.c[A3][2 * h] = spread16(limb(X, k));
    Q.c[A4][2 * h] = spread16(limb(Y, k));
    Q.c[A6][2 * h] = zk >> 15;
    Q.c[A7][2 * h] = wk;
    Q.c[A8][2 * h] = spread16(wk);
    lrow(Q, 2 * h + 1, limb(o, k));
  }
  if (q == 0) Q.fx[0] = (1u << S_B2) | (1u << S_IJKL);
}

__device__ __forceinline__ void q_add(Quad& Q, uint64_t A, uint64_t B, uint64_t M, bool has_m,
                                      int sel) {
  uint64_t s1 = A + B;
  uint32_t c1 = s1 < A;
  uint64_t s = s1 + M;
  uint32_t c2 = s < s1;
#pragma unroll
  for (int j = 0; j < 4; j++) {
    lrow(Q, j, limb(s, j));
    Q.c[A3][j] = limb(A, j);
    Q.c[A4][j] = limb(B, j);
    Q.c[A5][j] = has_m ? limb(M, j) : 0u;
  }
  Q.c[A9][0] = c1 + c2;
  Q.fx[0] = 1u << sel;
}

__device__ __forceinline__ void q_xor3(Quad& Q, uint64_t H, uint64_t V, uint64_t U, uint32_t q) {
  uint64_t e = H ^ V ^ U, mj = (H & V) | (H & U) | (V & U);
#pragma unroll
  for (int h = 0; h < 2; h++) {
    uint32_t k = 2 * q + h;
    lrow(Q, 2 * h, limb(e, k));
    Q.c[A3][2 * h] = spread16(limb(H, k));
    Q.c[A4][2 * h] = spread16(limb(V, k));
    Q.c[A5][2 * h] = spread16(limb(U, k));
    lrow(Q, 2 * h + 1, limb(mj, k));
  }
  if (q == 0) {
    Q.c[A7][0] = (uint32_t)e;
    Q.c[A8][0] = (uint32_t)(e >> 32);
    Q.fx[0] = (1u << S_XOR3) | (1u << S_DIGEST);
  }
}

__device__ __forceinline__ void quad_cells(Quad& Q, const b2f_input* __restrict__ x,
                                           const uint64_t* __restrict__ states,
                                           uint32_t rounds, uint32_t lq) {
  QuadInfo d = decode_quad(lq, rounds);
  switch (d.kind) {
    case K_INW: {
      uint64_t W = d.a < 8 ? x->h[d.a] : (d.a < 24 ? x->m[d.a - 8] : x->t[d.a - 24]);
#pragma unroll
      for (int j = 0; j < 4; j++) lrow(Q, j, limb(W, j));
      Q.c[A7][0] = (uint32_t)W;
      Q.c[A8][0] = (uint32_t)(W >> 32);
      Q.fx[0] = 1u << S_ABCD;
      break;
    }
    case K_FMASK: {
      uint32_t f = x->f ? 1u : 0u;
#pragma unroll
      for (int j = 0; j < 4; j++) lrow(Q, j, f ? 0xffffu : 0u);
      Q.c[A5][0] = f;
      Q.fx[0] = 1u << S_FMASK;
      break;
    }
    case K_CONST: {
      uint64_t W = c_iv[d.a];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        lrow(Q, j, limb(W, j));
        Q.fx[j] = (1u << S_CONST) | (limb(W, j) << 16);
      }
      break;
    }
    case K_XOR3: {
      const uint64_t* fin = states + 16ull * (2ull * rounds);
      q_xor3(Q, x->h[d.a], fin[d.a], fin[d.a + 8], d.q);
      break;
    }
    default: {
      if (d.block < INIT_ROWS) {  // init XORs: v12 = IV4^t0, v13 = IV5^t1, v14 = IV6^fmask
        uint64_t Y = d.a < 2 ? x->t[d.a] : (x->f ? ~0ull : 0ull);
        q_xor(Q, c_iv[4 + d.a], Y, d.q, S_XOR);
        break;
      }
      // round quad: recompute this G from the half-round state up to its step
      uint32_t r = d.a, g = d.g;
      const uint64_t* st = states + 16ull * (2ull * r + (g >= 4));
      uint64_t a = st[c_gidx[g][0]], b = st[c_gidx[g][1]];
      uint64_t c = st[c_gidx[g][2]], dd = st[c_gidx[g][3]];
      const uint8_t* sg = c_sigma[r % 10];
      uint64_t mx = x->m[sg[2 * g]], my = x->m[sg[2 * g + 1]];
      uint64_t a1 = a + b + mx;
      uint64_t d1 = rotr64(dd ^ a1, 32);
      uint64_t c1 = c + d1;
      uint64_t b1 = rotr64(b ^ c1, 24);
      uint64_t a2 = a1 + b1 + my;
      uint64_t d2 = rotr64(d1 ^ a2, 16);
      uint64_t c2 = c1 + d2;
      switch (d.step) {
        case 0: q_add(Q, a, b, mx, true, S_A1); break;
        case 1: q_xor(Q, dd, a1, d.q, S_D1); break;
        case 2: q_add(Q, c, d1, 0, false, S_C1); break;
        case 3: q_xor24(Q, b, c1, d.q); break;
        case 4: q_add(Q, a1, b1, my, true, S_A2); break;
        case 5: q_xor(Q, d1, a2, d.q, S_D2); break;
        case 6: q_add(Q, c1, d2, 0, false, S_C2); break;
        default: q_xor63(Q, b1, c2, d.q); break;
      }
      break;
    }
  }
}

constexpr uint64_t MAX_INSTANCE_ROWS = FIXED_ROWS + (uint64_t)ROUND_ROWS * B2F_MAX_ROUNDS;
static_assert(MAX_INSTANCE_ROWS < (1ull << 31), "instance-relative rows fit in int32");
constexpr int HIST = 384;                // >= 361 + quad alignment
constexpr int WSTRIDE = HIST + TSTRIDE;  // 1424
constexpr int NOFF = 9;                  // offsets of the first 8 instances of a tile (+1)

// Per-tile instance context, written by tile_info_kernel (96 bytes = 6 x 16 B).
struct TileInfo {
  uint32_t first;      // instance holding the tile's first row (n: none)
  uint32_t pad;
  uint64_t off[NOFF];  // off[first + i], clamped to off[n]
  uint64_t pad2[2];
};
static_assert(sizeof(TileInfo) == 96, "TileInfo is six 16-byte loads");

// Per-tile instance context: the instance holding the tile's first row and the offsets of the
// next 8 instances. One tiny prepass shared by the fill and eval launches of a call.
__global__ void tile_info_kernel(const uint64_t* __restrict__ off, uint32_t n, uint64_t n_tiles,
                                 TileInfo* __restrict__ ti) {
  uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tiles) return;
  uint64_t row = t * TILE_ROWS;
  TileInfo x;
  x.first = row < off[n] ? find_instance(off, n, row) : n;
  x.pad = 0;
#pragma unroll
  for (int i = 0; i < NOFF; i++) {
    uint64_t idx = (uint64_t)x.first + i;
    x.off[i] = off[idx < n ? idx : n];
  }
  x.pad2[0] = x.pad2[1] = 0;
  ti[t] = x;
}

// Round quads: one branch-free recipe for all eight G steps. The G is recomputed from its
// half-round state, the step's operands (X, Y, M) are selected, and every row of the quad is
// built from a per-(quad, row) recipe word, so all lanes of a wave run the same instructions
// whatever block they are in (LAYOUT.md §4 blocks ADD3/ADD2/XOR/XOR24/XOR63).
//   bits 0-1 limb k | 2-3 lookup source (0 S = X+Y+M, 1 Z = X^Y, 2 O = X&Y) | 4 lookup >> 8 |
//   5-6 lookup mask (0 0xffff, 1 0xff, 2 0x7fff) | 7-8 a3/a4 (0 none, 1 dense, 2 spread) |
//   9 a5 = M_k | 10 a7/a8 = W_k, spread(W_k) | 11 a6 = Z_k >> 15 | 12 a9 = carry |
//   16-31 selector bits of the row
struct RowTable {
  uint32_t r[G_QUADS][4];
};
constexpr uint32_t row_recipe(uint32_t k, uint32_t src, uint32_t sh8, uint32_t mask, uint32_t ops,
                              uint32_t m, uint32_t w, uint32_t zb, uint32_t cy, uint32_t sel) {
  return k | (src << 2) | (sh8 << 4) | (mask << 5) | (ops << 7) | (m << 9) | (w << 10) |
         (zb << 11) | (cy << 12) | (sel << 16);
}
constexpr uint32_t step_of_quad(uint32_t p) {  // a1 | d1 d1 | c1 | b1 b1 b1 | a2 | d2 d2 | c2 | b2 b2
  return (p >= 1) + (p >= 3) + (p >= 4) + (p >= 7) + (p >= 8) + (p >= 10) + (p >= 11);
}
constexpr RowTable make_rows() {
  RowTable T{};
  const uint32_t first_quad[8] = {0, 1, 3, 4, 7, 8, 10, 11};
  const uint32_t add_sel[8] = {1u << S_A1, 0, 1u << S_C1, 0, 1u << S_A2, 0, 1u << S_C2, 0};
  for (uint32_t p = 0; p < G_QUADS; p++) {
    uint32_t st = step_of_quad(p), q = p - first_quad[st];
    for (uint32_t j = 0; j < 4; j++) {
      uint32_t R = 4 * q + j, e = 0;
      if (st % 2 == 0) {  // ADD3 (a1, a2) / ADD2 (c1, c2)
        e = row_recipe(j, 0, 0, 0, 1, (st == 0 || st == 4) ? 1 : 0, 0, 0, j == 0, j == 0 ? add_sel[st] : 0);
      } else if (st == 1 || st == 5) {  // XOR (d1, d2)
        uint32_t sel = R == 0 ? (st == 1 ? 1u << S_D1 : 1u << S_D2) : 0;
        e = (R % 2 == 0) ? row_recipe(R / 2, 1, 0, 0, 2, 0, 0, 0, 0, sel)
                         : row_recipe(R / 2, 2, 0, 0, 0, 0, 0, 0, 0, 0);
      } else if (st == 3) {  // XOR24 (b1)
        uint32_t k = R / 3, t3 = R % 3, sel = R == 0 ? (1u << S_B1) | (1u << S_EFGH) : 0;
        e = t3 == 0 ? row_recipe(k, 1, 0, 1, 2, 0, 1, 0, 0, sel)
                    : t3 == 1 ? row_recipe(k, 1, 1, 1, 0, 0, 0, 0, 0, 0)
                              : row_recipe(k, 2, 0, 0, 0, 0, 0, 0, 0, 0);
      } else {  // XOR63 (b2)
        uint32_t sel = R == 0 ? (1u << S_B2) | (1u << S_IJKL) : 0;
        e = (R % 2 == 0) ? row_recipe(R / 2, 1, 0, 2, 2, 0, 1, 1, 0, sel)
                         : row_recipe(R / 2, 2, 0, 0, 0, 0, 0, 0, 0, 0);
      }
      T.r[p][j] = e;
    }
  }
  return T;
}
__constant__ __attribute__((aligned(16))) RowTable c_rows = make_rows();

__device__ __forceinline__ void quad_round(Quad& Q, uint64_t a, uint64_t b, uint64_t c,
                                           uint64_t d, uint64_t mx, uint64_t my, uint32_t p,
                                           const uint32_t* __restrict__ rows) {
  const uint64_t a1 = a + b + mx;
  const uint64_t d1 = rotr64(d ^ a1, 32);
  const uint64_t c1 = c + d1;
  const uint64_t b1 = rotr64(b ^ c1, 24);
  const uint64_t a2 = a1 + b1 + my;
  const uint64_t d2 = rotr64(d1 ^ a2, 16);
  const uint64_t c2 = c1 + d2;
  const uint32_t st = (p >= 1) + (p >= 3) + (p >= 4) + (p >= 7) + (p >= 8) + (p >= 10) + (p >= 11);
  const uint64_t X = st == 0 ? a : st == 1 ? d : st == 2 ? c : st == 3 ? b
                   : st == 4 ? a1 : st == 5 ? d1 : st == 6 ? c1 : b1;
  const uint64_t Y = st == 0 ? b : st == 1 ? a1 : st == 2 ? d1 : st == 3 ? c1
                   : st == 4 ? b1 : st == 5 ? a2 : st == 6 ? d2 : c2;
  const uint64_t M = st == 0 ? mx : st == 4 ? my : 0ull;
  const uint64_t s1 = X + Y, S = s1 + M;
  const uint32_t carry = (uint32_t)(s1 < X) + (uint32_t)(S < s1);
  const uint64_t Z = X ^ Y, O = X & Y;
  const uint64_t W = st == 3 ? rotr64(Z, 24) : rotr64(Z, 63);
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint32_t e = rows[4 * p + j];
    const uint32_t sh = 16 * (e & 3u);
    const uint32_t srcw = (e >> 2) & 3u;
    const uint64_t V = srcw == 0 ? S : srcw == 1 ? Z : O;
    const uint32_t mcode = (e >> 5) & 3u;
    const uint32_t v = (uint32_t)(V >> (sh + 8 * ((e >> 4) & 1u))) &
                       (mcode == 0 ? 0xffffu : mcode == 1 ? 0xffu : 0x7fffu);
    lrow(Q, j, v);
    const uint32_t xk = (uint32_t)(X >> sh) & 0xffffu, yk = (uint32_t)(Y >> sh) & 0xffffu;
    const uint32_t ops = (e >> 7) & 3u;
    Q.c[A3][j] = ops == 1 ? xk : ops == 2 ? spread16(xk) : 0u;
    Q.c[A4][j] = ops == 1 ? yk : ops == 2 ? spread16(yk) : 0u;
    Q.c[A5][j] = (e >> 9) & 1u ? (uint32_t)(M >> sh) & 0xffffu : 0u;
    Q.c[A6][j] = (e >> 11) & 1u ? ((uint32_t)(Z >> sh) & 0xffffu) >> 15 : 0u;
    const uint32_t wk = (uint32_t)(W >> sh) & 0xffffu;
    const bool hw = (e >> 10) & 1u;
    Q.c[A7][j] = hw ? wk : 0u;
    Q.c[A8][j] = hw ? spread16(wk) : 0u;
    Q.c[A9][j] = (e >> 12) & 1u ? carry : 0u;
    Q.fx[j] = e >> 16;
  }
}

// MODE (diagnostics; the product uses FILL_FULL): bit 0 = compute the cells (else zeros),
// bit 1 = non-temporal stores (else plain stores).
enum { FILL_COMPUTE = 1, FILL_NT = 2, FILL_FULL = 3 };

// Tiles of 1024 rows are dealt round-robin over the (persistent) workgroups, so at any time
// the chip writes a narrow band of every column: one DRAM-friendly front per column instead
// of one per workgroup.
template <int MODE>
__global__ void __launch_bounds__(BLOCK) fill_kernel(const b2f_input* __restrict__ in,
                                                    uint32_t n,
                                                    const uint64_t* __restrict__ off,
                                                    uint64_t total_rows,
                                                    const uint64_t* __restrict__ rec,
                                                    uint32_t* __restrict__ adv,
                                                    uint32_t* __restrict__ fixed,
                                                    const int* __restrict__ status,
                                                    const TileInfo* __restrict__ tinfo,
                                                    uint64_t n_tiles) {
  __shared__ uint32_t rows[G_QUADS * 4];
  if (threadIdx.x < G_QUADS * 4) rows[threadIdx.x] = (&c_rows.r[0][0])[threadIdx.x];
  __syncthreads();
  if (*status) return;  // the record kernel rejected the layout: write nothing
  const uint64_t total_quads = total_rows >> 2;
  const uint64_t used_rows = off[n];
  for (uint64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    uint64_t gq = t * BLOCK + threadIdx.x;
    if (gq >= total_quads) break;
    uint64_t row = 4 * gq;
    Quad Q;
    zero(Q);
    if ((MODE & FILL_COMPUTE) && row < used_rows) {
      uint32_t inst = tinfo[t].first;
      while (off[inst + 1] <= row) inst++;
      uint64_t o = off[inst];
      const b2f_input* x = in + inst;
      uint32_t rounds = x->rounds;
      const uint64_t* states = rec + 16ull * state_index(o, inst);
      const uint32_t lq = (uint32_t)((row - o) >> 2), rq = lq - INIT_QUADS;
      if (lq >= INIT_QUADS && rq < ROUND_QUADS * rounds) {
        const uint32_t r = rq / ROUND_QUADS, w = rq - r * ROUND_QUADS;
        const uint32_t g = w / G_QUADS, p = w - g * G_QUADS;
        const uint64_t* st = states + 16ull * (2ull * r + (g >= 4));
        const uint32_t gi = c_gidx_word[g];  // a | b << 8 | c << 16 | d << 24
        const uint32_t sg = c_sigma_pair[r % 10][g];
        quad_round(Q, st[gi & 0xff], st[(gi >> 8) & 0xff], st[(gi >> 16) & 0xff], st[gi >> 24],
                   x->m[sg & 0xff], x->m[sg >> 8], p, rows);
      } else {
        quad_cells(Q, x, states, rounds, lq);  // init and final regions
      }
    }
#pragma unroll
    for (int c = 0; c < 11; c++) {
      u32x4 v = c < 10 ? u32x4{Q.c[c][0], Q.c[c][1], Q.c[c][2], Q.c[c][3]}
                       : u32x4{Q.fx[0], Q.fx[1], Q.fx[2], Q.fx[3]};
      u32x4* dst = reinterpret_cast<u32x4*>((c < 10 ? adv + (uint64_t)c * total_rows : fixed) + row);
      if (MODE & FILL_NT) __builtin_nontemporal_store(v, dst);
      else *dst = v;
    }
  }
}

// --------------------------------------------------------------------------- eval kernel
//
// Software-pipelined over 1024-row tiles dealt round-robin to persistent workgroups (3 per
// CU). While a workgroup checks tile t out of LDS, its loads for tile t + gridDim are already
// in flight into registers; at the next iteration they are written to LDS behind one barrier.
//
// Per tile, one lane of the first wave per G whose rows meet the tile builds the G table (its
// window/init-cache bases, message rows, G index) and marks which quads are round quads; the
// gates of canonical round blocks and the 72 copy checks of every G then run from that table
// spread evenly over the workgroup, whatever block each quad holds. Only init/final quads
// (about 4% at 12 rounds) and non-canonical selector rows take per-quad paths.
//
// LDS per workgroup (one array, 16-byte aligned carve):
//   W   the canonical columns a_1 a_2 a_7 a_8 (every copy source is one of them) for rows
//       [tile0 - HIST, tile0 + TILE_ROWS + HALO): the tile plus a history window holding
//       every state-word source (<= 361 rows back, see max_copy_distance);
//   G   the other gate columns a_0 a_3 a_4 a_5 a_6 for rows [tile0, tile0 + TILE_ROWS + HALO);
//   CT  copy-check table (make_check_table), SG SIGMA, INFO the tile's TileInfo,
//   IC  init-region cache: a_1 | a_2 of rows 0..163 of the tile's first instance, the only
//       instance whose init region (h, m, t, fmask, IV, v12..v14) can lie before the window;
//   GT  the tile's G table, QM quad -> position in its G (0xff: not a round quad),
//   QSEL / A9 per quad: row-0 selector bits (| 1 << 16 if rows 1-3 carry any) and row-0 a_9.
// a_9 and the fixed column are otherwise only read on their own row: kept in registers.

constexpr int G_CHECKS = 72;  // copy constraints per G (static_assert below)
constexpr int MAX_TILE_G = 24;  // G starts in [tile0 - 51, tile0 + 1023]: at most 21
constexpr int GT_WORDS = 8;

constexpr int L_W = 0;
constexpr int L_G = L_W + 4 * WSTRIDE;
constexpr int L_CT = L_G + 5 * TSTRIDE;
constexpr int L_SG = L_CT + 12 * G_CHECKS;
constexpr int L_INFO = L_SG + 40;
constexpr int L_IC = L_INFO + 24;
constexpr int L_XS = L_IC + 2 * INIT_ROWS;   // expected row-0 selector bits per G quad (16)
constexpr int L_QSEL = L_XS + 16;
constexpr int L_A9 = L_QSEL + BLOCK;
constexpr int L_INFO2 = L_A9 + BLOCK;        // the TileInfo two tiles ahead (t + gridDim)
// G set: G table (MAX_TILE_G x GT_WORDS), QM (BLOCK bytes), NG (entries); two sets, the one of
// the current tile and the one being built for the next
constexpr int GS_GT = 0, GS_QM = MAX_TILE_G * GT_WORDS, GS_NG = GS_QM + BLOCK / 4;
constexpr int GSET = GS_NG + 4;
constexpr int L_GS = L_INFO2 + 24;
constexpr int L_ACC = L_GS + 2 * GSET;  // 16 gate + lookup + copy counters, first (u64)
constexpr int LDS_WORDS = L_ACC + 20 + 2;
static_assert(L_INFO % 4 == 0 && L_IC % 4 == 0 && L_G % 4 == 0 && L_CT % 4 == 0 && L_ACC % 2 == 0,
              "aligned carve");
static_assert(LDS_WORDS * 4 * 3 <= 160 * 1024, "three eval workgroups per CU");

// Row-0 selector bits of each quad of a G when the fixed column is canonical (LAYOUT.md §5:
// a1 | d1 d1 | c1 | b1 b1 b1 | a2 | d2 d2 | c2 | b2 b2, blocks start on a quad, rows 1-3 of
// every round quad carry no selector).
constexpr uint32_t expected_sel(uint32_t p) {
  return p == 0 ? 1u << S_A1 : p == 1 ? 1u << S_D1 : p == 3 ? 1u << S_C1
       : p == 4 ? (1u << S_B1) | (1u << S_EFGH) : p == 7 ? 1u << S_A2 : p == 8 ? 1u << S_D2
       : p == 10 ? 1u << S_C2 : p == 11 ? (1u << S_B2) | (1u << S_IJKL) : 0u;
}
constexpr bool expected_sel_matches_fill() {
  RowTable R = make_rows();
  for (uint32_t p = 0; p < G_QUADS; p++)
    for (uint32_t j = 0; j < 4; j++)
      if ((R.r[p][j] >> 16) != (j == 0 ? expected_sel(p) : 0u)) return false;
  return true;
}
static_assert(expected_sel_matches_fill(), "eval's canonical selectors = the fill's");

// Extra (non-own-quad) loads of a tile: 2 slots per thread.
constexpr int X_HIST = 4 * (HIST / 4);          // 384: 96 quads x 4 canonical columns
constexpr int X_HALO = X_HIST + 9 * (HALO_ROWS / 4);  // +36: 4 quads x 9 gate columns
constexpr int X_INIT = X_HALO + 2 * INIT_QUADS;  // +82: 41 quads x (a_1, a_2)
constexpr int X_INFO = X_INIT + 5;               // +5: TileInfo words 0..19 (first, off[9])
constexpr int X_INFO2 = X_INFO + 5;              // +5: the same for tile t + gridDim
static_assert(X_INFO2 <= 2 * BLOCK, "two extra slots per thread");

// copy-source descriptor (u16): bits 0-1 kind: 0 none, 1 in-G (bits 2-7 row from the G's first
// row, bits 8-11 column), 2 state word at the half-round start (bits 2-3 role a/b/c/d, bits 4-5
// limb, bit 6 spread), 3 message word (bit 2: y instead of x, bits 4-5 limb).
struct DescTable {
  uint16_t d[G_QUADS][4][3];
};
constexpr uint16_t d_ing(uint32_t rel, uint32_t col) { return (uint16_t)(1 | (rel << 2) | (col << 8)); }
constexpr uint16_t d_state(uint32_t role, uint32_t k, uint32_t spread) {
  return (uint16_t)(2 | (role << 2) | (k << 4) | (spread << 6));
}
constexpr uint16_t d_msg(uint32_t y, uint32_t k) { return (uint16_t)(3 | (y << 2) | (k << 4)); }

// LAYOUT.md §5 round table, operand by operand.
constexpr DescTable make_desc() {
  DescTable T{};
  for (uint32_t k = 0; k < 4; k++) {
    T.d[0][k][0] = d_state(0, k, 0);  // a1 = a + b + x
    T.d[0][k][1] = d_state(1, k, 0);
    T.d[0][k][2] = d_msg(0, k);
    T.d[3][k][0] = d_state(2, k, 0);  // c1 = c + d1
    T.d[3][k][1] = d_ing(4 + 2 * ((k + 2) & 3), A1);
    T.d[7][k][0] = d_ing(0 + k, A1);  // a2 = a1 + b1 + y
    T.d[7][k][1] = d_ing(16 + 3 * k, A7);
    T.d[7][k][2] = d_msg(1, k);
    T.d[10][k][0] = d_ing(12 + k, A1);  // c2 = c1 + d2
    T.d[10][k][1] = d_ing(32 + 2 * ((k + 1) & 3), A1);
  }
  for (uint32_t p = 0; p < 2; p++)
    for (uint32_t j = 0; j < 4; j += 2) {
      uint32_t k = (4 * p + j) / 2;
      T.d[1 + p][j][0] = d_state(3, k, 1);  // d1 = (d ^ a1) >>> 32
      T.d[1 + p][j][1] = d_ing(0 + k, A2);
      T.d[8 + p][j][0] = d_ing(4 + 2 * ((k + 2) & 3), A2);  // d2 = (d1 ^ a2) >>> 16
      T.d[8 + p][j][1] = d_ing(28 + k, A2);
      T.d[11 + p][j][0] = d_ing(16 + 3 * k, A8);  // b2 = (b1 ^ c2) >>> 63
      T.d[11 + p][j][1] = d_ing(40 + k, A2);
    }
  for (uint32_t p = 0; p < 3; p++)
    for (uint32_t j = 0; j < 4; j++) {
      uint32_t R = 4 * p + j;
      if (R % 3) continue;
      uint32_t k = R / 3;
      T.d[4 + p][j][0] = d_state(1, k, 1);  // b1 = (b ^ c1) >>> 24
      T.d[4 + p][j][1] = d_ing(12 + k, A2);
    }
  return T;
}

// The copy sources of every operand cell of a round quad, resolved per G index g at compile
// time (u32 per (g, quad, row, operand)):
//   bits 0-1  kind (0 none, 1 in-G, 2 state word, 3 message word)
//   bits 2-3  source column as W index (a_1 a_2 a_7 a_8 -> 0..3), for half-rounds >= 1
//   bits 4-5  limb k, bit 6: message y instead of x
//   bits 7-16 row offset from the consumer G's first row, +512 (in-G; state for hr >= 1)
//   bits 17-24 row inside the instance's init region (state word at hr = 0)
//   bits 25-26 source column (W index) at hr = 0
// Rows of half-round hr start at 164 + 208 hr, G g at + 52 (g & 3); the producer of a state
// word sits in the previous half-round, whose parity is fixed by g, so the offset from the
// consumer's G is a constant of (g, role, limb).
constexpr uint8_t kGidx[8][4] = {{0, 4, 8, 12}, {1, 5, 9, 13}, {2, 6, 10, 14}, {3, 7, 11, 15},
                                 {0, 5, 10, 15}, {1, 6, 11, 12}, {2, 7, 8, 13}, {3, 4, 9, 14}};
constexpr uint32_t wc_of(uint32_t col) { return col == A1 ? 0 : col == A2 ? 1 : col == A7 ? 2 : 3; }

// The copy checks of one G as a flat list (every operand cell of its eight blocks that is a
// copy, LAYOUT.md §5 round table), with each source resolved at compile time per G index g:
// entry [g] for half-rounds >= 1, [8 + g] for the first half-round (g < 4), whose state words
// come from the instance's init region. Entry (u32):
//   bits 0-13  C: LDS offset of the source relative to the per-G base chosen by bits 14-16
//   bits 14-16 base: 0 window at the G start (- CBIAS), 1 init-region a_1, 2 init-region a_2,
//              3 message x row, 4 message y row (GT words 0..4)
//   bits 17-18 operand column a_3 / a_4 / a_5;  bits 19-24 operand row in the G (0..51)
// In-G and state-word sources are `rel` rows from the G start: the state word of role a/b/c/d
// of the half-round start was produced by the G of the previous half-round that owns it, in
// its last step of that role (a <- a2 +28, b <- b2 +44 stride 2, c <- c2 +40, d <- d2 +32
// rot 16), whose index is fixed by g, so rel is a constant of (g, role, limb).
constexpr int CBIAS = 512;
struct CheckTable {
  uint32_t e[12][G_CHECKS];
};
constexpr uint32_t pack_check(uint32_t C, uint32_t base, uint32_t dcol, uint32_t drow) {
  return C | (base << 14) | (dcol << 17) | (drow << 19);
}
constexpr int state_rel(uint32_t g, uint32_t role, uint32_t k) {
  uint32_t w = kGidx[g][role], pos = w & 3u;
  uint32_t prev_odd = g < 4 ? 1u : 0u;  // parity of the previous half-round
  uint32_t gp = prev_odd ? ((pos - role) & 3u) : pos;
  uint32_t off = role == 0 ? 28 + k : role == 1 ? 44 + 2 * k : role == 2 ? 40 + k
                                                               : 32 + 2 * ((k + 1) & 3u);
  return -(int)ROUND_ROWS / 2 + (int)G_ROWS * ((int)gp - (int)(g & 3u)) + (int)off;
}
constexpr uint32_t state_abs0(uint32_t g, uint32_t role, uint32_t k) {  // init-region row
  uint32_t w = kGidx[g][role];
  return w < 8 ? 4 * w + k : (w >= 12 && w < 15) ? 140 + 8 * (w - 12) + 2 * k
                                                 : 108 + 4 * (w == 15 ? 7u : w - 8) + k;
}
constexpr CheckTable make_check_table() {
  CheckTable T{};
  DescTable D = make_desc();
  for (uint32_t v = 0; v < 12; v++) {
    uint32_t g = v < 8 ? v : v - 8;
    bool hr0 = v >= 8;
    int ci = 0;
    for (uint32_t p = 0; p < G_QUADS; p++)
      for (uint32_t j = 0; j < 4; j++)
        for (uint32_t c = 0; c < 3; c++) {
          uint32_t d = D.d[p][j][c], kind = d & 3u, drow = 4 * p + j, e = 0;
          if (kind == 0) continue;
          if (kind == 1) {
            uint32_t rel = (d >> 2) & 63u, wc = wc_of(d >> 8);
            e = pack_check(L_W + wc * WSTRIDE + rel + CBIAS, 0, c, drow);
          } else if (kind == 2) {
            uint32_t role = (d >> 2) & 3u, k = (d >> 4) & 3u, sp = (d >> 6) & 1u;
            if (hr0) {
              e = pack_check(state_abs0(g, role, k), 1 + sp, c, drow);
            } else {
              uint32_t col = role == 1 ? (sp ? A8 : A7) : (sp ? A2 : A1);
              e = pack_check((uint32_t)((int)(L_W + wc_of(col) * WSTRIDE) + state_rel(g, role, k) + CBIAS),
                             0, c, drow);
            }
          } else {
            e = pack_check((d >> 4) & 3u, 3 + ((d >> 2) & 1u), c, drow);
          }
          if (ci < G_CHECKS) T.e[v][ci] = e;
          ci++;
        }
    if (ci != G_CHECKS) T.e[0][0] = 0xffffffffu;  // trips the static_assert below
  }
  return T;
}
constexpr bool check_table_ok() {
  CheckTable T = make_check_table();
  if (T.e[0][0] == 0xffffffffu) return false;
  for (int v = 0; v < 12; v++)
    for (int i = 0; i < G_CHECKS; i++) {
      uint32_t e = T.e[v][i];
      if (((e >> 14) & 7u) > 4 || ((e >> 19) & 63u) >= G_ROWS || ((e >> 17) & 3u) > 2) return false;
    }
  return true;
}
static_assert(check_table_ok(), "72 copy checks per G, fields in range");
// The deepest state-word source (consumer row - source row) must fit the history window.
constexpr int max_copy_distance() {
  DescTable D = make_desc();
  int m = 0;
  for (uint32_t g = 0; g < 8; g++)
    for (uint32_t p = 0; p < G_QUADS; p++)
      for (uint32_t j = 0; j < 4; j++)
        for (uint32_t c = 0; c < 3; c++) {
          uint32_t d = D.d[p][j][c];
          if ((d & 3u) != 2) continue;
          int dist = (int)(4 * p + j) - state_rel(g, (d >> 2) & 3u, (d >> 4) & 3u);
          m = dist > m ? dist : m;
        }
  return m;
}
static_assert(max_copy_distance() + 4 <= HIST, "history window too small for state sources");

__constant__ __attribute__((aligned(16))) CheckTable c_checks = make_check_table();
constexpr int CHECK_WORDS = (int)(sizeof(CheckTable) / 4);  // 864

// Failure accounting. Failures are rare, so they go straight to LDS atomics (per-workgroup
// counters, flushed once at the end) instead of occupying registers on the hot path.
struct EvalAcc {
  uint32_t* c;  // [0..15] gates, [16] lookup, [17] copy, [18..19] pad, [20..21] first (u64)
  __device__ __forceinline__ void fail(uint64_t row, uint32_t code) {
    atomicAdd(&c[code], 1u);
    atomicMin(reinterpret_cast<unsigned long long*>(c + 20), (unsigned long long)((row << 8) | code));
  }
  __device__ __forceinline__ void fail_gates(uint64_t row, uint32_t mask) {
    for (uint32_t m = mask; m; m &= m - 1) atomicAdd(&c[__builtin_ctz(m)], 1u);
    atomicMin(reinterpret_cast<unsigned long long*>(c + 20),
              (unsigned long long)((row << 8) | (uint32_t)__builtin_ctz(mask)));
  }
};

// component j of a quad register (select chain: never an indexed access into a register array)
__device__ __forceinline__ uint32_t comp(const uint4& v, int j) {
  return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}

// LDS cell accessor: column c, tile-local row r (r may reach TILE_ROWS + 11)
struct Tile {
  const uint32_t* L;
  __device__ __forceinline__ uint32_t at(int c, uint32_t r) const {
    switch (c) {
      case A1: return L[L_W + 0 * WSTRIDE + HIST + r];
      case A2: return L[L_W + 1 * WSTRIDE + HIST + r];
      case A7: return L[L_W + 2 * WSTRIDE + HIST + r];
      case A8: return L[L_W + 3 * WSTRIDE + HIST + r];
      case A0: return L[L_G + 0 * TSTRIDE + r];
      case A3: return L[L_G + 1 * TSTRIDE + r];
      case A4: return L[L_G + 2 * TSTRIDE + r];
      case A5: return L[L_G + 3 * TSTRIDE + r];
      default: return L[L_G + 4 * TSTRIDE + r];  // A6
    }
  }
  __device__ __forceinline__ uint4 quad(int c, uint32_t r) const {
    return *reinterpret_cast<const uint4*>(&L[(c == A1 || c == A2 || c == A7 || c == A8)
                                                  ? L_W + (c == A1 ? 0 : c == A2 ? 1 : c == A7 ? 2 : 3) * WSTRIDE + HIST + r
                                                  : L_G + (c == A0 ? 0 : c - 2) * TSTRIDE + r]);
  }
};
#define TC(c, r) T.at((c), (r))

// LDS word offset of column c (a_0..a_8) at tile-local row r
__device__ __forceinline__ int lds_cell(int c, int r) {
  switch (c) {
    case A1: return L_W + 0 * WSTRIDE + HIST + r;
    case A2: return L_W + 1 * WSTRIDE + HIST + r;
    case A7: return L_W + 2 * WSTRIDE + HIST + r;
    case A8: return L_W + 3 * WSTRIDE + HIST + r;
    case A0: return L_G + r;
    default: return L_G + (c - 2) * TSTRIDE + r;  // A3..A6 -> 1..4
  }
}

// Evaluate gate `s` on the block whose selector row is tile-local row r. Every identity of
// LAYOUT.md §4 is checked in an exact integer form: linear identities as equalities in
// 64/128-bit arithmetic (all terms are < 2^100), the root constraints c(c-1)(c-2), t(t-1),
// b(b-1) as range tests (equivalent for non-negative integers < p). a9 and k0 are the
// selector row's own a_9 and fixed cells.
__device__ __forceinline__ bool gate_ok(const Tile& T, int s, uint32_t r, uint32_t a9,
                                        uint32_t k0) {
  typedef unsigned __int128 u128;
  switch (s) {
    case S_ABCD:
      return (uint64_t)TC(A7, r) == (uint64_t)TC(A1, r) + ((uint64_t)TC(A1, r + 1) << 16) &&
             (uint64_t)TC(A8, r) == (uint64_t)TC(A1, r + 2) + ((uint64_t)TC(A1, r + 3) << 16);
    case S_DIGEST:
      return (uint64_t)TC(A7, r) == (uint64_t)TC(A1, r) + ((uint64_t)TC(A1, r + 2) << 16) &&
             (uint64_t)TC(A8, r) == (uint64_t)TC(A1, r + 4) + ((uint64_t)TC(A1, r + 6) << 16);
    case S_EFGH: {
      bool ok = true;
#pragma unroll 1
      for (uint32_t k = 0; k < 4; k++) {
        uint32_t k1 = (k + 1) & 3, k2 = (k + 2) & 3;
        ok &= (uint64_t)TC(A7, r + 3 * k) ==
              (uint64_t)TC(A1, r + 3 * k1 + 1) + ((uint64_t)TC(A1, r + 3 * k2) << 8);
        ok &= (uint64_t)TC(A8, r + 3 * k) ==
              (uint64_t)TC(A2, r + 3 * k1 + 1) + ((uint64_t)TC(A2, r + 3 * k2) << 16);
      }
      return ok;
    }
    case S_IJKL: {
      bool ok = true;
#pragma unroll 1
      for (uint32_t k = 0; k < 4; k++) {
        uint32_t k3 = (k + 3) & 3;
        uint64_t zb = TC(A6, r + 2 * k3);
        ok &= (uint64_t)TC(A7, r + 2 * k) == zb + 2 * (uint64_t)TC(A1, r + 2 * k);
        ok &= (uint64_t)TC(A8, r + 2 * k) == zb + 4 * (uint64_t)TC(A2, r + 2 * k);
      }
      return ok;
    }
    case S_A1:
    case S_A2:
    case S_C1:
    case S_C2: {
      bool three = (s == S_A1 || s == S_A2);
      u128 lhs = 0, rhs = 0;
#pragma unroll 1
      for (uint32_t k = 0; k < 4; k++) {
        uint64_t in = (uint64_t)TC(A3, r + k) + TC(A4, r + k) + (three ? TC(A5, r + k) : 0u);
        lhs += (u128)in << (16 * k);
        rhs += (u128)TC(A1, r + k) << (16 * k);
      }
      rhs += (u128)a9 << 64;
      return lhs == rhs && a9 <= (three ? 2u : 1u);
    }
    case S_B1: {
      bool ok = true;
#pragma unroll 1
      for (uint32_t k = 0; k < 4; k++) {
        uint32_t b = r + 3 * k;
        ok &= (uint64_t)TC(A3, b) + TC(A4, b) ==
              (uint64_t)TC(A2, b) + ((uint64_t)TC(A2, b + 1) << 16) + 2 * (uint64_t)TC(A2, b + 2);
        ok &= TC(A0, b) == 0u && TC(A0, b + 1) == 0u;
      }
      return ok;
    }
    case S_D1:
    case S_D2:
    case S_XOR: {
      bool ok = true;
#pragma unroll 1
      for (uint32_t k = 0; k < 4; k++) {
        uint32_t b = r + 2 * k;
        ok &= (uint64_t)TC(A3, b) + TC(A4, b) == (uint64_t)TC(A2, b) + 2 * (uint64_t)TC(A2, b + 1);
      }
      return ok;
    }
    case S_B2: {
      bool ok = true;
#pragma unroll 1
      for (uint32_t k = 0; k < 4; k++) {
        uint32_t b = r + 2 * k;
        uint32_t zb = TC(A6, b);
        ok &= (uint64_t)TC(A3, b) + TC(A4, b) ==
              (uint64_t)TC(A2, b) + ((uint64_t)zb << 30) + 2 * (uint64_t)TC(A2, b + 1);
        ok &= TC(A0, b) <= 1u && zb <= 1u;
      }
      return ok;
    }
    case S_XOR3: {
      bool ok = true;
#pragma unroll 1
      for (uint32_t k = 0; k < 4; k++) {
        uint32_t b = r + 2 * k;
        ok &= (uint64_t)TC(A3, b) + TC(A4, b) + TC(A5, b) ==
              (uint64_t)TC(A2, b) + 2 * (uint64_t)TC(A2, b + 1);
      }
      return ok;
    }
    case S_CONST:
      return TC(A1, r) == (k0 >> 16);
    case S_FMASK: {
      uint32_t f = TC(A5, r);
      bool ok = f <= 1u;
#pragma unroll 1
      for (uint32_t k = 0; k < 4; k++) ok &= (uint64_t)TC(A1, r + k) == 65535ull * f;
      return ok;
    }
  }
  return true;
}

// Block gate evaluators: the gates of one block from 4-row LDS vectors (ds_read_b128), for
// the selector patterns LAYOUT v1 writes. Each returns the mask of failing selector bits.
// Any other selector combination (only a corrupted fixed column has one) is evaluated one
// gate at a time by gate_ok. Both paths check the same identities.
struct V3 {  // 12 consecutive rows of one column
  uint4 a, b, c;
  __device__ __forceinline__ uint32_t operator[](int i) const {
    const uint4& v = i < 4 ? a : (i < 8 ? b : c);
    return comp(v, i & 3);
  }
};
__device__ __forceinline__ V3 rows12(const Tile& T, int col, uint32_t r) {
  return V3{T.quad(col, r), T.quad(col, r + 4), T.quad(col, r + 8)};
}
__device__ __forceinline__ V3 rows8(const Tile& T, int col, uint32_t r) {
  return V3{T.quad(col, r), T.quad(col, r + 4), make_uint4(0, 0, 0, 0)};
}

// XOR (s_spread_d1, s_spread_d2, s_xor) and XOR3 (s_xor3): operands on the even rows
__device__ __forceinline__ bool g_xor(const Tile& T, uint32_t r, bool three) {
  V3 s2 = rows8(T, A2, r);
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint64_t in = (uint64_t)T.at(A3, r + 2 * k) + T.at(A4, r + 2 * k) + (three ? T.at(A5, r + 2 * k) : 0u);
    ok &= in == (uint64_t)s2[2 * k] + 2 * (uint64_t)s2[2 * k + 1];
  }
  return ok;
}
__device__ __forceinline__ bool g_digest(const Tile& T, uint32_t r) {
  V3 d = rows8(T, A1, r);
  return (uint64_t)T.at(A7, r) == (uint64_t)d[0] + ((uint64_t)d[2] << 16) &&
         (uint64_t)T.at(A8, r) == (uint64_t)d[4] + ((uint64_t)d[6] << 16);
}
__device__ __forceinline__ bool g_add(const Tile& T, uint32_t r, uint32_t a9, bool three) {
  typedef unsigned __int128 u128;
  uint4 s = T.quad(A1, r), x = T.quad(A3, r), y = T.quad(A4, r);
  uint4 z = three ? T.quad(A5, r) : make_uint4(0, 0, 0, 0);
  u128 lhs = 0, rhs = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    lhs += (u128)((uint64_t)comp(x, k) + comp(y, k) + comp(z, k)) << (16 * k);
    rhs += (u128)comp(s, k) << (16 * k);
  }
  rhs += (u128)a9 << 64;
  return lhs == rhs && a9 <= (three ? 2u : 1u);
}
__device__ __forceinline__ uint32_t g_xor24(const Tile& T, uint32_t r, uint32_t sel) {
  bool b1 = true, efgh = true;
#pragma unroll 1
  for (int k = 0; k < 4; k++) {
    uint32_t b = r + 3 * k, k1 = r + 3 * ((k + 1) & 3), k2 = r + 3 * ((k + 2) & 3);
    b1 &= (uint64_t)T.at(A3, b) + T.at(A4, b) ==
          (uint64_t)T.at(A2, b) + ((uint64_t)T.at(A2, b + 1) << 16) + 2 * (uint64_t)T.at(A2, b + 2);
    b1 &= (T.at(A0, b) | T.at(A0, b + 1)) == 0u;
    efgh &= (uint64_t)T.at(A7, b) == (uint64_t)T.at(A1, k1 + 1) + ((uint64_t)T.at(A1, k2) << 8);
    efgh &= (uint64_t)T.at(A8, b) == (uint64_t)T.at(A2, k1 + 1) + ((uint64_t)T.at(A2, k2) << 16);
  }
  return ((b1 ? 0u : 1u << S_B1) | (efgh ? 0u : 1u << S_EFGH)) & sel;
}
__device__ __forceinline__ uint32_t g_xor63(const Tile& T, uint32_t r, uint32_t sel) {
  V3 a2 = rows8(T, A2, r);
  bool b2 = true, ijkl = true;
#pragma unroll 1
  for (int k = 0; k < 4; k++) {
    uint32_t b = 2 * k, k3 = 2 * ((k + 3) & 3);
    uint32_t zb = T.at(A6, r + b), zp = T.at(A6, r + k3);
    b2 &= (uint64_t)T.at(A3, r + b) + T.at(A4, r + b) ==
          (uint64_t)a2[b] + ((uint64_t)zb << 30) + 2 * (uint64_t)a2[b + 1];
    b2 &= T.at(A0, r + b) <= 1u && zb <= 1u;
    ijkl &= (uint64_t)T.at(A7, r + b) == (uint64_t)zp + 2 * (uint64_t)T.at(A1, r + b);
    ijkl &= (uint64_t)T.at(A8, r + b) == (uint64_t)zp + 4 * (uint64_t)a2[b];
  }
  return ((b2 ? 0u : 1u << S_B2) | (ijkl ? 0u : 1u << S_IJKL)) & sel;
}

// Any selector combination, one gate at a time (kept out of line: the hot path never takes it
// for a trace this engine wrote).
__device__ __noinline__ uint32_t gates_generic(const Tile& T, uint32_t sel, uint32_t r, uint32_t a9,
                                               uint32_t k0) {
  uint32_t failed = 0;
  while (sel) {
    int s = __builtin_ctz(sel);
    sel &= sel - 1;
    if (!gate_ok(T, s, r, a9, k0)) failed |= 1u << s;
  }
  return failed;
}

// Failing selector bits of selector row r (tile-local), for rows the per-G pass does not take:
// the init and final blocks (XOR, XOR3 + digest inline; the rest out of line) and any
// non-canonical selector row of a corrupted fixed column.
__device__ __forceinline__ uint32_t row_gates(const Tile& T, uint32_t sel, uint32_t r, uint32_t a9,
                                              uint32_t k0) {
  switch (sel) {
    case 1u << S_XOR:
      return g_xor(T, r, false) ? 0u : sel;
    case (1u << S_XOR3) | (1u << S_DIGEST):
      return (g_xor(T, r, true) ? 0u : 1u << S_XOR3) | (g_digest(T, r) ? 0u : 1u << S_DIGEST);
    default:
      return gates_generic(T, sel, r, a9, k0);
  }
}

// G table of a tile (first wave, lane l = l-th G in row order whose start lies in
// [tile0 - 51, tile0 + 1023], over the instances cached in INFO). GT words:
//   0 window base of the G start - CBIAS     1, 2 init-region base of a_1, a_2
//   3, 4 message x / y row bases             5 G start, tile-local      6 check-table row
// Init-region bases point into the init cache for the tile's first instance (its init region
// may lie before the window) and into the window for any later instance (which starts inside
// the tile, so its init region is in the window). QM[q] = position of quad q in its G.
// Instances past the cached eight cannot occur in a valid layout (each is >= 228 rows);
// b2f_eval_dev flags invalid layouts separately (offsets_check_kernel).
__device__ __forceinline__ void build_g_table(uint32_t* S, const uint32_t* info, const uint8_t* Sg,
                                              uint64_t tile0, uint32_t n, uint64_t total_rows,
                                              uint32_t lane) {
  // one wave: its lanes reset QM, then mark their G's quads (LDS order within a wave)
  S[GS_QM + lane] = 0xffffffffu;
  const uint32_t first = info[0];
  const uint64_t* Off = reinterpret_cast<const uint64_t*>(info + 2);
  const int64_t lo = (int64_t)tile0 - (G_ROWS - 1), hi = (int64_t)tile0 + TILE_ROWS - 1;
  uint32_t base = 0, m = 0;
  int64_t o_mine = -1;
  bool ofst = false;
  for (int i = 0; i + 1 < NOFF; i++) {
    if (first + (uint32_t)i >= n) break;
    const uint64_t o = Off[i], o1 = Off[i + 1];
    if ((int64_t)o > hi) break;
    if (o1 <= o || o1 > total_rows || o1 - o > MAX_INSTANCE_ROWS) continue;
    const uint32_t R = (uint32_t)(o1 - o);
    if (R < FIXED_ROWS || (R - FIXED_ROWS) % ROUND_ROWS) continue;
    const uint32_t n_g = 8 * ((R - FIXED_ROWS) / ROUND_ROWS);
    // G m starts at g0 + 52 m; o > tile0 - MAX_INSTANCE_ROWS, so these fit in 32 bits
    const int64_t g0 = (int64_t)o + INIT_ROWS;
    const int b = (int)(hi - g0);
    if (n_g == 0 || b < 0) continue;
    const int a = (int)(lo - g0);
    const uint32_t m_lo = a <= 0 ? 0u : ((uint32_t)a + G_ROWS - 1) / G_ROWS;
    uint32_t m_hi = (uint32_t)b / G_ROWS;
    if (m_hi >= n_g) m_hi = n_g - 1;
    if (m_lo > m_hi) continue;
    const uint32_t cnt = m_hi - m_lo + 1;
    if (o_mine < 0 && lane >= base && lane < base + cnt) {
      o_mine = (int64_t)o;
      m = m_lo + (lane - base);
      ofst = i == 0;
    }
    base += cnt;
  }
  if (lane == 0) S[GS_NG] = base < (uint32_t)MAX_TILE_G ? base : (uint32_t)MAX_TILE_G;
  if (o_mine < 0 || lane >= (uint32_t)MAX_TILE_G) return;
  const uint32_t r = m >> 3, g = m & 7u;
  const int gl = (int)(o_mine + INIT_ROWS + (int64_t)G_ROWS * m - (int64_t)tile0);
  const int64_t ob64 = o_mine - (int64_t)tile0 + HIST;  // instance start, window index
  const int ob = ofst ? 0 : (int)ob64;                    // (later instances: in the window)
  const int ib0 = ofst ? L_IC : L_W + ob;
  const int ib1 = ofst ? L_IC + (int)INIT_ROWS : L_W + WSTRIDE + ob;
  const uint8_t* sg = Sg + 16 * (r % 10) + 2 * g;
  uint32_t* gt = S + GS_GT + GT_WORDS * lane;
  gt[0] = (uint32_t)(gl + HIST - CBIAS);
  gt[1] = (uint32_t)ib0;
  gt[2] = (uint32_t)ib1;
  gt[3] = (uint32_t)(ib0 + 32 + 4 * sg[0]);
  gt[4] = (uint32_t)(ib0 + 32 + 4 * sg[1]);
  gt[5] = (uint32_t)gl;
  gt[6] = (m < 4 ? 8 + g : g) * G_CHECKS;
  uint8_t* qm = reinterpret_cast<uint8_t*>(S + GS_QM);
#pragma unroll
  for (int p = 0; p < (int)G_QUADS; p++) {
    int q = (gl >> 2) + p;
    if (q >= 0 && q < BLOCK) qm[q] = (uint8_t)p;
  }
}

// Gates of the canonical round blocks of a tile. Lane l of every wave takes item l =
// (G table entry l >> 1, half l & 1), and wave w checks block kind w of it: 0 a1/a2 (ADD3,
// +0/+28), 1 d1/d2 (XOR, +4/+32), 2 c1/c2 (ADD2, +12/+40), 3 b1 (XOR24, +16) / b2 (XOR63,
// +44). Each wave thus runs one evaluator (the b wave two) instead of every wave running all
// five block kinds mostly masked, as a quad-per-lane assignment would. A block is checked here
// only if its selector row lies in this tile and its quad is canonical: row-0 selector bits
// exactly the block's and none on rows 1-3 (QSEL, staged). Every other selector row is
// evaluated by its own quad's lane (row_gates), so each selector row is evaluated once.
__device__ __forceinline__ void half_g_gates(const Tile& T, EvalAcc& A, const uint32_t* L,
                                             const uint32_t* S, uint64_t tile0, uint32_t lane,
                                             uint32_t kind) {
  if (lane >= 2 * S[GS_NG]) return;
  const uint32_t h = lane & 1u;
  const int off = kind == 0 ? 0 : kind == 1 ? 4 : kind == 2 ? 12 : 16;
  const int rl = (int)S[GS_GT + GT_WORDS * (lane >> 1) + 5] + 28 * (int)h + off;  // selector row
  const uint32_t want = kind == 0 ? 1u << (h ? S_A2 : S_A1)
                      : kind == 1 ? 1u << (h ? S_D2 : S_D1)
                      : kind == 2 ? 1u << (h ? S_C2 : S_C1)
                      : h ? (1u << S_B2) | (1u << S_IJKL) : (1u << S_B1) | (1u << S_EFGH);
  if (rl < 0 || rl >= TILE_ROWS || L[L_QSEL + (rl >> 2)] != want) return;
  const uint32_t r = (uint32_t)rl;
  uint32_t f;
  if (kind == 0 || kind == 2) {
    f = g_add(T, r, L[L_A9 + (r >> 2)], kind == 0) ? 0u : want;
  } else if (kind == 1) {
    f = g_xor(T, r, false) ? 0u : want;
  } else {
    f = h ? g_xor63(T, r, want) : g_xor24(T, r, want);
  }
  if (f) A.fail_gates(tile0 + r, f);
}

// The copy checks of the tile's G's: item it = (G table entry it / 72, check it % 72), spread
// over all threads. A check belongs to this tile if its operand row does; its source is one
// LDS read at (per-G base) + C for every valid layout.
__device__ __forceinline__ void round_copies(EvalAcc& A, const uint32_t* L, const uint32_t* S,
                                             uint64_t tile0, uint32_t tid) {
  const uint32_t nchk = S[GS_NG] * G_CHECKS;
#pragma unroll 2
  for (uint32_t k = 0; k < (MAX_TILE_G * G_CHECKS + BLOCK - 1) / BLOCK; k++) {
    const uint32_t it = tid + k * BLOCK;
    if (it >= nchk) break;
    const uint32_t gi = it / G_CHECKS, ci = it - gi * G_CHECKS;
    const uint32_t* gt = S + GS_GT + GT_WORDS * gi;
    const uint32_t e = L[L_CT + gt[6] + ci];
    const int dl = (int)gt[5] + (int)((e >> 19) & 63u);
    const int src = (int)gt[(e >> 14) & 7u] + (int)(e & 16383u);
    const uint32_t sv = L[src < 0 ? 0 : src];  // < 0 only for checks outside the tile
    const int dlc = dl < 0 ? 0 : (dl >= TILE_ROWS ? TILE_ROWS - 1 : dl);
    const uint32_t dv = L[L_G + (1 + ((e >> 17) & 3u)) * TSTRIDE + dlc];
    if (dl >= 0 && dl < TILE_ROWS && dv != sv) A.fail(tile0 + (uint64_t)dl, B2F_CODE_COPY);
  }
}

// Copy-source lookup, all from LDS for a valid trace: rows inside the window come from W;
// init-region words (h, m, t, fmask, IV, v12..v14) of the tile's first instance, which may
// start before the window, from the init cache I (a_1 | a_2 of its rows 0..163). Anything
// else (only reachable through a corrupted layout) is read from global memory.
struct Src {
  const uint32_t* W;
  const uint32_t* I;
  const uint32_t* adv;
  uint64_t total_rows, wlo, ofirst;
  // wc: source column as W index (a_1 a_2 a_7 a_8 -> 0 1 2 3)
  __device__ __forceinline__ uint32_t at(uint64_t gs, uint32_t wc) const {
    uint64_t d = gs - wlo;  // wraps for gs < wlo
    if (d < (uint64_t)WSTRIDE) return W[wc * WSTRIDE + (uint32_t)d];
    uint64_t e = gs - ofirst;
    if (e < (uint64_t)INIT_ROWS && wc < 2) return I[wc * INIT_ROWS + (uint32_t)e];
    uint32_t col = wc < 2 ? wc + 1 : wc + 5;
    return adv[(uint64_t)col * total_rows + gs];
  }
  __device__ __forceinline__ uint32_t operator()(uint64_t gs, uint32_t col) const {
    return at(gs, col < 3 ? col - 1 : col - 5);
  }
};

__device__ __forceinline__ void copy_check(EvalAcc& A, uint32_t dv, uint32_t sv, uint64_t gd) {
  if (dv != sv) A.fail(gd, B2F_CODE_COPY);
}

// canonical cell of limb k of state word w as half-round hr starts (instance-local row)
__device__ __forceinline__ uint32_t state_src(uint32_t w, uint32_t k, uint32_t spread, uint32_t hr,
                                              uint32_t& col) {
  if (hr == 0) {
    col = spread ? A2 : A1;
    if (w < 8) return 4 * w + k;
    if (w >= 12 && w < 15) return 140 + 8 * (w - 12) + 2 * k;
    return 108 + 4 * (w == 15 ? 7u : w - 8) + k;
  }
  uint32_t hp = hr - 1, role = w >> 2, pos = w & 3;
  uint32_t g = (hp & 1) ? 4 + ((pos - role) & 3u) : pos;
  uint32_t gb = INIT_ROWS + ROUND_ROWS * (hp >> 1) + G_ROWS * g;
  col = role == 1 ? (spread ? A8 : A7) : (spread ? A2 : A1);
  // a <- a2 (+28), b <- b2 (+44, stride 2), c <- c2 (+40), d <- d2 (+32, rot 16)
  uint32_t off = role == 0 ? 28 + k : role == 1 ? 44 + 2 * k : role == 2 ? 40 + k
                                                             : 32 + 2 * ((k + 1) & 3);
  return gb + off;
}

// Copy constraints of the init XOR blocks and of the final XOR3 blocks (57 of the R/4 quads
// of an instance): decoded directly.
__device__ void copies_edge(EvalAcc& A, const uint4* dst, const Src& src, uint64_t o,
                            uint32_t rounds, uint32_t lq) {
  QuadInfo d = decode_quad(lq, rounds);
  const uint32_t r0 = 4 * lq;
  if (d.kind == K_XOR && d.block < INIT_ROWS) {
    // v12 = IV4 ^ t0, v13 = IV5 ^ t1, v14 = IV6 ^ fmask
#pragma unroll
    for (uint32_t h = 0; h < 2; h++) {
      uint32_t k = 2 * d.q + h;
      uint32_t xs = 108 + 4 * (4 + d.a) + k;
      uint32_t ys = (d.a < 2 ? 96 + 4 * d.a : 104) + k;
      uint32_t dx = comp(dst[0], 2 * h), dy = comp(dst[1], 2 * h);
      copy_check(A, dx, src(o + xs, A2), o + r0 + 2 * h);
      copy_check(A, dy, src(o + ys, A2), o + r0 + 2 * h);
    }
  } else if (d.kind == K_XOR3) {
#pragma unroll
    for (uint32_t h = 0; h < 2; h++) {
      uint32_t k = 2 * d.q + h, cv, cu;
      uint32_t vs = state_src(d.a, k, 1, 2 * rounds, cv);
      uint32_t us = state_src(d.a + 8, k, 1, 2 * rounds, cu);
      uint64_t gd = o + r0 + 2 * h;
      copy_check(A, comp(dst[0], 2 * h), src(o + 4 * d.a + k, A2), gd);
      copy_check(A, comp(dst[1], 2 * h), src(o + vs, cv), gd);
      copy_check(A, comp(dst[2], 2 * h), src(o + us, cu), gd);
    }
  }
}

// MODE (diagnostics; the product uses EVAL_FULL): which checks run on a staged tile.
enum { EVAL_LOOKUP = 1, EVAL_GATES = 2, EVAL_COPIES = 4, EVAL_FULL = 7, EVAL_TOUCH = 8 };

// The two extra (non-own-quad) loads a thread issues per tile, as a compact descriptor:
// kind, LDS destination, and a base pointer the tile position is added to.
enum { XK_NONE = 0, XK_HIST, XK_HALO, XK_INIT, XK_INFO, XK_INFO2 };
struct Extra {
  const uint32_t* base;  // HIST/HALO: + tile0 rows; INIT: + off[first]; INFO: + 24 t words
  uint32_t lds;          // LDS word offset of the 16-byte destination
  uint32_t kind;
  uint32_t q;            // HALO: quad index inside the halo
};

__device__ __forceinline__ Extra make_extra(int slot, const uint32_t* adv, uint64_t total_rows,
                                            const TileInfo* tinfo) {
  Extra x;
  x.q = 0;
  if (slot < X_HIST) {
    int ci = slot / (HIST / 4), hq = slot - ci * (HIST / 4);
    int col = ci == 0 ? A1 : ci == 1 ? A2 : ci == 2 ? A7 : A8;
    x.kind = XK_HIST;
    x.base = adv + (uint64_t)col * total_rows - HIST + 4 * hq;
    x.lds = L_W + ci * WSTRIDE + 4 * hq;
  } else if (slot < X_HALO) {
    int e = slot - X_HIST, gi = e >> 2, q = e & 3;
    x.kind = XK_HALO;
    x.q = q;
    x.base = adv + (uint64_t)gi * total_rows + TILE_ROWS + 4 * q;  // gate columns a_0..a_8
    x.lds = lds_cell(gi, TILE_ROWS + 4 * q);
  } else if (slot < X_INIT) {
    int e = slot - X_HALO, ci = e / INIT_QUADS, q = e - ci * INIT_QUADS;
    x.kind = XK_INIT;
    x.base = adv + (uint64_t)(A1 + ci) * total_rows + 4 * q;
    x.lds = L_IC + ci * INIT_ROWS + 4 * q;
  } else if (slot < X_INFO) {
    x.kind = XK_INFO;
    x.base = reinterpret_cast<const uint32_t*>(tinfo) + 4 * (slot - X_INIT);
    x.lds = L_INFO + 4 * (slot - X_INIT);
  } else if (slot < X_INFO2) {
    x.kind = XK_INFO2;
    x.base = reinterpret_cast<const uint32_t*>(tinfo) + 4 * (slot - X_INFO);
    x.lds = L_INFO2 + 4 * (slot - X_INFO);
  } else {
    x.kind = XK_NONE;
    x.base = adv;
    x.lds = 0;
  }
  return x;
}

// fo = {first, -, off[first] lo, hi} of tile t (only INIT slots read it). One predicated
// 16-byte load whatever the slot kind (a switch around the loads serialises their issue).
__device__ __forceinline__ uint4 extra_load(const Extra& x, uint64_t t, const uint4& fo, uint32_t n,
                                            uint64_t total_rows, uint64_t total_quads,
                                            uint64_t G, uint64_t n_tiles) {
  const uint64_t tile0 = t * TILE_ROWS;
  const uint64_t of = ((uint64_t)fo.w << 32) | fo.z;
  const uint32_t k = x.kind;
  const uint64_t w = k == XK_INIT ? of : k == XK_INFO ? 24 * t : k == XK_INFO2 ? 24 * (t + G) : tile0;
  const bool ok = k == XK_HIST    ? tile0 >= (uint64_t)HIST
                : k == XK_HALO    ? (t + 1) * BLOCK + x.q < total_quads
                : k == XK_INIT    ? fo.x < n && of + INIT_ROWS <= total_rows
                : k == XK_INFO    ? true
                : k == XK_INFO2   ? t + G < n_tiles
                                  : false;
  return ok ? *reinterpret_cast<const uint4*>(x.base + w) : make_uint4(0, 0, 0, 0);
}

template <int MODE>
#ifndef B2F_EVAL_WAVES
#define B2F_EVAL_WAVES 3  // waves per SIMD the eval kernel is compiled for (LDS allows 3 WGs/CU)
#endif
__global__ void __launch_bounds__(BLOCK, B2F_EVAL_WAVES) eval_kernel(const uint32_t* __restrict__ adv,
                                                    const uint32_t* __restrict__ fixed,
                                                    const uint64_t* __restrict__ off, uint32_t n,
                                                    uint64_t total_rows,
                                                    const TileInfo* __restrict__ tinfo,
                                                    uint64_t n_tiles,
                                                    b2f_eval_report* __restrict__ rep,
                                                    int* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) uint32_t L[LDS_WORDS];
  const int tid = threadIdx.x;
  for (int i = tid; i < CHECK_WORDS; i += BLOCK)
    L[L_CT + i] = reinterpret_cast<const uint32_t*>(&c_checks)[i];
  if (tid < 40) L[L_SG + tid] = reinterpret_cast<const uint32_t*>(c_sigma)[tid];
  if (tid < 16) L[L_XS + tid] = expected_sel((uint32_t)tid);
  const Tile T{L};
  const uint8_t* Sg = reinterpret_cast<const uint8_t*>(L + L_SG);  // [10][16]

  EvalAcc A{L + L_ACC};
  if (tid < 20) L[L_ACC + tid] = 0;
  if (tid == 20) *reinterpret_cast<uint64_t*>(L + L_ACC + 20) = ~0ull;

  const uint64_t total_quads = total_rows >> 2;
  const uint64_t used_rows = off[n];
  const bool layout_ok = used_rows <= total_rows && off[0] == 0;  // never read past the trace
  if (!layout_ok && blockIdx.x == 0 && tid == 0) atomicOr(status, 1 << B2F_ERR_LAYOUT);
  const uint64_t G = gridDim.x;

  // XCD-aware deal: workgroups are dispatched to the 8 XCDs round-robin (b % 8), so give each
  // XCD a contiguous run of G / 8 tiles per band. A tile's history window and halo are then the
  // rows its same-XCD neighbours just loaded, served from that XCD's L2 rather than refetched
  // (placement is only a speed hint; any placement gives the same result).
  uint64_t t = (G % 8 == 0) ? (blockIdx.x % 8) * (G / 8) + blockIdx.x / 8 : blockIdx.x;
  // fo / fo_next (first instance and its offset, per tile) are workgroup-uniform: SGPRs
  uint4 q[NCOL_T], x0 = make_uint4(0, 0, 0, 0), x1 = x0, fo = x0, fo_next = x0;
  const Extra e0 = make_extra(tid, adv, total_rows, tinfo);
  const Extra e1 = make_extra(tid + BLOCK, adv, total_rows, tinfo);
  auto load_tile = [&](uint64_t tt, const uint4& f) {
    const uint64_t gq = tt * BLOCK + tid;
#pragma unroll
    for (int c = 0; c < NCOL_T; c++)
      q[c] = gq < total_quads
                 ? *reinterpret_cast<const uint4*>((c < 10 ? adv + (uint64_t)c * total_rows : fixed) + 4 * gq)
                 : make_uint4(0, 0, 0, 0);
    x0 = extra_load(e0, tt, f, n, total_rows, total_quads, G, n_tiles);
    x1 = extra_load(e1, tt, f, n, total_rows, total_quads, G, n_tiles);
  };
  if (layout_ok && t < n_tiles) {
    fo = *reinterpret_cast<const uint4*>(tinfo + t);
    load_tile(t, fo);
    if (t + G < n_tiles) fo_next = *reinterpret_cast<const uint4*>(tinfo + t + G);
  }
  for (uint32_t iter = 0; layout_ok && t < n_tiles; t += G, iter++) {
    // ---- stage tile t: registers -> LDS
#pragma unroll
    for (int c = 0; c < 9; c++) *reinterpret_cast<uint4*>(&L[lds_cell(c, 4 * tid)]) = q[c];
    const uint4 cur9 = q[A9], curfx = q[10];
    if (MODE & (EVAL_GATES | EVAL_COPIES)) {
      L[L_QSEL + tid] = (curfx.x & 0xffffu) | (((curfx.y | curfx.z | curfx.w) & 0xffffu) ? 1u << 16 : 0u);
      L[L_A9 + tid] = cur9.x;
    }
    if (e0.kind != XK_NONE) *reinterpret_cast<uint4*>(&L[e0.lds]) = x0;
    if (e1.kind != XK_NONE) *reinterpret_cast<uint4*>(&L[e1.lds]) = x1;
    __syncthreads();
    // ---- prefetch tile t + G into registers while tile t is checked
    const uint64_t tn = t + G;
    if (tn < n_tiles) {
      load_tile(tn, fo_next);
      if (tn + G < n_tiles) fo_next = *reinterpret_cast<const uint4*>(tinfo + tn + G);
    }
    const uint64_t tile0 = t * TILE_ROWS;
    const uint64_t gq = t * BLOCK + tid;
    const uint64_t row0 = 4 * gq;
    const uint32_t lr0 = 4 * tid;
    if ((MODE & EVAL_TOUCH) && gq < total_quads) {  // diagnostics: keep the staged words alive
      uint4 a = T.quad(A0, 4 * tid), b = T.quad(A8, 4 * tid);
      uint32_t x = a.x ^ b.w ^ cur9.x ^ curfx.y ^ L[L_W + 4 * tid] ^ L[L_IC + (tid & 255)] ^
                   L[L_INFO + (tid & 15)] ^ T.at(A3, 4 * tid + 13);
      if (x == 0x12345678u) A.fail(0, B2F_CODE_LOOKUP);
    }
    // ---- lookups on the 4 rows (before the G table barrier: they need only the staged tile)
    if ((MODE & EVAL_LOOKUP) && gq < total_quads) {
      const uint4 q0 = T.quad(A0, lr0), q1 = T.quad(A1, lr0), q2 = T.quad(A2, lr0);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        uint32_t tg = comp(q0, j), de = comp(q1, j), sp = comp(q2, j);
        bool ok = de < 65536u && tg == tag16(de) && sp == spread16(de & 0xffffu);
        if (!ok) A.fail(row0 + j, B2F_CODE_LOOKUP);
      }
    }
    if (MODE & (EVAL_GATES | EVAL_COPIES)) {
      // ---- G tables: the first wave builds the next tile's (from INFO2) while this tile is
      // checked with the one built during the previous iteration
      const uint32_t* S = L + L_GS + (iter & 1) * GSET;
      uint32_t* Sn = L + L_GS + ((iter + 1) & 1) * GSET;
      if (iter == 0) {  // nothing was built ahead for the first tile
        if (tid < 64) build_g_table(L + L_GS, L + L_INFO, Sg, tile0, n, total_rows, (uint32_t)tid);
        __syncthreads();
      }
      if (tid < 64) build_g_table(Sn, L + L_INFO2, Sg, (t + G) * TILE_ROWS, t + G < n_tiles ? n : 0,
                                  total_rows, (uint32_t)tid);
      if (MODE & EVAL_GATES) half_g_gates(T, A, L, S, tile0, (uint32_t)tid & 63u, (uint32_t)tid >> 6);
      if (MODE & EVAL_COPIES) round_copies(A, L, S, tile0, (uint32_t)tid);
      // ---- per quad: selector rows the G pass does not take, and init/final-block copies
      if (gq < total_quads) {
        const uint32_t pq = reinterpret_cast<const uint8_t*>(S + GS_QM)[tid];
        const bool in_g = pq != 0xffu;
        if (MODE & EVAL_GATES) {
          const uint32_t rest = (curfx.y | curfx.z | curfx.w) & 0xffffu;
          const bool regular = in_g && rest == 0 && (curfx.x & 0xffffu) == L[L_XS + (pq & 15u)];
          if (!regular) {
            uint32_t rowmask = ((curfx.x & 0xffffu) ? 1u : 0u) | ((curfx.y & 0xffffu) ? 2u : 0u) |
                               ((curfx.z & 0xffffu) ? 4u : 0u) | ((curfx.w & 0xffffu) ? 8u : 0u);
            while (rowmask) {
              int j = __builtin_ctz(rowmask);
              rowmask &= rowmask - 1;
              uint32_t k0 = comp(curfx, j);
              uint32_t failed;
              if ((k0 & 0xffffu) == (1u << S_CONST)) failed = T.at(A1, lr0 + j) == (k0 >> 16) ? 0u : 1u << S_CONST;
              else failed = row_gates(T, k0 & 0xffffu, lr0 + j, comp(cur9, j), k0);
              if (failed) A.fail_gates(row0 + j, failed);
            }
          }
        }
        if ((MODE & EVAL_COPIES) && !in_g && row0 < used_rows) {
          // the quad's instance: scan the tile's cached offsets (a valid layout never needs
          // more; offsets_check_kernel flags any other)
          const uint32_t first = L[L_INFO];
          const uint64_t* Off = reinterpret_cast<const uint64_t*>(L + L_INFO + 2);
          uint32_t i = 0;
          while (i + 2 < NOFF && Off[i + 1] <= row0) i++;
          const uint64_t o = Off[i], o1 = Off[i + 1];
          const uint64_t R = o1 - o;
          if (first + i < n && o1 > row0 && o1 <= total_rows && R >= FIXED_ROWS &&
              R <= MAX_INSTANCE_ROWS && ((uint32_t)R - FIXED_ROWS) % ROUND_ROWS == 0) {
            const uint32_t rounds = ((uint32_t)R - FIXED_ROWS) / ROUND_ROWS;
            const uint64_t ofirst = first < n ? Off[0] : ~0ull;
            const Src src{L + L_W, L + L_IC, adv, total_rows, tile0 - HIST, ofirst};
            const uint4 dq[3] = {T.quad(A3, lr0), T.quad(A4, lr0), T.quad(A5, lr0)};
            copies_edge(A, dq, src, o, rounds, (uint32_t)((row0 - o) >> 2));
          }
        }
      }
    }
    __syncthreads();
  }
  // ---- flush the workgroup's counters: one global atomic per non-zero counter
  __syncthreads();
  if (tid < 18) {
    uint32_t v = L[L_ACC + tid];
    if (v) {
      unsigned long long* dst = tid < 16 ? (unsigned long long*)&rep->gate_failures[tid]
                                         : tid == 16 ? (unsigned long long*)&rep->lookup_failures
                                                     : (unsigned long long*)&rep->copy_failures;
      atomicAdd(dst, (unsigned long long)v);
    }
  } else if (tid == 18) {
    uint64_t fm = *reinterpret_cast<const uint64_t*>(L + L_ACC + 20);
    if (fm != ~0ull) atomicMin((unsigned long long*)&rep->first_failure, (unsigned long long)fm);
  }
}

// Device-side layout validation for b2f_eval_dev: every instance's rows must be R(rounds) for
// some rounds and lie inside the trace. The eval kernel relies on it (an invalid layout is an
// error whatever the counters say; it only has to stay in bounds).
__global__ void offsets_check_kernel(const uint64_t* __restrict__ off, uint32_t n,
                                     uint64_t total_rows, int* __restrict__ status) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t o = off[i], o1 = off[i + 1], R = o1 - o;
  const bool bad = o1 < o || o1 > total_rows || (i == 0 && o != 0) || R < FIXED_ROWS ||
                   R > MAX_INSTANCE_ROWS || ((uint32_t)R - FIXED_ROWS) % ROUND_ROWS != 0;
  if (bad) atomicOr(status, 1 << B2F_ERR_LAYOUT);
}

__global__ void report_init_kernel(b2f_eval_report* rep, uint64_t total_rows) {
  for (int s = 0; s < B2F_NUM_GATES; s++) rep->gate_failures[s] = 0;
  rep->lookup_failures = 0;
  rep->copy_failures = 0;
  rep->first_failure = ~0ull;
  rep->rows_checked = total_rows;
}

}  // namespace

// ============================================================================ host / C ABI

struct b2f_ctx {
  int device;
  char err[512];
  int* d_status;       // [0] fill, [1] eval
  uint64_t* d_rec;     // half-round states
  uint64_t rec_cap;    // in states (16 x u64 each)
  TileInfo* d_tiles;   // per-tile instance context
  uint64_t tiles_cap;
  int timing;
  std::vector<hipEvent_t> pool;  // event pairs, reused after every b2f_kernel_times
  std::vector<int> kinds;        // kernel kind of pair i
  int cu_count;
};

namespace {

int set_err(b2f_ctx* ctx, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int set_err(b2f_ctx* ctx, int code, const char* fmt, ...) {
  if (ctx) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(ctx->err, sizeof ctx->err, fmt, ap);
    va_end(ap);
  }
  return code;
}

#define HIPCHK(ctx, expr)                                                              \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return set_err(ctx, B2F_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_));        \
  } while (0)

// Record the start event of a timed launch; returns the pair index or -1.
int timed_begin(b2f_ctx* ctx, int kind, hipStream_t s) {
  if (!ctx->timing) return -1;
  size_t i = ctx->kinds.size();
  while (ctx->pool.size() < 2 * (i + 1)) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return -1;
    ctx->pool.push_back(e);
  }
  if (hipEventRecord(ctx->pool[2 * i], s) != hipSuccess) return -1;
  ctx->kinds.push_back(kind);
  return (int)i;
}
void timed_end(b2f_ctx* ctx, int i, hipStream_t s) {
  if (i >= 0) (void)hipEventRecord(ctx->pool[2 * i + 1], s);
}

// Diagnostic kernel variants for ablation runs (B2F_DIAG_FILL / B2F_DIAG_EVAL); unset in
// every product run, where the full kernels launch.
int diag_mode(const char* var, int full) {
  const char* v = getenv(var);
  return v ? atoi(v) : full;
}

uint64_t layout_rows(uint32_t rounds) {
  if (rounds > B2F_MAX_ROUNDS) return 0;
  return (uint64_t)FIXED_ROWS + (uint64_t)ROUND_ROWS * rounds;
}

uint64_t n_tiles_of(uint64_t total_rows) { return (total_rows + TILE_ROWS - 1) / TILE_ROWS; }

uint32_t grid_for(const b2f_ctx* ctx, uint64_t n_tiles, int wgs_per_cu) {
  uint64_t m = (uint64_t)ctx->cu_count * wgs_per_cu;
  uint64_t g = n_tiles < m ? n_tiles : m;
  return (uint32_t)(g ? g : 1);
}

// per-tile instance context for this call's offsets (scratch owned by the context)
int launch_tile_index(b2f_ctx* ctx, const uint64_t* d_offsets, size_t n, uint64_t n_tiles,
                      hipStream_t s) {
  if (n_tiles > ctx->tiles_cap) {
    HIPCHK(ctx, hipStreamSynchronize(s));
    if (ctx->d_tiles) HIPCHK(ctx, hipFree(ctx->d_tiles));
    ctx->d_tiles = nullptr;
    ctx->tiles_cap = 0;
    HIPCHK(ctx, hipMalloc(&ctx->d_tiles, n_tiles * sizeof(TileInfo)));
    ctx->tiles_cap = n_tiles;
  }
  hipLaunchKernelGGL(tile_info_kernel, dim3((uint32_t)((n_tiles + 255) / 256)), dim3(256), 0, s,
                     d_offsets, (uint32_t)n, n_tiles, ctx->d_tiles);
  HIPCHK(ctx, hipGetLastError());
  return B2F_OK;
}

}  // namespace

extern "C" {

B2F_API int b2f_version(void) { return 1; }

B2F_API uint64_t b2f_layout_rows(uint32_t rounds) { return layout_rows(rounds); }

B2F_API int b2f_layout_offsets(const b2f_input* in, size_t n, uint64_t* offsets) {
  if ((!in && n) || !offsets) return B2F_ERR_ARG;
  offsets[0] = 0;
  for (size_t i = 0; i < n; i++) {
    uint64_t R = layout_rows(in[i].rounds);
    if (!R) return B2F_ERR_ROUNDS;
    offsets[i + 1] = offsets[i] + R;
  }
  return B2F_OK;
}

B2F_API int b2f_halo2_column_index(int a) {
  static const int idx[10] = {7, 8, 9, 1, 2, 0, 3, 4, 5, 6};
  return (a >= 0 && a < 10) ? idx[a] : -1;
}

B2F_API int b2f_parse_eip152(const uint8_t* raw, size_t len, b2f_input* out) {
  if (!raw || !out) return B2F_ERR_ARG;
  if (len != 213) return B2F_ERR_INPUT;
  auto le64 = [](const uint8_t* p) {
    uint64_t v = 0;
    for (int k = 7; k >= 0; k--) v = (v << 8) | p[k];
    return v;
  };
  if (raw[212] > 1) return B2F_ERR_INPUT;
  b2f_input x;
  x.rounds = ((uint32_t)raw[0] << 24) | ((uint32_t)raw[1] << 16) | ((uint32_t)raw[2] << 8) | raw[3];
  for (int k = 0; k < 8; k++) x.h[k] = le64(raw + 4 + 8 * k);
  for (int k = 0; k < 16; k++) x.m[k] = le64(raw + 68 + 8 * k);
  x.t[0] = le64(raw + 196);
  x.t[1] = le64(raw + 204);
  x.f = raw[212];
  *out = x;
  return B2F_OK;
}

B2F_API b2f_ctx* b2f_create(int device) {
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  b2f_ctx* ctx = new (std::nothrow) b2f_ctx();
  if (!ctx) return nullptr;
  ctx->device = device;
  ctx->err[0] = 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) { delete ctx; return nullptr; }
  ctx->cu_count = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  if (hipMalloc(&ctx->d_status, 4 * sizeof(int)) != hipSuccess) { delete ctx; return nullptr; }
  if (hipMemset(ctx->d_status, 0, 4 * sizeof(int)) != hipSuccess) { delete ctx; return nullptr; }
  return ctx;
}

B2F_API void b2f_destroy(b2f_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipFree(ctx->d_status);
  (void)hipFree(ctx->d_rec);
  (void)hipFree(ctx->d_tiles);
  for (hipEvent_t e : ctx->pool) (void)hipEventDestroy(e);
  delete ctx;
}

B2F_API const char* b2f_last_error(const b2f_ctx* ctx) { return ctx ? ctx->err : "null context"; }

B2F_API int b2f_set_timing(b2f_ctx* ctx, int enable) {
  if (!ctx) return B2F_ERR_ARG;
  ctx->timing = enable ? 1 : 0;
  ctx->kinds.clear();
  return B2F_OK;
}

B2F_API int b2f_kernel_times(b2f_ctx* ctx, double* total_ms, uint32_t* count) {
  if (!ctx || !total_ms || !count) return B2F_ERR_ARG;
  for (int k = 0; k < B2F_NUM_KERNELS; k++) { total_ms[k] = 0; count[k] = 0; }
  for (size_t i = 0; i < ctx->kinds.size(); i++) {
    HIPCHK(ctx, hipEventSynchronize(ctx->pool[2 * i + 1]));
    float t = 0;
    HIPCHK(ctx, hipEventElapsedTime(&t, ctx->pool[2 * i], ctx->pool[2 * i + 1]));
    total_ms[ctx->kinds[i]] += t;
    count[ctx->kinds[i]] += 1;
  }
  ctx->kinds.clear();
  return B2F_OK;
}

B2F_API int b2f_fill_dev(b2f_ctx* ctx, const b2f_input* d_in, size_t n, const uint64_t* d_offsets,
                         uint64_t total_rows, uint32_t* d_advice, uint32_t* d_fixed,
                         uint64_t* d_h_out, void* stream) {
  if (!ctx) return B2F_ERR_ARG;
  if (!d_in || !d_offsets || !d_advice || !d_fixed || n == 0)
    return set_err(ctx, B2F_ERR_ARG, "fill: null buffer or empty batch");
  if (n > 0xffffffffull) return set_err(ctx, B2F_ERR_ARG, "fill: more than 2^32 instances");
  if (total_rows % 4) return set_err(ctx, B2F_ERR_ARG, "fill: total_rows %% 4 != 0");
  if (((uintptr_t)d_advice | (uintptr_t)d_fixed | (uintptr_t)d_in) & 15)
    return set_err(ctx, B2F_ERR_ARG, "fill: buffers must be 16-byte aligned");
  if (total_rows < (uint64_t)FIXED_ROWS * n)
    return set_err(ctx, B2F_ERR_ROWS, "fill: %llu rows cannot hold %zu instances",
                   (unsigned long long)total_rows, n);
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  // states = 2*sum(rounds) + n  <=  2*(total_rows - 228 n)/416 + n
  uint64_t states = 2 * ((total_rows - (uint64_t)FIXED_ROWS * n) / ROUND_ROWS) + n;
  if (states > ctx->rec_cap) {
    HIPCHK(ctx, hipStreamSynchronize(s));
    if (ctx->d_rec) HIPCHK(ctx, hipFree(ctx->d_rec));
    ctx->d_rec = nullptr;
    ctx->rec_cap = 0;
    HIPCHK(ctx, hipMalloc(&ctx->d_rec, states * 16 * sizeof(uint64_t)));
    ctx->rec_cap = states;
  }
  HIPCHK(ctx, hipMemsetAsync(ctx->d_status, 0, sizeof(int), s));
  uint32_t nn = (uint32_t)n;
  int tk = timed_begin(ctx, B2F_KERNEL_RECORD, s);
  hipLaunchKernelGGL(record_kernel, dim3((nn + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, d_in, nn,
                     d_offsets, total_rows, ctx->rec_cap, ctx->d_rec, d_h_out, ctx->d_status);
  HIPCHK(ctx, hipGetLastError());
  timed_end(ctx, tk, s);
  uint64_t nt = n_tiles_of(total_rows);
  int rc = launch_tile_index(ctx, d_offsets, n, nt, s);
  if (rc) return rc;
  uint32_t wgs = grid_for(ctx, nt, 8);
  tk = timed_begin(ctx, B2F_KERNEL_FILL, s);
  switch (diag_mode("B2F_DIAG_FILL", FILL_FULL)) {
#define B2F_FILL(M)                                                                            \
  case M:                                                                                      \
    hipLaunchKernelGGL(fill_kernel<M>, dim3(wgs), dim3(BLOCK), 0, s, d_in, nn, d_offsets,      \
                       total_rows, ctx->d_rec, d_advice, d_fixed, ctx->d_status, ctx->d_tiles, \
                       nt);                                                                    \
    break;
    B2F_FILL(0) B2F_FILL(1) B2F_FILL(2) default: B2F_FILL(3)
#undef B2F_FILL
  }
  HIPCHK(ctx, hipGetLastError());
  timed_end(ctx, tk, s);
  return B2F_OK;
}

B2F_API int b2f_eval_dev(b2f_ctx* ctx, const uint32_t* d_advice, const uint32_t* d_fixed,
                         const uint64_t* d_offsets, size_t n, uint64_t total_rows,
                         b2f_eval_report* d_report, void* stream) {
  if (!ctx) return B2F_ERR_ARG;
  if (!d_advice || !d_fixed || !d_offsets || !d_report || n == 0)
    return set_err(ctx, B2F_ERR_ARG, "eval: null buffer or empty batch");
  if (n > 0xffffffffull) return set_err(ctx, B2F_ERR_ARG, "eval: more than 2^32 instances");
  if (total_rows % 4) return set_err(ctx, B2F_ERR_ARG, "eval: total_rows %% 4 != 0");
  if (((uintptr_t)d_advice | (uintptr_t)d_fixed) & 15)
    return set_err(ctx, B2F_ERR_ARG, "eval: buffers must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipMemsetAsync(ctx->d_status + 1, 0, sizeof(int), s));
  hipLaunchKernelGGL(report_init_kernel, dim3(1), dim3(1), 0, s, d_report, total_rows);
  HIPCHK(ctx, hipGetLastError());
  hipLaunchKernelGGL(offsets_check_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s,
                     d_offsets, (uint32_t)n, total_rows, ctx->d_status + 1);
  HIPCHK(ctx, hipGetLastError());
  uint64_t nt = n_tiles_of(total_rows);
  int rc = launch_tile_index(ctx, d_offsets, n, nt, s);
  if (rc) return rc;
  uint32_t wgs = grid_for(ctx, nt, 3);
  int tk = timed_begin(ctx, B2F_KERNEL_EVAL, s);
  switch (diag_mode("B2F_DIAG_EVAL", EVAL_FULL)) {
#define B2F_EVAL(M)                                                                             \
  case M:                                                                                       \
    hipLaunchKernelGGL(eval_kernel<M>, dim3(wgs), dim3(BLOCK), 0, s, d_advice, d_fixed,         \
                       d_offsets, (uint32_t)n, total_rows, ctx->d_tiles, nt, d_report,          \
                       ctx->d_status + 1);                                                      \
    break;
    B2F_EVAL(1) B2F_EVAL(2) B2F_EVAL(3) B2F_EVAL(4) B2F_EVAL(5) B2F_EVAL(6) B2F_EVAL(8)
    default: B2F_EVAL(7)
#undef B2F_EVAL
  }
  HIPCHK(ctx, hipGetLastError());
  timed_end(ctx, tk, s);
  return B2F_OK;
}

B2F_API int b2f_export_fp_dev(b2f_ctx* ctx, const uint32_t* d_advice, uint64_t total_rows,
                              uint64_t row_begin, uint64_t nrows, uint32_t form,
                              uint64_t* d_out, uint64_t out_rows, void* stream) {
  if (!ctx) return B2F_ERR_ARG;
  if (!d_advice || !d_out) return set_err(ctx, B2F_ERR_ARG, "export: null buffer");
  if (form != B2F_FP_CANONICAL && form != B2F_FP_MONTGOMERY)
    return set_err(ctx, B2F_ERR_ARG, "export: unknown form %u", form);
  if ((uintptr_t)d_out & 15) return set_err(ctx, B2F_ERR_ARG, "export: d_out must be 16-byte aligned");
  if (row_begin > total_rows || nrows > total_rows - row_begin)
    return set_err(ctx, B2F_ERR_ROWS, "export: rows [%llu, +%llu) exceed total_rows %llu",
                   (unsigned long long)row_begin, (unsigned long long)nrows,
                   (unsigned long long)total_rows);
  if (out_rows < nrows) return set_err(ctx, B2F_ERR_ROWS, "export: out_rows < nrows");
  if (nrows == 0) return B2F_OK;
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  int tk = timed_begin(ctx, B2F_KERNEL_EXPORT, s);
  HIPCHK(ctx, launch_export_fp(d_advice, total_rows, row_begin, nrows, form, d_out, out_rows,
                               ctx->cu_count, s));
  timed_end(ctx, tk, s);
  return B2F_OK;
}

B2F_API int b2f_sync(b2f_ctx* ctx, void* stream) {
  if (!ctx) return B2F_ERR_ARG;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipStreamSynchronize((hipStream_t)stream));
  int st[2] = {0, 0};
  HIPCHK(ctx, hipMemcpy(st, ctx->d_status, sizeof st, hipMemcpyDeviceToHost));
  HIPCHK(ctx, hipMemset(ctx->d_status, 0, sizeof st));
  int bits = st[0] | st[1];
  if (bits & (1 << B2F_ERR_ROUNDS)) return set_err(ctx, B2F_ERR_ROUNDS, "rounds > %u", B2F_MAX_ROUNDS);
  if (bits & (1 << B2F_ERR_LAYOUT))
    return set_err(ctx, B2F_ERR_LAYOUT, "row offsets are not the LAYOUT v1 prefix sums");
  return B2F_OK;
}

B2F_API int b2f_fill(b2f_ctx* ctx, const b2f_input* in, size_t n, uint32_t* advice,
                     uint32_t* fixed, uint64_t* h_out) {
  if (!ctx) return B2F_ERR_ARG;
  if (!in || !advice || !fixed || n == 0) return set_err(ctx, B2F_ERR_ARG, "fill: null buffer");
  std::vector<uint64_t> off(n + 1);
  int rc = b2f_layout_offsets(in, n, off.data());
  if (rc) return set_err(ctx, rc, "fill: rounds > %u", B2F_MAX_ROUNDS);
  uint64_t total = off[n];
  HIPCHK(ctx, hipSetDevice(ctx->device));
  b2f_input* d_in = nullptr; uint64_t* d_off = nullptr; uint32_t* d_adv = nullptr;
  uint32_t* d_fx = nullptr; uint64_t* d_h = nullptr;
  int ret = B2F_OK;
  do {
    if (hipMalloc(&d_in, n * sizeof(b2f_input)) || hipMalloc(&d_off, (n + 1) * 8) ||
        hipMalloc(&d_adv, 10 * total * 4) || hipMalloc(&d_fx, total * 4) || hipMalloc(&d_h, n * 64)) {
      ret = set_err(ctx, B2F_ERR_HIP, "fill: device allocation failed");
      break;
    }
    if (hipMemcpy(d_in, in, n * sizeof(b2f_input), hipMemcpyHostToDevice) ||
        hipMemcpy(d_off, off.data(), (n + 1) * 8, hipMemcpyHostToDevice)) {
      ret = set_err(ctx, B2F_ERR_HIP, "fill: upload failed");
      break;
    }
    ret = b2f_fill_dev(ctx, d_in, n, d_off, total, d_adv, d_fx, d_h, nullptr);
    if (ret) break;
    ret = b2f_sync(ctx, nullptr);
    if (ret) break;
    if (hipMemcpy(advice, d_adv, 10 * total * 4, hipMemcpyDeviceToHost) ||
        hipMemcpy(fixed, d_fx, total * 4, hipMemcpyDeviceToHost) ||
        (h_out && hipMemcpy(h_out, d_h, n * 64, hipMemcpyDeviceToHost))) {
      ret = set_err(ctx, B2F_ERR_HIP, "fill: download failed");
      break;
    }
  } while (0);
  (void)hipFree(d_in); (void)hipFree(d_off); (void)hipFree(d_adv); (void)hipFree(d_fx); (void)hipFree(d_h);
  return ret;
}

B2F_API int b2f_eval(b2f_ctx* ctx, const uint32_t* advice, const uint32_t* fixed,
                     const uint64_t* offsets, size_t n, uint64_t total_rows,
                     b2f_eval_report* report) {
  if (!ctx) return B2F_ERR_ARG;
  if (!advice || !fixed || !offsets || !report || n == 0)
    return set_err(ctx, B2F_ERR_ARG, "eval: null buffer");
  if (total_rows % 4) return set_err(ctx, B2F_ERR_ARG, "eval: total_rows %% 4 != 0");
  for (size_t i = 0; i < n; i++) {
    uint64_t R = offsets[i + 1] - offsets[i];
    if (offsets[i + 1] < offsets[i] || R < FIXED_ROWS || (R - FIXED_ROWS) % ROUND_ROWS)
      return set_err(ctx, B2F_ERR_LAYOUT, "eval: instance %zu has %llu rows", i, (unsigned long long)R);
  }
  if (offsets[0] != 0 || offsets[n] > total_rows)
    return set_err(ctx, B2F_ERR_ROWS, "eval: offsets exceed total_rows");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  uint32_t* d_adv = nullptr; uint32_t* d_fx = nullptr; uint64_t* d_off = nullptr;
  b2f_eval_report* d_rep = nullptr;
  int ret = B2F_OK;
  do {
    if (hipMalloc(&d_adv, 10 * total_rows * 4) || hipMalloc(&d_fx, total_rows * 4) ||
        hipMalloc(&d_off, (n + 1) * 8) || hipMalloc(&d_rep, sizeof(b2f_eval_report))) {
      ret = set_err(ctx, B2F_ERR_HIP, "eval: device allocation failed");
      break;
    }
    if (hipMemcpy(d_adv, advice, 10 * total_rows * 4, hipMemcpyHostToDevice) ||
        hipMemcpy(d_fx, fixed, total_rows * 4, hipMemcpyHostToDevice) ||
        hipMemcpy(d_off, offsets, (n + 1) * 8, hipMemcpyHostToDevice)) {
      ret = set_err(ctx, B2F_ERR_HIP, "eval: upload failed");
      break;
    }
    ret = b2f_eval_dev(ctx, d_adv, d_fx, d_off, n, total_rows, d_rep, nullptr);
    if (ret) break;
    ret = b2f_sync(ctx, nullptr);
    if (ret) break;
    if (hipMemcpy(report, d_rep, sizeof *report, hipMemcpyDeviceToHost)) {
      ret = set_err(ctx, B2F_ERR_HIP, "eval: download failed");
      break;
    }
  } while (0);
  (void)hipFree(d_adv); (void)hipFree(d_fx); (void)hipFree(d_off); (void)hipFree(d_rep);
  return ret;
}

}  // extern "C"

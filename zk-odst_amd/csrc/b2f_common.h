// b2f_common.h -- device code shared by the fill/eval kernels (b2f_kernels.hip) and the fused
// fill+eval kernel (b2f_fused.hip): constants, the quad builders of the fill, the per-tile
// instance context, the copy-check tables and the gate evaluators. Product code; it does not
// include or link anything under oracle/. Trace contract: docs/LAYOUT.md.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/b2f.h"
#include "b2f_layout.h"

using namespace b2f;

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
  uint32_t slot[G_QUADS];  // per-quad operand slots (make_slots)
};
constexpr int ROW_TABLE_WORDS = G_QUADS * 5;
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
  // Operand slots: the (at most two) rows of a quad whose a_3/a_4 hold spread operand limbs
  // (XOR, XOR24, XOR63 blocks), with their limb, so a quad needs six operand spreads instead of
  // three per row. bits 0-1 row A, 2-3 limb A, 4 A used, 5-6 row B, 7-8 limb B, 9 B used,
  // 10 a7/a8 = W limb / spread at the slot rows, 11 a6 = Z limb >> 15 at the slot rows,
  // 12 dense a3/a4 (ADD: limb j on row j), 13 a5 = M limb (ADD3).
  for (uint32_t p = 0; p < G_QUADS; p++) {
    const uint32_t st = step_of_quad(p), q = p - first_quad[st];
    uint32_t d = 0;
    if (st % 2 == 0) {
      d = (1u << 12) | ((st == 0 || st == 4) ? 1u << 13 : 0u);
    } else if (st == 3) {  // XOR24: rows R = 4q + j with R % 3 == 0, limb R / 3
      d = q == 0 ? (0u | (0u << 2) | (1u << 4) | (3u << 5) | (1u << 7) | (1u << 9))
        : q == 1 ? (2u | (2u << 2) | (1u << 4))
                 : (1u | (3u << 2) | (1u << 4));
      d |= 1u << 10;
    } else {  // XOR / XOR63: rows 0 and 2, limbs 2q and 2q + 1
      d = 0u | ((2 * q) << 2) | (1u << 4) | (2u << 5) | ((2 * q + 1) << 7) | (1u << 9);
      if (st == 7) d |= (1u << 10) | (1u << 11);
    }
    T.slot[p] = d;
  }
  return T;
}
__constant__ __attribute__((aligned(16))) RowTable c_rows = make_rows();

// `rows`: the RowTable staged in LDS (ROW_TABLE_WORDS words).
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
  // operand slots A and B: limbs of X, Y, W, Z and the spreads of the first three
  const uint32_t sd = rows[4 * G_QUADS + p];
  const uint32_t jA = sd & 3u, shA = 16 * ((sd >> 2) & 3u), jB = (sd >> 5) & 3u, shB = 16 * ((sd >> 7) & 3u);
  const bool vA = (sd >> 4) & 1u, vB = (sd >> 9) & 1u, has_w = (sd >> 10) & 1u, has_z = (sd >> 11) & 1u;
  const bool dense = (sd >> 12) & 1u, has_m = (sd >> 13) & 1u;
  const uint32_t xA = (uint32_t)(X >> shA) & 0xffffu, yA = (uint32_t)(Y >> shA) & 0xffffu;
  const uint32_t xB = (uint32_t)(X >> shB) & 0xffffu, yB = (uint32_t)(Y >> shB) & 0xffffu;
  const uint32_t wA = (uint32_t)(W >> shA) & 0xffffu, wB = (uint32_t)(W >> shB) & 0xffffu;
  const uint32_t zA = ((uint32_t)(Z >> shA) & 0xffffu) >> 15, zB = ((uint32_t)(Z >> shB) & 0xffffu) >> 15;
  const uint32_t sxA = spread16(xA), syA = spread16(yA), swA = spread16(wA);
  const uint32_t sxB = spread16(xB), syB = spread16(yB), swB = spread16(wB);
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
    const bool isA = vA && jA == (uint32_t)j, isB = vB && jB == (uint32_t)j;
    Q.c[A3][j] = dense ? (uint32_t)(X >> (16 * j)) & 0xffffu : isA ? sxA : isB ? sxB : 0u;
    Q.c[A4][j] = dense ? (uint32_t)(Y >> (16 * j)) & 0xffffu : isA ? syA : isB ? syB : 0u;
    Q.c[A5][j] = has_m ? (uint32_t)(M >> (16 * j)) & 0xffffu : 0u;
    Q.c[A6][j] = has_z ? (isA ? zA : isB ? zB : 0u) : 0u;
    Q.c[A7][j] = has_w ? (isA ? wA : isB ? wB : 0u) : 0u;
    Q.c[A8][j] = has_w ? (isA ? swA : isB ? swB : 0u) : 0u;
    Q.c[A9][j] = (e >> 12) & 1u ? carry : 0u;
    Q.fx[j] = e >> 16;
  }
}

// Operand words of one quad, loaded one tile ahead of its use.
struct QuadOps {
  uint64_t w[6];
  uint32_t lq;      // quad inside its instance
  uint32_t rounds;  // ~0u: no live quad (past the batch)
};

// Address computation and loads for the quad at `row` of instance `inst` (rows [o, o1)).
__device__ __forceinline__ void quad_ops_at(QuadOps& P, uint64_t row, uint32_t inst, uint64_t o,
                                            uint64_t o1, const b2f_input* __restrict__ in,
                                            const uint64_t* __restrict__ rec, const uint8_t* Sg) {
  const uint32_t rounds = ((uint32_t)(o1 - o) - FIXED_ROWS) / ROUND_ROWS;
  const uint32_t lq = (uint32_t)((row - o) >> 2);
  const b2f_input* x = in + inst;
  const uint64_t* st0 = rec + 16ull * state_index(o, inst);
  const uint64_t* fw = reinterpret_cast<const uint64_t*>(&x->rounds);  // rounds | f << 32
  P.lq = lq;
  P.rounds = rounds;
  const uint64_t *p0 = fw, *p1 = fw, *p2 = fw, *p3 = fw, *p4 = fw, *p5 = fw;
  uint32_t m = 0;
  const uint32_t rq = lq - INIT_QUADS;
  if (lq >= INIT_QUADS && rq < ROUND_QUADS * rounds) {
    const uint32_t r = rq / ROUND_QUADS, g = (rq - r * ROUND_QUADS) / G_QUADS;
    const uint64_t* st = st0 + 16ull * (2ull * r + (g >= 4));
    // (a, b, c, d) of G g: column g (g < 4) or diagonal g - 4 of the 4x4 work matrix
    const uint32_t gl = g & 3u, dg = g >> 2;
    const uint8_t* sg = Sg + 16 * (r % 10) + 2 * g;
    p0 = st + gl;
    p1 = st + 4 + ((gl + dg) & 3u);
    p2 = st + 8 + ((gl + 2 * dg) & 3u);
    p3 = st + 12 + ((gl + 3 * dg) & 3u);
    p4 = x->m + sg[0];
    p5 = x->m + sg[1];
    m = 63;
  } else if (lq < INIT_QUADS) {
    if (lq < 26) {
      p0 = lq < 8 ? x->h + lq : (lq < 24 ? x->m + (lq - 8) : x->t + (lq - 24));
      m = 1;
    } else if (lq == 26) {
      m = 1;  // fmask: the f word
    } else if (lq >= 35) {
      const uint32_t a = (lq - 35) >> 1;
      if (a < 2) p0 = x->t + a;
      m = 1;  // v12 = IV4 ^ t0, v13 = IV5 ^ t1, v14 = IV6 ^ fmask(f)
    }
  } else {
    const uint32_t a = (rq - ROUND_QUADS * rounds) >> 1;
    const uint64_t* fin = st0 + 16ull * (2ull * rounds);
    p0 = x->h + a;
    p1 = fin + a;
    p2 = fin + a + 8;
    m = 7;
  }
  P.w[0] = (m & 1u) ? *p0 : 0ull;
  P.w[1] = (m & 2u) ? *p1 : 0ull;
  P.w[2] = (m & 4u) ? *p2 : 0ull;
  P.w[3] = (m & 8u) ? *p3 : 0ull;
  P.w[4] = (m & 16u) ? *p4 : 0ull;
  P.w[5] = (m & 32u) ? *p5 : 0ull;
}

// Operand addresses of the quad at `row`, for instances first .. first + 7 with offsets
// Off[0..8] (LDS or global), then the loads. Round quads: the four state words of their G at
// the half-round start and the two message words; init quads: the input word they decompose
// (h/m/t, or the `rounds | f << 32` word for the fmask); final quads: h_i and the final
// v_i, v_{i+8}. Same data the fill_kernel reads (quad_cells / quad_round).
// Everything the address computation reads is in registers or LDS (Off, Sg): on CDNA, vmcnt
// counts stores and loads in issue order, so a global load here would wait for every store
// the wave has in flight.
__device__ __forceinline__ void quad_ops(QuadOps& P, uint64_t row, uint32_t first,
                                         const uint64_t* Off, uint32_t n, uint64_t used_rows,
                                         const b2f_input* __restrict__ in,
                                         const uint64_t* __restrict__ rec, const uint8_t* Sg) {
  P.rounds = ~0u;
  P.lq = 0;
#pragma unroll
  for (int k = 0; k < 6; k++) P.w[k] = 0;
  if (row >= used_rows || first >= n) return;
  uint32_t i = 0;
  while (i + 2 < NOFF && Off[i + 1] <= row) i++;
  const uint64_t o = Off[i], o1 = Off[i + 1];
  if (row < o || row >= o1 || first + i >= n) return;  // not for a layout the record kernel accepted
  quad_ops_at(P, row, first + i, o, o1, in, rec, Sg);
}

// The same from a TileInfo held in scalar registers (the fill kernel): the instance is found by
// a branch-free scan of the eight cached offsets.
__device__ __forceinline__ void quad_ops_ti(QuadOps& P, uint64_t row, const TileInfo& ti,
                                            uint32_t n, uint64_t used_rows,
                                            const b2f_input* __restrict__ in,
                                            const uint64_t* __restrict__ rec, const uint8_t* Sg) {
  P.rounds = ~0u;
  P.lq = 0;
#pragma unroll
  for (int k = 0; k < 6; k++) P.w[k] = 0;
  if (row >= used_rows || ti.first >= n) return;
  uint64_t o = ti.off[0], o1 = ti.off[1];
  uint32_t i = 0;
#pragma unroll
  for (int k = 1; k + 1 < NOFF; k++)
    if (ti.off[k] <= row) { o = ti.off[k]; o1 = ti.off[k + 1]; i = (uint32_t)k; }
  if (row < o || row >= o1 || ti.first + i >= n) return;
  quad_ops_at(P, row, ti.first + i, o, o1, in, rec, Sg);
}

// The operand word of init quad lq (< 41) of instance x: what quad_ops loads for it.
__device__ __forceinline__ uint64_t init_word(const b2f_input* __restrict__ x, uint32_t lq) {
  const uint64_t* fw = reinterpret_cast<const uint64_t*>(&x->rounds);
  if (lq < 26) return lq < 8 ? x->h[lq] : (lq < 24 ? x->m[lq - 8] : x->t[lq - 24]);
  if (lq == 26) return *fw;
  if (lq < 35) return 0;
  const uint32_t a = (lq - 35) >> 1;
  return a < 2 ? x->t[a] : *fw;
}

// Init and final quads from their operand words (the fill's quad_cells, register-fed).
__device__ __forceinline__ void quad_cells_ops(Quad& Q, const QuadOps& P, const uint64_t* IV) {
  const QuadInfo d = decode_quad(P.lq, P.rounds);
  switch (d.kind) {
    case K_INW: {
      const uint64_t W = P.w[0];
#pragma unroll
      for (int j = 0; j < 4; j++) lrow(Q, j, limb(W, j));
      Q.c[A7][0] = (uint32_t)W;
      Q.c[A8][0] = (uint32_t)(W >> 32);
      Q.fx[0] = 1u << S_ABCD;
      break;
    }
    case K_FMASK: {
      const uint32_t f = (P.w[0] >> 32) ? 1u : 0u;
#pragma unroll
      for (int j = 0; j < 4; j++) lrow(Q, j, f ? 0xffffu : 0u);
      Q.c[A5][0] = f;
      Q.fx[0] = 1u << S_FMASK;
      break;
    }
    case K_CONST: {
      const uint64_t W = IV[d.a];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        lrow(Q, j, limb(W, j));
        Q.fx[j] = (1u << S_CONST) | (limb(W, j) << 16);
      }
      break;
    }
    case K_XOR3:
      q_xor3(Q, P.w[0], P.w[1], P.w[2], d.q);
      break;
    default: {  // init XORs (round quads never come here)
      const uint64_t Y = d.a < 2 ? P.w[0] : ((P.w[0] >> 32) ? ~0ull : 0ull);
      q_xor(Q, IV[4 + d.a], Y, d.q, S_XOR);
      break;
    }
  }
}

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
constexpr int G_CHECKS = 72;  // copy constraints per G (check_table_ok)
constexpr int GT_WORDS_ = 8;  // words per G table entry
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
template <int LW, int WS>
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
            e = pack_check(LW + wc * WS + rel + CBIAS, 0, c, drow);
          } else if (kind == 2) {
            uint32_t role = (d >> 2) & 3u, k = (d >> 4) & 3u, sp = (d >> 6) & 1u;
            if (hr0) {
              e = pack_check(state_abs0(g, role, k), 1 + sp, c, drow);
            } else {
              uint32_t col = role == 1 ? (sp ? A8 : A7) : (sp ? A2 : A1);
              e = pack_check((uint32_t)((int)(LW + wc_of(col) * WS) + state_rel(g, role, k) + CBIAS),
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
template <int LW, int WS>
constexpr bool check_table_ok() {
  CheckTable T = make_check_table<LW, WS>();
  if (T.e[0][0] == 0xffffffffu) return false;
  for (int v = 0; v < 12; v++)
    for (int i = 0; i < G_CHECKS; i++) {
      uint32_t e = T.e[v][i];
      if (((e >> 14) & 7u) > 4 || ((e >> 19) & 63u) >= G_ROWS || ((e >> 17) & 3u) > 2) return false;
    }
  return true;
}
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
static_assert(B2F_CODE_FIXED == 18, "the fixed-column counter is word 18 of the accumulator");

// Failure bookkeeping of a half-round tile's checks. REC = false: every check is evaluated and
// only "some check failed" is kept (a flag, no branch around the bookkeeping: the common case,
// a valid trace); REC = true: every failure is recorded exactly as the eval kernel records it
// (counters, first failing row, deferred rows) -- run only when the fast pass flagged the tile.
template <bool REC>
struct Fails {
  EvalAcc A;
  bool bad;
  __device__ __forceinline__ void fail(bool cond, uint64_t row, uint32_t code) {
    if (REC) {
      if (cond) A.fail(row, code);
    } else {
      bad |= cond;
    }
  }
  __device__ __forceinline__ void gates(bool cond, uint64_t row, uint32_t mask) {
    if (REC) {
      if (cond) A.fail_gates(row, mask);
    } else {
      bad |= cond;
    }
  }
};


// A workgroup's counters into the report: one global atomic per non-zero counter (call after
// a barrier, every thread of the workgroup).
__device__ __forceinline__ void flush_report(const EvalAcc& A, b2f_eval_report* rep, int tid) {
  if (tid < 19) {
    const uint32_t v = A.c[tid];
    if (v) {
      unsigned long long* dst = tid < 16    ? (unsigned long long*)&rep->gate_failures[tid]
                              : tid == 16   ? (unsigned long long*)&rep->lookup_failures
                              : tid == 17   ? (unsigned long long*)&rep->copy_failures
                                            : (unsigned long long*)&rep->fixed_failures;
      atomicAdd(dst, (unsigned long long)v);
    }
  } else if (tid == 19) {
    const uint64_t fm = *reinterpret_cast<const uint64_t*>(A.c + 20);
    if (fm != ~0ull) atomicMin((unsigned long long*)&rep->first_failure, (unsigned long long)fm);
  }
}

// component j of a quad register (select chain: never an indexed access into a register array)
__device__ __forceinline__ uint32_t comp(const uint4& v, int j) {
  return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}

// LDS cell accessor: column c, tile-local row r (r may reach TILE_ROWS + 11)
template <int LW, int WS, int LG, int TS>
struct TileT {
  const uint32_t* L;
  __device__ __forceinline__ uint32_t at(int c, uint32_t r) const {
    switch (c) {
      case A1: return L[LW + 0 * WS + HIST + r];
      case A2: return L[LW + 1 * WS + HIST + r];
      case A7: return L[LW + 2 * WS + HIST + r];
      case A8: return L[LW + 3 * WS + HIST + r];
      case A0: return L[LG + 0 * TS + r];
      case A3: return L[LG + 1 * TS + r];
      case A4: return L[LG + 2 * TS + r];
      case A5: return L[LG + 3 * TS + r];
      default: return L[LG + 4 * TS + r];  // A6
    }
  }
  __device__ __forceinline__ uint4 quad(int c, uint32_t r) const {
    return *reinterpret_cast<const uint4*>(&L[(c == A1 || c == A2 || c == A7 || c == A8)
                                                  ? LW + (c == A1 ? 0 : c == A2 ? 1 : c == A7 ? 2 : 3) * WS + HIST + r
                                                  : LG + (c == A0 ? 0 : c - 2) * TS + r]);
  }
};
#define TC(c, r) T.at((c), (r))

// Evaluate gate `s` on the block whose selector row is tile-local row r. Every identity of
// LAYOUT.md §4 is checked in an exact integer form: linear identities as equalities in
// 64/128-bit arithmetic (all terms are < 2^100), the root constraints c(c-1)(c-2), t(t-1),
// b(b-1) as range tests (equivalent for non-negative integers < p). a9 and k0 are the
// selector row's own a_9 and fixed cells.
template <class Tile>
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
template <class Tile>
__device__ __forceinline__ V3 rows8(const Tile& T, int col, uint32_t r) {
  return V3{T.quad(col, r), T.quad(col, r + 4), make_uint4(0, 0, 0, 0)};
}

// XOR (s_spread_d1, s_spread_d2, s_xor) and XOR3 (s_xor3): operands on the even rows
template <class Tile>
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
template <class Tile>
__device__ __forceinline__ bool g_digest(const Tile& T, uint32_t r) {
  V3 d = rows8(T, A1, r);
  return (uint64_t)T.at(A7, r) == (uint64_t)d[0] + ((uint64_t)d[2] << 16) &&
         (uint64_t)T.at(A8, r) == (uint64_t)d[4] + ((uint64_t)d[6] << 16);
}
template <class Tile>
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
template <class Tile>
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
template <class Tile>
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

// ---------------------------------------------------------------- per-tile G table
// The G table of a tile (one wave, lane l = l-th G in row order whose start lies in
// [base0 + shift - 51, base0 + shift + 1023]): per G its window / init-cache bases, message
// rows, tile-local start and check-table row (g_pass / g_copies), plus QM[q] = position of
// quad q in its G (0xff: not a round quad). base0 is the row of LDS coordinate 0 (eval: the
// tile's first row; fused: 16 rows before it). The cached instances are walked in order (one
// or two for 12-round instances; a lane-parallel walk with readlane broadcasts measured
// slower). Init-region bases point into the init cache for the
// tile's first instance (its init region may lie before the window) and into the window for
// any later instance (which starts inside the tile). Instances past the cached eight cannot
// occur in a valid layout (each is >= 228 rows); invalid layouts are flagged elsewhere
// (offsets_check_kernel / the record kernel) and only have to stay in bounds here.
struct GTCarve {
  int qm, ng, gt;  // offsets inside the G set: QM bytes, entry count, entries
  int ic, w, ws;   // LDS: init cache, window base, window stride
  int qm_words, nq;
  int shift;
  int max_g;
};
__device__ __forceinline__ void build_g_table(uint32_t* S, const uint32_t* info, const uint8_t* Sg,
                                              int64_t base0, uint32_t n, uint64_t total_rows,
                                              uint32_t lane, const GTCarve& K) {
  // one wave: its lanes reset QM, then mark their G's quads (LDS order within a wave)
  if ((int)lane < K.qm_words) S[K.qm + lane] = 0xffffffffu;
  if (lane == 0 && K.qm_words > 64) S[K.qm + 64] = 0xffffffffu;
  const uint32_t first = info[0];
  const uint64_t* Off = reinterpret_cast<const uint64_t*>(info + 2);
  const int64_t lo = base0 + K.shift - (G_ROWS - 1), hi = base0 + K.shift + TILE_ROWS - 1;
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
    // G m starts at g0 + 52 m; o > base0 - MAX_INSTANCE_ROWS, so these fit in 32 bits
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
  if (lane == 0) S[K.ng] = base < (uint32_t)K.max_g ? base : (uint32_t)K.max_g;
  if (o_mine < 0 || lane >= (uint32_t)K.max_g) return;
  const uint32_t r = m >> 3, g = m & 7u;
  const int gl = (int)(o_mine + INIT_ROWS + (int64_t)G_ROWS * m - base0);
  const int ob = ofst ? 0 : (int)(o_mine - base0 + HIST);  // later instances: in the window
  const int ib0 = ofst ? K.ic : K.w + ob;
  const int ib1 = ofst ? K.ic + (int)INIT_ROWS : K.w + K.ws + ob;
  const uint8_t* sg = Sg + 16 * (r % 10) + 2 * g;
  uint32_t* gt = S + K.gt + GT_WORDS_ * lane;
  *reinterpret_cast<uint4*>(gt) = make_uint4((uint32_t)(gl + HIST - CBIAS), (uint32_t)ib0,
                                             (uint32_t)ib1, (uint32_t)(ib0 + 32 + 4 * sg[0]));
  *reinterpret_cast<uint4*>(gt + 4) = make_uint4((uint32_t)(ib0 + 32 + 4 * sg[1]), (uint32_t)gl,
                                                 (m < 4 ? 8 + g : g) * G_CHECKS, 0u);
  uint8_t* qm = reinterpret_cast<uint8_t*>(S + K.qm);
#pragma unroll
  for (int p = 0; p < (int)G_QUADS; p++) {
    const int q = (gl >> 2) + p;
    if (q >= 0 && q < K.nq) qm[q] = (uint8_t)p;
  }
}

// ---------------------------------------------------------------- per-tile G pass and copies
// Shared by eval_kernel (check rows = selector rows / operand rows in [0, 1024) of the tile)
// and fused_kernel (u coordinates: a block is checked where its last row lands, u in
// [16, 1040); operand rows in [16, 1040)). A G table entry is GT_WORDS words: 0 window base -
// CBIAS, 1/2 init-region a_1/a_2 bases, 3/4 message x/y row bases, 5 G start (tile-local),
// 6 check-table row.
struct GCarve {
  int qsel, a9;     // LDS: per-quad row-0 selector word | rest flag, row-0 a_9
  int ct;           // LDS: copy-check table
  int g, ts;        // LDS: gate columns a_0 a_3 a_4 a_5 a_6, stride
  int lo, hi;       // check-row range (tile-local)
  bool last_rule;   // fused: a block belongs to the tile holding its last row
};

// One limb k of an XOR24 (b1 + efgh) or XOR63 (b2 + ijkl) block: bit 0 = the spread-XOR
// identity of limb k fails, bit 1 = the re-split identity of limb k fails. The block's gate
// fails iff some limb's bit is set (the polynomials of LAYOUT.md §4 are per-limb conjunctions).
template <class Tile>
__device__ __forceinline__ uint32_t g_xor24_limb(const Tile& T, uint32_t r, uint32_t k) {
  const uint32_t b = r + 3 * k, k1 = r + 3 * ((k + 1) & 3u), k2 = r + 3 * ((k + 2) & 3u);
  const bool b1 = (uint64_t)T.at(A3, b) + T.at(A4, b) ==
                      (uint64_t)T.at(A2, b) + ((uint64_t)T.at(A2, b + 1) << 16) + 2 * (uint64_t)T.at(A2, b + 2) &&
                  (T.at(A0, b) | T.at(A0, b + 1)) == 0u;
  const bool efgh = (uint64_t)T.at(A7, b) == (uint64_t)T.at(A1, k1 + 1) + ((uint64_t)T.at(A1, k2) << 8) &&
                    (uint64_t)T.at(A8, b) == (uint64_t)T.at(A2, k1 + 1) + ((uint64_t)T.at(A2, k2) << 16);
  return (b1 ? 0u : 1u) | (efgh ? 0u : 2u);
}
template <class Tile>
__device__ __forceinline__ uint32_t g_xor63_limb(const Tile& T, uint32_t r, uint32_t k) {
  const uint32_t b = r + 2 * k, p = r + 2 * ((k + 3) & 3u);
  const uint32_t zb = T.at(A6, b), zp = T.at(A6, p), s0 = T.at(A2, b);
  const bool b2 = (uint64_t)T.at(A3, b) + T.at(A4, b) ==
                      (uint64_t)s0 + ((uint64_t)zb << 30) + 2 * (uint64_t)T.at(A2, b + 1) &&
                  T.at(A0, b) <= 1u && zb <= 1u;
  const bool ijkl = (uint64_t)T.at(A7, b) == (uint64_t)zp + 2 * (uint64_t)T.at(A1, b) &&
                    (uint64_t)T.at(A8, b) == (uint64_t)zp + 4 * (uint64_t)s0;
  return (b2 ? 0u : 1u) | (ijkl ? 0u : 2u);
}

// OR of v over the four lanes of a DPP quad (lanes 4i .. 4i + 3); every lane must be active.
__device__ __forceinline__ uint32_t quad_or(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
  return v;
}

// Canonical round blocks of the tile's G's, one block kind per wave so that every wave runs a
// single evaluator: wave 0 the four adds (a1 c1 a2 c2, a lane per block), wave 1 the two XORs
// (d1 d2, a lane per block), wave 2 XOR24 (b1) and wave 3 XOR63 (b2) with the four limbs of a
// block on the four lanes of a DPP quad, combined before the block is reported. A block is
// taken only if its quad carries exactly the canonical selectors (QSEL); every other selector
// row goes through the per-quad path.
template <class Tile, class Sink>
__device__ __forceinline__ void g_pass(const Tile& T, Sink& A, const uint32_t* L,
                                       const uint32_t* gt_base, uint32_t ng, int64_t row_base,
                                       uint32_t lane, uint32_t wave, const GCarve& C) {
  const uint32_t per_g = wave == 1 ? 2u : 4u;
  const uint32_t items = per_g * ng;
#pragma unroll 1
  for (uint32_t it0 = 0; it0 < items; it0 += 64) {  // uniform trip count (DPP below)
    const uint32_t it = it0 + lane;
    const uint32_t g = wave == 1 ? it >> 1 : it >> 2;
    const uint32_t w = wave == 1 ? it & 1u : it & 3u;  // waves 2, 3: w = limb
    // wave 0: a1 +0, c1 +12, a2 +28, c2 +40; wave 1: d1 +4, d2 +32; b1 +16; b2 +44
    const int off = wave == 0 ? (w == 0 ? 0 : w == 1 ? 12 : w == 2 ? 28 : 40)
                  : wave == 1 ? (w ? 32 : 4) : wave == 2 ? 16 : 44;
    const int len = wave == 0 ? 4 : wave == 2 ? 12 : 8;
    const uint32_t want = wave == 0 ? 1u << (w == 0 ? S_A1 : w == 1 ? S_C1 : w == 2 ? S_A2 : S_C2)
                        : wave == 1 ? 1u << (w ? S_D2 : S_D1)
                        : wave == 2 ? (1u << S_B1) | (1u << S_EFGH) : (1u << S_B2) | (1u << S_IJKL);
    const int rl = it < items ? (int)gt_base[GT_WORDS_ * g + 5] + off : -1;
    const int key = C.last_rule ? rl + len - 1 : rl;
    const bool take = rl >= 0 && key >= C.lo && key < C.hi && L[C.qsel + (rl >> 2)] == want;
    const uint32_t r = (uint32_t)rl;
    uint32_t f = 0;
    if (wave >= 2) {
      uint32_t bits = 0;
      if (take) bits = wave == 2 ? g_xor24_limb(T, r, w) : g_xor63_limb(T, r, w);
      bits = quad_or(bits);
      if (take && w == 0 && bits)
        f = ((bits & 1u) ? 1u << (wave == 2 ? S_B1 : S_B2) : 0u) |
            ((bits & 2u) ? 1u << (wave == 2 ? S_EFGH : S_IJKL) : 0u);
    } else if (take) {
      f = (wave == 0 ? g_add(T, r, L[C.a9 + (r >> 2)], (w & 1u) == 0) : g_xor(T, r, false)) ? 0u : want;
    }
    A.gates(f != 0, (uint64_t)(row_base + rl), f);
  }
}

// The 72 copy checks of every G of the tile: LPG lanes per G table entry, each reading the
// entry once and then issuing its checks' LDS reads independently (source cell at per-G base
// + table offset, operand cell at its row). A check belongs to the tile holding its operand row.
constexpr int LPG = 10;
#ifndef B2F_COPY_REMAP
#define B2F_COPY_REMAP 1
#endif
#ifndef B2F_COPY_UNROLL
#define B2F_COPY_UNROLL 4
#endif
#ifndef B2F_GT_WAVE
#define B2F_GT_WAVE 1
#endif
constexpr int GT_WAVE = B2F_GT_WAVE;  // wave that builds the next tile's G table (g_pass: XOR)
template <class Sink>
__device__ __forceinline__ void g_copies(Sink& A, const uint32_t* L, const uint32_t* gt_base,
                                         uint32_t ng, int64_t row_base, uint32_t tid,
                                         const GCarve& C) {
  // the wave that built the G table takes the last slice of lanes (the fewest G entries)
  const uint32_t w = tid >> 6, slot = w == (uint32_t)GT_WAVE ? 3u : (w < (uint32_t)GT_WAVE ? w : w - 1);
  const uint32_t ctid = (B2F_COPY_REMAP ? slot : w) * 64 + (tid & 63u);
  const uint32_t gi = ctid / LPG, c0 = ctid - gi * LPG;
  if (gi >= ng) return;
  const uint4 g0 = *reinterpret_cast<const uint4*>(gt_base + GT_WORDS_ * gi);
  const uint4 g1 = *reinterpret_cast<const uint4*>(gt_base + GT_WORDS_ * gi + 4);
#pragma unroll B2F_COPY_UNROLL
  for (int j = 0; j < (G_CHECKS + LPG - 1) / LPG; j++) {
    const uint32_t ci = c0 + LPG * j;
    if (ci >= (uint32_t)G_CHECKS) break;
    const uint32_t e = L[C.ct + g1.z + ci];
    const uint32_t sel = (e >> 14) & 7u;
    const uint32_t base = sel == 0 ? g0.x : sel == 1 ? g0.y : sel == 2 ? g0.z : sel == 3 ? g0.w : g1.x;
    const int src = (int)base + (int)(e & 16383u);
    const int dl = (int)g1.y + (int)((e >> 19) & 63u);
    const uint32_t sv = L[src < 0 ? 0 : src];  // < 0 only for checks outside the tile
    const int dlc = dl < C.lo ? C.lo : (dl >= C.hi ? C.hi - 1 : dl);
    const uint32_t dv = L[C.g + (1 + ((e >> 17) & 3u)) * C.ts + dlc];
    A.fail(dl >= C.lo && dl < C.hi && dv != sv, (uint64_t)(row_base + dl), B2F_CODE_COPY);
  }
}

// Any selector combination, one gate at a time (kept out of line: the hot path never takes it
// for a trace this engine wrote).
template <class Tile>
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
template <class Tile>
__device__ __forceinline__ uint32_t row_gates(const Tile& T, uint32_t sel, uint32_t r, uint32_t a9,
                                              uint32_t k0) {
  switch (sel) {
    case 1u << S_XOR:
      return g_xor(T, r, false) ? 0u : sel;
    case (1u << S_XOR3) | (1u << S_DIGEST):
      return (g_xor(T, r, true) ? 0u : 1u << S_XOR3) | (g_digest(T, r) ? 0u : 1u << S_DIGEST);
    case 1u << S_ABCD:  // input-word decompositions (26 per instance)
      return gate_ok(T, S_ABCD, r, a9, k0) ? 0u : sel;
    case 1u << S_FMASK:
      return gate_ok(T, S_FMASK, r, a9, k0) ? 0u : sel;
    default:
      return gates_generic(T, sel, r, a9, k0);
  }
}

// Copy-source lookup, all from LDS for a valid trace: rows inside the window come from W;
// init-region words (h, m, t, fmask, IV, v12..v14) of the tile's first instance, which may
// start before the window, from the init cache I (a_1 | a_2 of its rows 0..163). Anything
// else (only reachable through a corrupted layout) is read from global memory.
template <int WS>
struct Src {
  const uint32_t* W;
  const uint32_t* I;
  const uint32_t* adv;
  uint64_t total_rows, wlo, ofirst;
  // wc: source column as W index (a_1 a_2 a_7 a_8 -> 0 1 2 3)
  __device__ __forceinline__ uint32_t at(uint64_t gs, uint32_t wc) const {
    uint64_t d = gs - wlo;  // wraps for gs < wlo
    if (d < (uint64_t)WS) return W[wc * WS + (uint32_t)d];
    uint64_t e = gs - ofirst;
    if (e < (uint64_t)INIT_ROWS && wc < 2) return I[wc * INIT_ROWS + (uint32_t)e];
    uint32_t col = wc < 2 ? wc + 1 : wc + 5;
    return adv[(uint64_t)col * total_rows + gs];
  }
  __device__ __forceinline__ uint32_t operator()(uint64_t gs, uint32_t col) const {
    return at(gs, col < 3 ? col - 1 : col - 5);
  }
};

template <class Sink>
__device__ __forceinline__ void copy_check(Sink& A, uint32_t dv, uint32_t sv, uint64_t gd) {
  A.fail(dv != sv, gd, B2F_CODE_COPY);
}

// canonical cell of limb k of state word w as half-round hr starts (instance-local row)
__host__ __device__ __forceinline__ uint32_t state_src(uint32_t w, uint32_t k, uint32_t spread,
                                                       uint32_t hr, uint32_t& col) {
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
template <class Sink, class Src>
__device__ void copies_edge(Sink& A, uint4 d0, uint4 d1, uint4 d2, const Src& src, uint64_t o,
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
      uint32_t dx = comp(d0, 2 * h), dy = comp(d1, 2 * h);
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
      copy_check(A, comp(d0, 2 * h), src(o + 4 * d.a + k, A2), gd);
      copy_check(A, comp(d1, 2 * h), src(o + vs, cv), gd);
      copy_check(A, comp(d2, 2 * h), src(o + us, cu), gd);
    }
  }
}

}  // namespace

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

namespace {

__constant__ uint64_t c_iv[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL,
                                 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                                 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

// SIGMA = table16.rs:32-44
__constant__ uint8_t c_sigma[10][16] = {
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

__constant__ uint8_t c_gidx[8][4] = {{0, 4, 8, 12}, {1, 5, 9, 13}, {2, 6, 10, 14},
                                     {3, 7, 11, 15}, {0, 5, 10, 15}, {1, 6, 11, 12},
                                     {2, 7, 8, 13}, {3, 4, 9, 14}};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

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

__global__ void __launch_bounds__(BLOCK) fill_kernel(const b2f_input* __restrict__ in,
                                                    uint32_t n,
                                                    const uint64_t* __restrict__ off,
                                                    uint64_t total_rows,
                                                    const uint64_t* __restrict__ rec,
                                                    uint32_t* __restrict__ adv,
                                                    uint32_t* __restrict__ fixed,
                                                    const int* __restrict__ status,
                                                    uint64_t tiles_per_wg) {
  if (*status) return;  // the record kernel rejected the layout: write nothing
  const uint64_t total_quads = total_rows >> 2;
  const uint64_t used_rows = off[n];
  uint64_t t0 = (uint64_t)blockIdx.x * tiles_per_wg;
  uint64_t t1 = t0 + tiles_per_wg;
  uint64_t q_first = t0 * BLOCK + threadIdx.x;
  if (q_first >= total_quads) return;
  uint32_t inst = find_instance(off, n, min(4 * q_first, used_rows ? used_rows - 1 : 0));
  for (uint64_t t = t0; t < t1; t++) {
    uint64_t gq = t * BLOCK + threadIdx.x;
    if (gq >= total_quads) break;
    uint64_t row = 4 * gq;
    Quad Q;
    zero(Q);
    if (row < used_rows) {
      while (off[inst + 1] <= row) inst++;
      uint64_t o = off[inst];
      const b2f_input* x = in + inst;
      uint32_t rounds = x->rounds;
      const uint64_t* states = rec + 16ull * state_index(o, inst);
      quad_cells(Q, x, states, rounds, (uint32_t)((row - o) >> 2));
    }
#pragma unroll
    for (int c = 0; c < 10; c++) {
      u32x4 v = {Q.c[c][0], Q.c[c][1], Q.c[c][2], Q.c[c][3]};
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(adv + (uint64_t)c * total_rows + row));
    }
    u32x4 f = {Q.fx[0], Q.fx[1], Q.fx[2], Q.fx[3]};
    __builtin_nontemporal_store(f, reinterpret_cast<u32x4*>(fixed + row));
  }
}

// --------------------------------------------------------------------------- eval kernel

struct EvalAcc {
  uint32_t gate[B2F_NUM_GATES];
  uint32_t lookup, copy;
  uint64_t first;
};

__device__ __forceinline__ void note(EvalAcc& A, uint64_t row, uint32_t code) {
  uint64_t key = (row << 8) | code;
  A.first = key < A.first ? key : A.first;
}

// LDS tile accessor: column c (0..9 advice, 10 fixed), tile-local row r
#define TC(c, r) T[(c) * TSTRIDE + (r)]

// Evaluate gate `s` at tile-local row r. Every identity of LAYOUT.md §4 is checked in an
// exact integer form: linear identities as equalities in 64/128-bit arithmetic (all terms
// are < 2^100), the root constraints c(c-1)(c-2), t(t-1), b(b-1) as range tests (equivalent
// for non-negative integers < p).
__device__ __forceinline__ bool gate_ok(const uint32_t* __restrict__ T, int s, uint32_t r) {
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
#pragma unroll
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
#pragma unroll
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
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        uint64_t in = (uint64_t)TC(A3, r + k) + TC(A4, r + k) + (three ? TC(A5, r + k) : 0u);
        lhs += (u128)in << (16 * k);
        rhs += (u128)TC(A1, r + k) << (16 * k);
      }
      uint32_t cy = TC(A9, r);
      rhs += (u128)cy << 64;
      return lhs == rhs && cy <= (three ? 2u : 1u);
    }
    case S_B1: {
      bool ok = true;
#pragma unroll
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
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        uint32_t b = r + 2 * k;
        ok &= (uint64_t)TC(A3, b) + TC(A4, b) == (uint64_t)TC(A2, b) + 2 * (uint64_t)TC(A2, b + 1);
      }
      return ok;
    }
    case S_B2: {
      bool ok = true;
#pragma unroll
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
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        uint32_t b = r + 2 * k;
        ok &= (uint64_t)TC(A3, b) + TC(A4, b) + TC(A5, b) ==
              (uint64_t)TC(A2, b) + 2 * (uint64_t)TC(A2, b + 1);
      }
      return ok;
    }
    case S_CONST:
      return TC(A1, r) == (TC(10, r) >> 16);
    case S_FMASK: {
      uint32_t f = TC(A5, r);
      bool ok = f <= 1u;
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) ok &= (uint64_t)TC(A1, r + k) == 65535ull * f;
      return ok;
    }
  }
  return true;
}

// One copy constraint: operand cell (dcol, instance-local drow) == canonical (scol, srow).
__device__ __forceinline__ void copy_check(EvalAcc& A, const uint32_t* __restrict__ T,
                                           const uint32_t* __restrict__ adv,
                                           uint64_t total_rows, uint64_t tile0, uint64_t o,
                                           int dcol, uint32_t drow, int scol, uint32_t srow) {
  uint64_t gd = o + drow, gs = o + srow;
  uint32_t dv = TC(dcol, (uint32_t)(gd - tile0));  // the operand is in this thread's quad
  uint32_t sv;
  if (gs >= tile0 && gs < tile0 + TSTRIDE) sv = TC(scol, (uint32_t)(gs - tile0));
  else sv = adv[(uint64_t)scol * total_rows + gs];
  if (dv != sv) { A.copy++; note(A, gd, B2F_CODE_COPY); }
}

__device__ __forceinline__ void copies_of_quad(EvalAcc& A, const uint32_t* __restrict__ T,
                                               const uint32_t* __restrict__ adv,
                                               uint64_t total_rows, uint64_t tile0, uint64_t o,
                                               const b2f_input* __restrict__ unused,
                                               uint32_t rounds, uint32_t lq) {
  (void)unused;
  QuadInfo d = decode_quad(lq, rounds);
  const uint32_t r0 = 4 * lq;  // first row of the quad (instance-local)
  switch (d.kind) {
    case K_INW: case K_FMASK: case K_CONST: case K_PAD:
      return;
    case K_XOR3: {
      Canon H = canon_h(d.a), V = canon_state(d.a, 2 * rounds), U = canon_state(d.a + 8, 2 * rounds);
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        uint32_t k = 2 * d.q + h, row = r0 + 2 * h;
        copy_check(A, T, adv, total_rows, tile0, o, A3, row, H.scol, H.row(k));
        copy_check(A, T, adv, total_rows, tile0, o, A4, row, V.scol, V.row(k));
        copy_check(A, T, adv, total_rows, tile0, o, A5, row, U.scol, U.row(k));
      }
      return;
    }
    default:
      break;
  }
  // Operand words X, Y (and M for ADD3) of the block.
  Canon X, Y, M;
  M = canon_m(0);
  if (d.block < INIT_ROWS) {  // init XORs
    X = canon(108 + 4 * (4 + d.a), 1, 0, A1, A2);
    Y = d.a < 2 ? canon(96 + 4 * d.a, 1, 0, A1, A2) : canon(104, 1, 0, A1, A2);
  } else {
    uint32_t r = d.a, g = d.g, hr = 2 * r + (g >= 4);
    uint32_t gb = INIT_ROWS + ROUND_ROWS * r + G_ROWS * g;
    Canon va = canon_state(c_gidx[g][0], hr), vb = canon_state(c_gidx[g][1], hr);
    Canon vc = canon_state(c_gidx[g][2], hr), vd = canon_state(c_gidx[g][3], hr);
    Canon a1 = canon(gb + 0, 1, 0, A1, A2), d1 = canon(gb + 4, 2, 2, A1, A2);
    Canon c1 = canon(gb + 12, 1, 0, A1, A2), b1 = canon(gb + 16, 3, 0, A7, A8);
    Canon a2 = canon(gb + 28, 1, 0, A1, A2), d2 = canon(gb + 32, 2, 1, A1, A2);
    Canon c2 = canon(gb + 40, 1, 0, A1, A2);
    const uint8_t* sg = c_sigma[r % 10];
    switch (d.step) {
      case 0: X = va; Y = vb; M = canon_m(sg[2 * g]); break;
      case 1: X = vd; Y = a1; break;
      case 2: X = vc; Y = d1; break;
      case 3: X = vb; Y = c1; break;
      case 4: X = a1; Y = b1; M = canon_m(sg[2 * g + 1]); break;
      case 5: X = d1; Y = a2; break;
      case 6: X = c1; Y = d2; break;
      default: X = b1; Y = c2; break;
    }
  }
  switch (d.kind) {
    case K_ADD3:
    case K_ADD2:
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        uint32_t row = r0 + k;
        copy_check(A, T, adv, total_rows, tile0, o, A3, row, X.dcol, X.row(k));
        copy_check(A, T, adv, total_rows, tile0, o, A4, row, Y.dcol, Y.row(k));
        if (d.kind == K_ADD3) copy_check(A, T, adv, total_rows, tile0, o, A5, row, M.dcol, M.row(k));
      }
      return;
    case K_XOR:
    case K_XOR63:
#pragma unroll
      for (uint32_t h = 0; h < 2; h++) {
        uint32_t k = 2 * d.q + h, row = r0 + 2 * h;
        copy_check(A, T, adv, total_rows, tile0, o, A3, row, X.scol, X.row(k));
        copy_check(A, T, adv, total_rows, tile0, o, A4, row, Y.scol, Y.row(k));
      }
      return;
    case K_XOR24:
#pragma unroll
      for (uint32_t j = 0; j < 4; j++) {
        uint32_t R = 4 * d.q + j;
        if (R % 3 == 0) {
          uint32_t k = R / 3, row = r0 + j;
          copy_check(A, T, adv, total_rows, tile0, o, A3, row, X.scol, X.row(k));
          copy_check(A, T, adv, total_rows, tile0, o, A4, row, Y.scol, Y.row(k));
        }
      }
      return;
    default:
      return;
  }
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint64_t wave_min(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t u = __shfl_xor(v, o, 64);
    v = u < v ? u : v;
  }
  return v;
}

__global__ void __launch_bounds__(BLOCK) eval_kernel(const uint32_t* __restrict__ adv,
                                                    const uint32_t* __restrict__ fixed,
                                                    const uint64_t* __restrict__ off, uint32_t n,
                                                    uint64_t total_rows,
                                                    b2f_eval_report* __restrict__ rep,
                                                    int* __restrict__ status,
                                                    uint64_t tiles_per_wg) {
  __shared__ __attribute__((aligned(16))) uint32_t T[NCOL_T * TSTRIDE];
  EvalAcc A;
#pragma unroll
  for (int s = 0; s < B2F_NUM_GATES; s++) A.gate[s] = 0;
  A.lookup = 0; A.copy = 0; A.first = ~0ull;

  const uint64_t total_quads = total_rows >> 2;
  const uint64_t used_rows = off[n];
  if (used_rows > total_rows || off[0] != 0) {  // never read past the trace
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(status, 1 << B2F_ERR_LAYOUT);
    return;
  }
  const uint64_t t0 = (uint64_t)blockIdx.x * tiles_per_wg;
  const uint64_t t1 = t0 + tiles_per_wg;
  uint32_t inst = 0;
  bool have_inst = false;
  for (uint64_t t = t0; t < t1; t++) {
    const uint64_t tile0 = t * TILE_ROWS;
    if (tile0 >= total_rows) break;
    // ---- stage: every thread loads one quad (11 x 16 B); threads 0..3 also the halo
    const uint64_t gq = t * BLOCK + threadIdx.x;
    uint4 mine[NCOL_T];
    if (gq < total_quads) {
#pragma unroll
      for (int c = 0; c < 10; c++)
        mine[c] = *reinterpret_cast<const uint4*>(adv + (uint64_t)c * total_rows + 4 * gq);
      mine[10] = *reinterpret_cast<const uint4*>(fixed + 4 * gq);
    } else {
#pragma unroll
      for (int c = 0; c < NCOL_T; c++) mine[c] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < NCOL_T; c++)
      *reinterpret_cast<uint4*>(&T[c * TSTRIDE + 4 * threadIdx.x]) = mine[c];
    if (threadIdx.x < HALO_ROWS / 4) {
      uint64_t hq = (t + 1) * BLOCK + threadIdx.x;
#pragma unroll
      for (int c = 0; c < NCOL_T; c++) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (hq < total_quads)
          v = *reinterpret_cast<const uint4*>((c < 10 ? adv + (uint64_t)c * total_rows : fixed) + 4 * hq);
        *reinterpret_cast<uint4*>(&T[c * TSTRIDE + TILE_ROWS + 4 * threadIdx.x]) = v;
      }
    }
    __syncthreads();
    if (gq < total_quads) {
      const uint64_t row0 = 4 * gq;
      const uint32_t lr0 = 4 * threadIdx.x;
      // ---- lookups and gates on the 4 rows
#pragma unroll
      for (int j = 0; j < 4; j++) {
        uint32_t tg = (&mine[A0].x)[j], de = (&mine[A1].x)[j], sp = (&mine[A2].x)[j];
        bool ok = de < 65536u && tg == tag16(de) && sp == spread16(de & 0xffffu);
        if (!ok) { A.lookup++; note(A, row0 + j, B2F_CODE_LOOKUP); }
        uint32_t sel = (&mine[10].x)[j] & 0xffffu;
        while (sel) {
          int s = __builtin_ctz(sel);
          sel &= sel - 1;
          if (!gate_ok(T, s, lr0 + j)) { A.gate[s]++; note(A, row0 + j, (uint32_t)s); }
        }
      }
      // ---- copy constraints whose operand cell lies in this quad
      if (row0 < used_rows) {
        if (!have_inst) { inst = find_instance(off, n, row0); have_inst = true; }
        while (off[inst + 1] <= row0) inst++;
        uint64_t o = off[inst], o1 = off[inst + 1], R = o1 - o;
        if (o1 > o && o1 <= total_rows && R >= FIXED_ROWS && (R - FIXED_ROWS) % ROUND_ROWS == 0 &&
            (R - FIXED_ROWS) / ROUND_ROWS <= B2F_MAX_ROUNDS) {
          uint32_t rounds = (uint32_t)((R - FIXED_ROWS) / ROUND_ROWS);
          copies_of_quad(A, T, adv, total_rows, tile0, o, nullptr, rounds,
                         (uint32_t)((row0 - o) >> 2));
        } else {
          atomicOr(status, 1 << B2F_ERR_LAYOUT);
        }
      }
    }
    __syncthreads();
  }
  // ---- reduce: wave, then one atomic per counter per wave
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < B2F_NUM_GATES; s++) {
    uint64_t v = wave_sum(A.gate[s]);
    if (lane == 0 && v) atomicAdd((unsigned long long*)&rep->gate_failures[s], (unsigned long long)v);
  }
  uint64_t lk = wave_sum(A.lookup), cp = wave_sum(A.copy), fm = wave_min(A.first);
  if (lane == 0) {
    if (lk) atomicAdd((unsigned long long*)&rep->lookup_failures, (unsigned long long)lk);
    if (cp) atomicAdd((unsigned long long*)&rep->copy_failures, (unsigned long long)cp);
    if (fm != ~0ull) atomicMin((unsigned long long*)&rep->first_failure, (unsigned long long)fm);
  }
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

uint64_t layout_rows(uint32_t rounds) {
  if (rounds > B2F_MAX_ROUNDS) return 0;
  return (uint64_t)FIXED_ROWS + (uint64_t)ROUND_ROWS * rounds;
}

uint64_t grid_tiles(b2f_ctx* ctx, uint64_t total_rows, uint64_t* tiles_per_wg, int wgs_per_cu) {
  uint64_t tiles = (total_rows + TILE_ROWS - 1) / TILE_ROWS;
  uint64_t max_wg = (uint64_t)ctx->cu_count * wgs_per_cu;
  uint64_t wgs = tiles < max_wg ? tiles : max_wg;
  if (wgs == 0) wgs = 1;
  *tiles_per_wg = (tiles + wgs - 1) / wgs;
  return (tiles + *tiles_per_wg - 1) / *tiles_per_wg;
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
  uint64_t tpw;
  uint64_t wgs = grid_tiles(ctx, total_rows, &tpw, 8);
  tk = timed_begin(ctx, B2F_KERNEL_FILL, s);
  hipLaunchKernelGGL(fill_kernel, dim3((uint32_t)wgs), dim3(BLOCK), 0, s, d_in, nn, d_offsets,
                     total_rows, ctx->d_rec, d_advice, d_fixed, ctx->d_status, tpw);
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
  uint64_t tpw;
  uint64_t wgs = grid_tiles(ctx, total_rows, &tpw, 3);
  int tk = timed_begin(ctx, B2F_KERNEL_EVAL, s);
  hipLaunchKernelGGL(eval_kernel, dim3((uint32_t)wgs), dim3(BLOCK), 0, s, d_advice, d_fixed,
                     d_offsets, (uint32_t)n, total_rows, d_report, ctx->d_status + 1, tpw);
  HIPCHK(ctx, hipGetLastError());
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

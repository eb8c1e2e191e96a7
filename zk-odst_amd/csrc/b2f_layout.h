// b2f_layout.h -- device-side restatement of docs/LAYOUT.md (LAYOUT v1): row map, block
// decode and canonical-cell map, shared by the fill and eval kernels. Product code; it does
// not include or link anything under oracle/.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace b2f {

constexpr uint32_t INIT_ROWS = 164, ROUND_ROWS = 416, FINAL_ROWS = 64, G_ROWS = 52;
constexpr uint32_t INIT_QUADS = INIT_ROWS / 4, ROUND_QUADS = ROUND_ROWS / 4;
constexpr uint32_t G_QUADS = G_ROWS / 4, FINAL_QUADS = FINAL_ROWS / 4;
constexpr uint32_t FIXED_ROWS = INIT_ROWS + FINAL_ROWS;  // R(0)
// The fused half-round launch walks an instance's half-rounds on one wave in segments of at most
// SEG_HR (12 rounds): an instance's first segment is dealt with the instance, the later ones of a
// longer instance go to a list that every wave drains after its instances, each starting from
// recorded states (the record kernel keeps the state before and at every segment start).
constexpr uint32_t SEG_HR = 24;

// columns
enum : int { A0 = 0, A1, A2, A3, A4, A5, A6, A7, A8, A9 };
// selector bits (LAYOUT.md §4; bits 0..11 are the reference's compression.rs:561-577)
enum : int {
  S_ABCD = 0, S_EFGH, S_IJKL, S_A1, S_B1, S_C1, S_D1, S_A2, S_B2, S_C2, S_D2,
  S_DIGEST, S_XOR, S_XOR3, S_CONST, S_FMASK
};

// Block kinds of a quad (4 rows).
enum : int {
  K_INW = 0, K_FMASK, K_CONST, K_XOR, K_ADD3, K_ADD2, K_XOR24, K_XOR63, K_XOR3, K_PAD
};

// Where the four limbs of a word live: rows base + stride*perm(k) in columns (dcol, scol).
// perm(k) = (k + shift) & 3.
struct Canon {
  uint32_t base;   // instance-local row of the block
  uint8_t stride;  // 1 (lookup rows), 2 (XOR even rows), 3 (XOR24)
  uint8_t shift;   // limb relabelling of a rotation: 0, 1 (rot 16), 2 (rot 32)
  uint8_t dcol, scol;
  __device__ __forceinline__ uint32_t row(uint32_t k) const {
    return base + stride * ((k + shift) & 3u);
  }
};

__device__ __forceinline__ Canon canon(uint32_t base, uint32_t stride, uint32_t shift,
                                       int dcol, int scol) {
  Canon c;
  c.base = base; c.stride = (uint8_t)stride; c.shift = (uint8_t)shift;
  c.dcol = (uint8_t)dcol; c.scol = (uint8_t)scol;
  return c;
}

// Init-region words (LAYOUT.md §5 table).
__device__ __forceinline__ Canon canon_h(uint32_t i) { return canon(4 * i, 1, 0, A1, A2); }
__device__ __forceinline__ Canon canon_m(uint32_t j) { return canon(32 + 4 * j, 1, 0, A1, A2); }

// The canonical cells of state word w as the half-round `hr` starts (hr = 0 .. 2*rounds).
// hr = 0: the initial work vector. Otherwise the G of half-round hr-1 that owns w produced
// it in its last step of w's role: a <- a2 (ADD3 +28), b <- b2 (XOR63 +44),
// c <- c2 (ADD2 +40), d <- d2 (XOR rot16 +32).
__device__ __forceinline__ Canon canon_state(uint32_t w, uint32_t hr) {
  if (hr == 0) {
    if (w < 8) return canon_h(w);
    if (w == 12) return canon(140, 2, 0, A1, A2);
    if (w == 13) return canon(148, 2, 0, A1, A2);
    if (w == 14) return canon(156, 2, 0, A1, A2);
    uint32_t i = (w == 15) ? 7u : (w - 8);
    return canon(108 + 4 * i, 1, 0, A1, A2);
  }
  uint32_t hp = hr - 1, rp = hp >> 1;
  uint32_t role = w >> 2, pos = w & 3;
  uint32_t g = (hp & 1) ? 4 + ((pos - role) & 3u) : pos;
  uint32_t gb = INIT_ROWS + ROUND_ROWS * rp + G_ROWS * g;
  switch (role) {
    case 0: return canon(gb + 28, 1, 0, A1, A2);
    case 1: return canon(gb + 44, 2, 0, A7, A8);
    case 2: return canon(gb + 40, 1, 0, A1, A2);
    default: return canon(gb + 32, 2, 1, A1, A2);
  }
}

// Decoded quad: block kind, quad index inside the block, and the parameters that select the
// block's words.
struct QuadInfo {
  int kind;
  uint32_t q;      // quad inside the block
  uint32_t block;  // instance-local first row of the block
  int sel;         // selector bit of the block (XOR/ADD variants)
  uint32_t a;      // init: word index; round: round r; final: output word i
  uint32_t g;      // round: G index
  uint32_t step;   // round: 0..7 = a1 d1 c1 b1 a2 d2 c2 b2
};

// step of a quad inside a G (13 quads): a1 | d1 d1 | c1 | b1 b1 b1 | a2 | d2 d2 | c2 | b2 b2
__device__ __forceinline__ void g_quad(uint32_t wq, uint32_t& step, uint32_t& q, uint32_t& off) {
  // offsets in rows: 0 4 12 16 28 32 40 44
  if (wq < 1) { step = 0; q = wq; off = 0; }
  else if (wq < 3) { step = 1; q = wq - 1; off = 4; }
  else if (wq < 4) { step = 2; q = 0; off = 12; }
  else if (wq < 7) { step = 3; q = wq - 4; off = 16; }
  else if (wq < 8) { step = 4; q = 0; off = 28; }
  else if (wq < 10) { step = 5; q = wq - 8; off = 32; }
  else if (wq < 11) { step = 6; q = 0; off = 40; }
  else { step = 7; q = wq - 11; off = 44; }
}

__device__ __forceinline__ QuadInfo decode_quad(uint32_t lq, uint32_t rounds) {
  QuadInfo d;
  d.q = 0; d.g = 0; d.step = 0; d.sel = 0; d.a = 0;
  if (lq < INIT_QUADS) {
    if (lq < 26) {  // INW h0..7, m0..15, t0, t1
      d.kind = K_INW; d.a = lq; d.block = 4 * lq; d.sel = S_ABCD;
    } else if (lq == 26) {
      d.kind = K_FMASK; d.block = 104; d.sel = S_FMASK;
    } else if (lq < 35) {
      d.kind = K_CONST; d.a = lq - 27; d.block = 4 * lq; d.sel = S_CONST;
    } else {
      d.kind = K_XOR; d.a = (lq - 35) >> 1; d.q = (lq - 35) & 1;
      d.block = 140 + 8 * d.a; d.sel = S_XOR;
    }
    return d;
  }
  uint32_t rq = lq - INIT_QUADS;
  if (rq < ROUND_QUADS * rounds) {
    uint32_t r = rq / ROUND_QUADS, w = rq - r * ROUND_QUADS;
    uint32_t g = w / G_QUADS, wq = w - g * G_QUADS;
    uint32_t step, q, off;
    g_quad(wq, step, q, off);
    d.a = r; d.g = g; d.step = step; d.q = q;
    d.block = INIT_ROWS + ROUND_ROWS * r + G_ROWS * g + off;
    switch (step) {
      case 0: d.kind = K_ADD3; d.sel = S_A1; break;
      case 1: d.kind = K_XOR; d.sel = S_D1; break;
      case 2: d.kind = K_ADD2; d.sel = S_C1; break;
      case 3: d.kind = K_XOR24; d.sel = S_B1; break;
      case 4: d.kind = K_ADD3; d.sel = S_A2; break;
      case 5: d.kind = K_XOR; d.sel = S_D2; break;
      case 6: d.kind = K_ADD2; d.sel = S_C2; break;
      default: d.kind = K_XOR63; d.sel = S_B2; break;
    }
    return d;
  }
  uint32_t fq = rq - ROUND_QUADS * rounds;
  d.kind = K_XOR3; d.a = fq >> 1; d.q = fq & 1; d.sel = S_XOR3;
  d.block = INIT_ROWS + ROUND_ROWS * rounds + 8 * d.a;
  return d;
}

// The keygen structure of the fixed column (LAYOUT.md §4/§5): the four fixed cells of a
// decoded quad, from the row map alone. Selectors sit on a block's first row; CONST blocks
// carry `s_const | IV_k << 16` on each of their four rows. `ivw` = IV[d.a] (read only for
// CONST quads). halo2 fixes these at keygen (keygen_vk/keygen_pk,
// benchmarking/src/blake2f_circuit_bench.rs:54-55), so a witness never changes them.
__device__ __forceinline__ uint4 fixed_of_quad(const QuadInfo& d, uint64_t ivw) {
  uint4 f = make_uint4(0, 0, 0, 0);
  switch (d.kind) {
    case K_CONST: {
      const uint32_t s = 1u << S_CONST;
      f = make_uint4(s | ((uint32_t)(ivw & 0xffffu) << 16), s | ((uint32_t)((ivw >> 16) & 0xffffu) << 16),
                     s | ((uint32_t)((ivw >> 32) & 0xffffu) << 16), s | ((uint32_t)(ivw >> 48) << 16));
      break;
    }
    case K_XOR24: if (d.q == 0) f.x = (1u << S_B1) | (1u << S_EFGH); break;
    case K_XOR63: if (d.q == 0) f.x = (1u << S_B2) | (1u << S_IJKL); break;
    case K_XOR3: if (d.q == 0) f.x = (1u << S_XOR3) | (1u << S_DIGEST); break;
    case K_PAD: break;
    default: if (d.q == 0) f.x = 1u << d.sel; break;  // INW, FMASK, XOR, ADD3, ADD2
  }
  return f;
}

}  // namespace b2f

// b2f_fused.hip -- the fused witness fill + constraint evaluation (b2f_fill_eval_dev).
//
// One persistent kernel assigns every cell of a batch (the fill kernel's work) and checks the
// trace it assigns (the eval kernel's work) before the cells leave the CU: each cell is written
// to HBM once and never read back. The result is the same trace, h' and verdict as
// b2f_fill_dev followed by b2f_eval_dev -- MockProver::run (synthesize, blake2f.rs:301) then
// verify (:302) over the same assignment -- at the HBM cost of the fill alone.
//
// Work layout: the WAVE is the unit. The trace is cut at block boundaries into tiles: per
// instance the init region (41 quads), one tile per half-round (4 G's = 52 quads; every gate
// block lies inside its G) and the final region (16 quads); then 64-quad tiles of the zero rows
// past the last instance. Tile j of instance i is global tile T_i + j with
// T_i = 2 sum(rounds before i) + 2 i (tile_desc_kernel writes {i, j, rounds, state index}).
// Tiles are dealt round-robin to the waves of a persistent grid (wave w takes w, w + W, ...),
// so at any moment the chip writes one narrow band of every column -- the fill kernel's store
// pattern (tools/store_probe.hip: 8.8 ms for the 60 GB 2^18 x 12-round trace, the same as
// 1024-row workgroup tiles; per-wave instance ownership drops to 12.1 ms).
//
// A wave assigns its tile (lane = quad), stages the cells into its own LDS region, stores them
// (16-byte non-temporal column stores) and then checks the tile out of LDS: lookups per row,
// every canonical gate block by kind (one evaluator per lane group: adds, XORs, XOR24 and
// XOR63 limbs), every copy constraint whose operand cell lies in the tile, the fixed column
// against the keygen structure. No workgroup barrier: waves never share data. Copy sources in
// earlier tiles are the previous half-round's G outputs and the init region's words; the wave
// recomputes them from the producer side -- the previous half-round's four G chains from the
// record kernel's state at ITS start (four otherwise idle lanes), the init words from the input
// record -- so every copy compares the staged operand cell with the value its producer
// assigned (the test-only injection is applied to recomputed cells too). A selector row whose
// gate would read past the tile (only a corrupted fixed column has one) goes to a short list
// that a follow-up kernel evaluates on the written trace (deferred_gates_kernel).
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "../../include/b2f.h"
#include "b2f_common.h"

namespace {

constexpr int FW = 64;            // lanes per wave
constexpr int WAVES = 4;          // waves per workgroup
constexpr int STR = 208;          // staged rows per column (a half-round tile)
constexpr uint32_t HR_Q = 52, INIT_Q = 41, FINAL_Q = 16, PAD_Q = 64;
constexpr int NSTAGE = 9;         // staged columns a_0 .. a_8

// per-wave LDS region (words): a_0..a_8 [9][STR], per-quad canonical flag and row-0 a_9,
// the 16 producer words (u64)
constexpr int S_CANON = NSTAGE * STR;
constexpr int S_A9 = S_CANON + HR_Q;
constexpr int S_PROD = S_A9 + HR_Q;
constexpr int WAVE_WORDS = S_PROD + 32;
static_assert(S_PROD % 2 == 0 && WAVE_WORDS % 4 == 0 && STR % 4 == 0, "aligned wave carve");

// Copy checks of a half-round tile whose source is not a message word: 64 per G, 256 per tile,
// per parity of the half-round (column / diagonal G's). Entry (u32):
//   bits 0-7 operand row in the tile, 8-9 operand column (a_3, a_4, a_5),
//   bit 10 source kind: 0 a staged cell of this tile (bits 11-18 row, 19-20 column as W index
//   a_1 a_2 a_7 a_8), 1 a state word as the half-round starts (bits 11-14 word, 15-16 limb,
//   17 spread). The 8 message-word copies per G are checked apart (their source depends on
//   SIGMA[r mod 10]).
constexpr int HR_CHECKS = 256;
struct HrChecks {
  uint32_t e[2][HR_CHECKS];
};
constexpr HrChecks make_hr_checks() {
  HrChecks T{};
  DescTable D = make_desc();
  for (uint32_t par = 0; par < 2; par++) {
    uint32_t idx = 0;
    for (uint32_t gg = 0; gg < 4; gg++) {
      const uint32_t g = gg + 4 * par;
      for (uint32_t p = 0; p < G_QUADS; p++)
        for (uint32_t j = 0; j < 4; j++)
          for (uint32_t c = 0; c < 3; c++) {
            const uint32_t d = D.d[p][j][c], kind = d & 3u;
            if (kind == 0 || kind == 3) continue;
            uint32_t e = (52 * gg + 4 * p + j) | (c << 8);
            if (kind == 1) {
              e |= (52 * gg + ((d >> 2) & 63u)) << 11;
              e |= wc_of((d >> 8) & 15u) << 19;
            } else {
              e |= 1u << 10;
              e |= (uint32_t)kGidx[g][(d >> 2) & 3u] << 11;
              e |= ((d >> 4) & 3u) << 15;
              e |= ((d >> 6) & 1u) << 17;
            }
            if (idx < HR_CHECKS) T.e[par][idx] = e;
            idx++;
          }
    }
    if (idx != HR_CHECKS) T.e[0][0] = 0xffffffffu;
  }
  return T;
}
constexpr bool hr_checks_ok() { return make_hr_checks().e[0][0] != 0xffffffffu; }
static_assert(hr_checks_ok(), "64 non-message copy checks per G");
__constant__ HrChecks c_hr_checks = make_hr_checks();

// Rows each gate reads past its selector row, minus one (LAYOUT.md §4): abcd 4, efgh 11,
// ijkl 7, a1 4, b1 12, c1 4, d1 8, a2 4, b2 8, c2 4, d2 8, digest 7, xor 8, xor3 8, const 1,
// fmask 4.
constexpr uint64_t gate_span() {
  const uint32_t rows[16] = {4, 11, 7, 4, 12, 4, 8, 4, 8, 4, 8, 7, 8, 8, 1, 4};
  uint64_t s = 0;
  for (int i = 0; i < 16; i++) s |= (uint64_t)(rows[i] - 1) << (4 * i);
  return s;
}
constexpr uint64_t kGateSpan = gate_span();
__device__ __forceinline__ uint32_t span_of(uint32_t sel) {  // max over the set bits
  uint32_t m = 0;
  for (uint32_t b = sel; b; b &= b - 1) {
    const uint32_t s = (uint32_t)(kGateSpan >> (4 * __builtin_ctz(b))) & 15u;
    m = s > m ? s : m;
  }
  return m;
}

// (a, b, c, d) word indices of G g packed in bytes (column G's g < 4, diagonal g >= 4)
__device__ __forceinline__ uint32_t gidx_word(uint32_t g) {
  const uint32_t gl = g & 3u, dg = g >> 2;
  return gl | ((4 + ((gl + dg) & 3u)) << 8) | ((8 + ((gl + 2 * dg) & 3u)) << 16) |
         ((12 + ((gl + 3 * dg) & 3u)) << 24);
}
// staging column of a W index (a_1 a_2 a_7 a_8)
__device__ __forceinline__ int wcol(uint32_t wc) { return wc < 2 ? (int)wc + 1 : (int)wc + 5; }

// shared per-workgroup LDS (words)
constexpr int L_ACC = 0;                        // 16 gates, lookup, copy, fixed, pad, first u64
constexpr int L_IV = 24;                        // IV, 8 x u64
constexpr int L_SG = L_IV + 16;                 // SIGMA [10][16] bytes
constexpr int L_ROWS = L_SG + 40;               // RowTable (make_rows)
constexpr int L_CT = (L_ROWS + ROW_TABLE_WORDS + 3) & ~3;  // HrChecks
constexpr int L_WAVE = L_CT + 2 * HR_CHECKS;
constexpr int L_WORDS = L_WAVE + WAVES * WAVE_WORDS;
static_assert(L_IV % 2 == 0 && L_WAVE % 4 == 0, "aligned carve");
static_assert(L_WORDS * 4 * 4 <= 160 * 1024, "four fused workgroups per CU");

// The staged cells of one wave's tile: column c (a_0 .. a_8) at tile row r.
struct WaveTile {
  const uint32_t* S;
  __device__ __forceinline__ uint32_t at(int c, uint32_t r) const { return S[c * STR + r]; }
  __device__ __forceinline__ uint4 quad(int c, uint32_t r) const {
    return *reinterpret_cast<const uint4*>(S + c * STR + r);
  }
};

// The written trace from row `base` on, cells past the trace reading 0 (LAYOUT.md §6).
struct GlobalRows {
  const uint32_t* adv;
  uint64_t total, base;
  __device__ __forceinline__ uint32_t at(int c, uint32_t r) const {
    const uint64_t g = base + r;
    return g < total ? adv[(uint64_t)c * total + g] : 0u;
  }
  __device__ __forceinline__ uint4 quad(int c, uint32_t r) const {
    return make_uint4(at(c, r), at(c, r + 1), at(c, r + 2), at(c, r + 3));
  }
};

// Test-only fault injection (b2f_debug_inject): XOR `mask` into one cell as it is assigned,
// so the trace written and the trace checked are the corrupted one.
struct Inject {
  uint64_t row;   // ~0: none
  uint32_t col;   // 0..9 advice a_col, 10 fixed
  uint32_t mask;
};
__device__ __forceinline__ uint32_t inj_at(const Inject& inj, uint64_t row, uint32_t col) {
  return (row == inj.row && col == inj.col) ? inj.mask : 0u;
}

enum : uint32_t { T_INIT = 0, T_HR, T_FINAL, T_PAD };

struct TileDesc {  // 16 B, written by tile_desc_kernel
  uint32_t inst, j, rounds, st;
};

// A tile as the wave sees it (wave-uniform).
struct Ctx {
  uint32_t kind, inst, rounds, hr, nq;
  uint64_t off, st, row0;  // instance offset, its first state index, first row of the tile
};

__device__ __forceinline__ Ctx make_ctx(uint64_t t, uint64_t t_inst, const uint4& raw,
                                        uint64_t used_rows, uint64_t total_rows) {
  Ctx c;
  c.inst = __builtin_amdgcn_readfirstlane(raw.x);
  const uint32_t j = __builtin_amdgcn_readfirstlane(raw.y);
  c.rounds = __builtin_amdgcn_readfirstlane(raw.z);
  c.st = __builtin_amdgcn_readfirstlane(raw.w);
  c.off = 20ull * c.inst + 208ull * c.st;  // off_i = 228 i + 416 sum(rounds), st = 2 sum + i
  c.hr = 0;
  if (t >= t_inst) {
    c.kind = T_PAD;
    c.row0 = used_rows + (uint64_t)PAD_Q * 4 * (t - t_inst);
    const uint64_t left = c.row0 < total_rows ? (total_rows - c.row0) >> 2 : 0;
    c.nq = (uint32_t)(left < PAD_Q ? left : PAD_Q);
  } else if (j == 0) {
    c.kind = T_INIT;
    c.row0 = c.off;
    c.nq = INIT_Q;
  } else if (j <= 2 * c.rounds) {
    c.kind = T_HR;
    c.hr = j - 1;
    c.row0 = c.off + INIT_ROWS + 208ull * c.hr;
    c.nq = HR_Q;
  } else {
    c.kind = T_FINAL;
    c.row0 = c.off + INIT_ROWS + (uint64_t)ROUND_ROWS * c.rounds;
    c.nq = FINAL_Q;
  }
  return c;
}

// Operand words of one lane for a tile (loaded one tile ahead of their use):
//   quad lanes: the quad's operands (half-round: its G's a b c d at the half-round start and
//   message words x y; init: the input word it decomposes; final: h_i, v_i, v_{i+8});
//   producer lanes (the four lanes after the quads of half-round and final tiles): the G chain
//   operands of the previous half-round, whose outputs are this tile's state-word copy
//   sources, or for the first half-round / a 0-round final the initial work vector words;
//   aux (half-round lanes < 32): the message word of the lane's message-copy check.
struct Ops {
  uint64_t w[6];
  uint64_t aux;
};

__device__ __forceinline__ Ops load_ops(const Ctx& c, uint32_t lane, const b2f_input* __restrict__ in,
                                        const uint64_t* __restrict__ rec, const uint8_t* Sg,
                                        const uint64_t* IV) {
  Ops o;
#pragma unroll
  for (int k = 0; k < 6; k++) o.w[k] = 0;
  o.aux = 0;
  if (c.kind == T_PAD) return o;
  const b2f_input* x = in + c.inst;
  const uint64_t* fw = reinterpret_cast<const uint64_t*>(&x->rounds);  // rounds | f << 32
  if (c.kind == T_INIT) {
    if (lane < INIT_Q) {
      const uint64_t* p = fw;
      bool ld = true;
      if (lane < 26) p = lane < 8 ? x->h + lane : (lane < 24 ? x->m + (lane - 8) : x->t + (lane - 24));
      else if (lane < 35) ld = lane == 26;  // fmask reads the f word; CONST quads read nothing
      else p = ((lane - 35) >> 1) < 2 ? x->t + ((lane - 35) >> 1) : fw;
      o.w[0] = ld ? *p : 0ull;
    }
    return o;
  }
  const uint32_t npq = c.kind == T_HR ? HR_Q : FINAL_Q;
  const uint64_t* st0 = rec + 16ull * c.st;
  if (lane < npq) {
    if (c.kind == T_HR) {
      const uint32_t gg = lane / G_QUADS, g = gg + 4 * (c.hr & 1u);
      const uint64_t* s = st0 + 16ull * c.hr;
      const uint32_t gi = gidx_word(g);
      const uint8_t* sg = Sg + 16 * ((c.hr >> 1) % 10) + 2 * g;
      o.w[0] = s[gi & 15u];
      o.w[1] = s[(gi >> 8) & 15u];
      o.w[2] = s[(gi >> 16) & 15u];
      o.w[3] = s[(gi >> 24) & 15u];
      o.w[4] = x->m[sg[0]];
      o.w[5] = x->m[sg[1]];
    } else {
      const uint32_t a = lane >> 1;
      const uint64_t* fin = st0 + 16ull * (2ull * c.rounds);
      o.w[0] = x->h[a];
      o.w[1] = fin[a];
      o.w[2] = fin[a + 8];
    }
  } else if (lane < npq + 4) {
    const uint32_t gg = lane - npq;
    const bool first = c.kind == T_HR ? c.hr == 0 : c.rounds == 0;
    if (first) {  // the initial work vector words of column G gg: v_gg, v_gg+4, IV_gg, v_gg+12
      o.w[0] = x->h[gg];
      o.w[1] = x->h[gg + 4];
      o.w[2] = IV[gg];
      const uint64_t tw = gg < 2 ? x->t[gg] : (gg == 2 ? ((*fw >> 32) ? ~0ull : 0ull) : 0ull);
      o.w[3] = IV[gg + 4] ^ tw;
    } else {
      const uint32_t hp = c.kind == T_HR ? c.hr - 1 : 2 * c.rounds - 1;
      const uint32_t g = gg + 4 * (hp & 1u);
      const uint64_t* s = st0 + 16ull * hp;
      const uint32_t gi = gidx_word(g);
      const uint8_t* sg = Sg + 16 * ((hp >> 1) % 10) + 2 * g;
      o.w[0] = s[gi & 15u];
      o.w[1] = s[(gi >> 8) & 15u];
      o.w[2] = s[(gi >> 16) & 15u];
      o.w[3] = s[(gi >> 24) & 15u];
      o.w[4] = x->m[sg[0]];
      o.w[5] = x->m[sg[1]];
    }
  }
  if (c.kind == T_HR && lane < 32) {
    const uint32_t g = (lane >> 3) + 4 * (c.hr & 1u), which = (lane >> 2) & 1u;
    o.aux = x->m[Sg[16 * ((c.hr >> 1) % 10) + 2 * g + which]];
  }
  return o;
}

// MODE (diagnostics; the product launches FZ_FULL, with FZ_INJECT only under the test hook)
#ifndef B2F_FUSED_WAVES
#define B2F_FUSED_WAVES 2  // waves per SIMD the fused kernel is compiled for (VGPR budget)
#endif
enum { FZ_LOOKUP = 1, FZ_STORE = 2, FZ_INJECT = 4, FZ_GATES = 8, FZ_COPIES = 16, FZ_FULL = 27 };

template <int MODE>
__global__ void __launch_bounds__(FW * WAVES, B2F_FUSED_WAVES)
fused_kernel(const b2f_input* __restrict__ in, uint32_t n, const uint64_t* __restrict__ off,
             uint64_t total_rows, const uint64_t* __restrict__ rec, uint32_t* __restrict__ adv,
             uint32_t* __restrict__ fixed, const TileDesc* __restrict__ desc,
             b2f_eval_report* __restrict__ rep, const int* __restrict__ status, Inject inj,
             uint64_t* __restrict__ defer, uint32_t defer_cap) {
  __shared__ __attribute__((aligned(16))) uint32_t L[L_WORDS];
  const int tid = threadIdx.x;
  const uint32_t lane = (uint32_t)tid & 63u, wv = (uint32_t)tid >> 6;
  if (tid < 22) L[L_ACC + tid] = 0;
  if (tid == 22) *reinterpret_cast<uint64_t*>(L + L_ACC + 20) = ~0ull;
  if (tid < 16) L[L_IV + tid] = reinterpret_cast<const uint32_t*>(c_iv)[tid];
  if (tid < 40) L[L_SG + tid] = reinterpret_cast<const uint32_t*>(c_sigma)[tid];
  if (tid < ROW_TABLE_WORDS) L[L_ROWS + tid] = (&c_rows.r[0][0])[tid];
  for (int i = tid; i < 2 * HR_CHECKS; i += FW * WAVES) L[L_CT + i] = (&c_hr_checks.e[0][0])[i];
  __syncthreads();
  EvalAcc A{L + L_ACC};
  const uint64_t* IV = reinterpret_cast<const uint64_t*>(L + L_IV);
  const uint8_t* Sg = reinterpret_cast<const uint8_t*>(L + L_SG);
  const uint32_t* rows = L + L_ROWS;
  uint32_t* S = L + L_WAVE + wv * WAVE_WORDS;  // this wave's staging
  const WaveTile T{S};
  uint64_t* prod = reinterpret_cast<uint64_t*>(S + S_PROD);

  if (*status == 0) {  // the record kernel accepted the layout
    const uint64_t used_rows = off[n];
    const uint64_t t_inst = (used_rows - (uint64_t)FIXED_ROWS * n) / 208 + 2ull * n;
    const uint64_t t_all = t_inst + ((total_rows - used_rows) / 4 + PAD_Q - 1) / PAD_Q;
    const uint64_t W = (uint64_t)gridDim.x * WAVES;
    uint64_t t = (uint64_t)blockIdx.x * WAVES + wv;

    auto raw_desc = [&](uint64_t tt) -> uint4 {
      return tt < t_inst ? *reinterpret_cast<const uint4*>(desc + tt) : make_uint4(0, 0, 0, 0);
    };
    // software pipeline: operands one tile ahead, descriptors two tiles ahead (every load of
    // an iteration is issued before its stores: vmcnt retires loads and stores in order)
    Ctx c = make_ctx(t, t_inst, raw_desc(t), used_rows, total_rows);
    Ops P{};
    if (t < t_all) P = load_ops(c, lane, in, rec, Sg, IV);
    uint4 dn = raw_desc(t + W);
    for (; t < t_all; t += W) {
      const Ctx cn = make_ctx(t + W, t_inst, dn, used_rows, total_rows);
      Ops Pn{};
      if (t + W < t_all) Pn = load_ops(cn, lane, in, rec, Sg, IV);
      dn = raw_desc(t + 2 * W);

      // ---- assign this lane's quad
      const uint32_t nq = c.nq;
      const bool qlane = lane < nq;
      const uint64_t qrow = c.row0 + 4ull * lane;  // this lane's first row
      Quad Q;
      zero(Q);
      uint32_t p = 0;  // quad position inside its G (half-round tiles)
      if (c.kind == T_HR) {
        p = lane - G_QUADS * (lane / G_QUADS);
        quad_round(Q, P.w[0], P.w[1], P.w[2], P.w[3], P.w[4], P.w[5], p, rows);
      } else if (c.kind == T_INIT) {
        QuadOps qo;
        qo.w[0] = P.w[0];
#pragma unroll
        for (int k = 1; k < 6; k++) qo.w[k] = 0;
        qo.lq = lane < INIT_Q ? lane : 0;
        qo.rounds = c.rounds;
        quad_cells_ops(Q, qo, IV);
      } else if (c.kind == T_FINAL) {
        q_xor3(Q, P.w[0], P.w[1], P.w[2], lane & 1u);
      }
      if (!qlane) zero(Q);
      if (MODE & FZ_INJECT) {
        if (qlane && (inj.row >> 2) == (qrow >> 2)) {
#pragma unroll
          for (int j = 0; j < 4; j++) {
            if ((uint32_t)j != (uint32_t)(inj.row & 3)) continue;
#pragma unroll
            for (int cc = 0; cc < 10; cc++)
              if ((uint32_t)cc == inj.col) Q.c[cc][j] ^= inj.mask;
            if (inj.col == 10) Q.fx[j] ^= inj.mask;
          }
        }
      }
      // producer lanes: the outputs (a2, b2, c2, d2) of their G, or the initial words
      const uint32_t npq = c.kind == T_HR ? HR_Q : FINAL_Q;
      if ((c.kind == T_HR || c.kind == T_FINAL) && lane >= npq && lane < npq + 4) {
        const uint32_t gg = lane - npq;
        const bool first = c.kind == T_HR ? c.hr == 0 : c.rounds == 0;
        const uint32_t hp = c.kind == T_HR ? c.hr - 1 : 2 * c.rounds - 1;
        const uint32_t g = first ? gg : gg + 4 * (hp & 1u);
        uint64_t o0 = P.w[0], o1 = P.w[1], o2 = P.w[2], o3 = P.w[3];
        if (!first) {
          const uint64_t a1 = P.w[0] + P.w[1] + P.w[4];
          const uint64_t d1 = rotr64(P.w[3] ^ a1, 32);
          const uint64_t c1 = P.w[2] + d1;
          const uint64_t b1 = rotr64(P.w[1] ^ c1, 24);
          o0 = a1 + b1 + P.w[5];
          o3 = rotr64(d1 ^ o0, 16);
          o2 = c1 + o3;
          o1 = rotr64(b1 ^ o2, 63);
        }
        const uint32_t gi = gidx_word(g);
        prod[gi & 15u] = o0;
        prod[(gi >> 8) & 15u] = o1;
        prod[(gi >> 16) & 15u] = o2;
        prod[(gi >> 24) & 15u] = o3;
      }
      // ---- stage (every tile kind but the zero tail), then store
      const bool staged = c.kind != T_PAD;
      bool canon = false;
      if (staged && qlane) {
#pragma unroll
        for (int cc = 0; cc < NSTAGE; cc++)
          *reinterpret_cast<uint4*>(S + cc * STR + 4 * lane) = make_uint4(Q.c[cc][0], Q.c[cc][1], Q.c[cc][2], Q.c[cc][3]);
        if (c.kind == T_HR) {
          canon = (Q.fx[0] & 0xffffu) == expected_sel(p) && ((Q.fx[1] | Q.fx[2] | Q.fx[3]) & 0xffffu) == 0;
          S[S_CANON + lane] = canon ? 1u : 0u;
          S[S_A9 + lane] = Q.c[A9][0];
        }
      }
      if ((MODE & FZ_STORE) && qlane) {
#pragma unroll
        for (int cc = 0; cc < 11; cc++) {
          const u32x4 v = cc < 10 ? u32x4{Q.c[cc][0], Q.c[cc][1], Q.c[cc][2], Q.c[cc][3]}
                                  : u32x4{Q.fx[0], Q.fx[1], Q.fx[2], Q.fx[3]};
          __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>((cc < 10 ? adv + (uint64_t)cc * total_rows : fixed) + qrow));
        }
      }
      // the wave's LDS writes are complete and ordered before its reads below
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();

      // ---- lookups and the fixed column of this lane's quad
      if (qlane) {
        uint4 q0, q1, q2;
        if (staged) {
          q0 = T.quad(A0, 4 * lane);
          q1 = T.quad(A1, 4 * lane);
          q2 = T.quad(A2, 4 * lane);
        } else {
          q0 = make_uint4(Q.c[A0][0], Q.c[A0][1], Q.c[A0][2], Q.c[A0][3]);
          q1 = make_uint4(Q.c[A1][0], Q.c[A1][1], Q.c[A1][2], Q.c[A1][3]);
          q2 = make_uint4(Q.c[A2][0], Q.c[A2][1], Q.c[A2][2], Q.c[A2][3]);
        }
        if (MODE & FZ_LOOKUP) {
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const uint32_t tg = comp(q0, j), de = comp(q1, j), sp = comp(q2, j);
            if (!(de < 65536u && tg == tag16(de) && sp == spread16(de & 0xffffu)))
              A.fail(qrow + j, B2F_CODE_LOOKUP);
          }
        }
        if (MODE & FZ_GATES) {
          uint4 xf = make_uint4(0, 0, 0, 0);
          if (c.kind == T_HR) {
            xf.x = expected_sel(p);
          } else if (c.kind != T_PAD) {
            const QuadInfo d = decode_quad((uint32_t)((qrow - c.off) >> 2), c.rounds);
            xf = fixed_of_quad(d, d.kind == K_CONST ? IV[d.a & 7u] : 0ull);
          }
          if ((Q.fx[0] ^ xf.x) | (Q.fx[1] ^ xf.y) | (Q.fx[2] ^ xf.z) | (Q.fx[3] ^ xf.w)) {
#pragma unroll
            for (int j = 0; j < 4; j++)
              if (Q.fx[j] != comp(xf, j)) A.fail(qrow + j, B2F_CODE_FIXED);
          }
        }
      }

      // ---- gates
      if (MODE & FZ_GATES) {
        uint32_t bits = 0;  // XOR24 / XOR63 limb lanes (DPP quad OR below: all lanes active)
        const uint32_t kgg = (lane < 40 ? lane - 24 : lane - 40) >> 2, kk = lane & 3u;
        const uint32_t krow = 52 * kgg + (lane < 40 ? 16u : 44u);
        bool ktake = false;
        if (c.kind == T_HR) {
          if (lane < 16) {  // adds: a1 +0, c1 +12, a2 +28, c2 +40
            const uint32_t gg = lane >> 2, w = lane & 3u;
            const uint32_t r = 52 * gg + (w == 0 ? 0u : w == 1 ? 12u : w == 2 ? 28u : 40u);
            if (S[S_CANON + (r >> 2)] && !g_add(T, r, S[S_A9 + (r >> 2)], (w & 1u) == 0))
              A.fail_gates(c.row0 + r, 1u << (w == 0 ? S_A1 : w == 1 ? S_C1 : w == 2 ? S_A2 : S_C2));
          } else if (lane < 24) {  // XORs: d1 +4, d2 +32
            const uint32_t gg = (lane - 16) >> 1, w = lane & 1u;
            const uint32_t r = 52 * gg + (w ? 32u : 4u);
            if (S[S_CANON + (r >> 2)] && !g_xor(T, r, false)) A.fail_gates(c.row0 + r, 1u << (w ? S_D2 : S_D1));
          } else if (lane < 56) {  // XOR24 (b1 + efgh) / XOR63 (b2 + ijkl) limbs
            ktake = S[S_CANON + (krow >> 2)] != 0;
            if (ktake) bits = lane < 40 ? g_xor24_limb(T, krow, kk) : g_xor63_limb(T, krow, kk);
          }
        }
        bits = quad_or(bits);
        if (ktake && kk == 0 && bits) {
          const bool x24 = lane < 40;
          A.fail_gates(c.row0 + krow, ((bits & 1u) ? 1u << (x24 ? S_B1 : S_B2) : 0u) |
                                          ((bits & 2u) ? 1u << (x24 ? S_EFGH : S_IJKL) : 0u));
        }
        // every selector row the kind lanes do not take: init / final blocks, any row of a
        // non-canonical quad (a corrupted fixed column), the zero tail
        if (qlane && !(c.kind == T_HR && canon)) {
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const uint32_t k0 = Q.fx[j], sel = k0 & 0xffffu;
            if (!sel) continue;
            const uint32_t r = 4 * lane + j;
            if (staged && r + span_of(sel) < 4 * nq) {
              uint32_t failed;
              if (sel == (1u << S_CONST)) failed = T.at(A1, r) == (k0 >> 16) ? 0u : sel;
              else failed = row_gates(T, sel, r, Q.c[A9][j], k0);
              if (failed) A.fail_gates(qrow + j, failed);
            } else {  // the gate reads past this tile: evaluated on the written trace
              const uint64_t slot = atomicAdd((unsigned long long*)defer, 1ull);
              if (slot < defer_cap) defer[1 + slot] = qrow + j;
            }
          }
        }
      }

      // ---- copies
      if (MODE & FZ_COPIES) {
        if (c.kind == T_HR) {
          const uint32_t* ct = L + L_CT + (c.hr & 1u) * HR_CHECKS;
#pragma unroll
          for (int it = 0; it < HR_CHECKS / FW; it++) {
            const uint32_t e = ct[it * FW + lane];
            const uint32_t dr = e & 255u, dc = (e >> 8) & 3u;
            const uint32_t dv = T.at(A3 + (int)dc, dr);
            uint32_t sv;
            if (!((e >> 10) & 1u)) {
              sv = T.at(wcol((e >> 19) & 3u), (e >> 11) & 255u);
            } else {
              const uint32_t w = (e >> 11) & 15u, k = (e >> 15) & 3u, sp = (e >> 17) & 1u;
              const uint32_t lv = limb(prod[w], k);
              sv = sp ? spread16(lv) : lv;
              if (MODE & FZ_INJECT) {
                uint32_t col = 0;
                const uint32_t sr = state_src(w, k, sp, c.hr, col);
                sv ^= inj_at(inj, c.off + sr, col);
              }
            }
            if (dv != sv) A.fail(c.row0 + dr, B2F_CODE_COPY);
          }
          if (lane < 32) {  // message words: a1 (x) at +0 and a2 (y) at +28 of every G
            const uint32_t gg = lane >> 3, which = (lane >> 2) & 1u, k = lane & 3u;
            const uint32_t dr = 52 * gg + (which ? 28u : 0u) + k;
            const uint32_t dv = T.at(A5, dr);
            uint32_t sv = limb(P.aux, k);
            if (MODE & FZ_INJECT) {
              const uint32_t g = gg + 4 * (c.hr & 1u);
              const uint32_t mj = Sg[16 * ((c.hr >> 1) % 10) + 2 * g + which];
              sv ^= inj_at(inj, c.off + 32 + 4 * mj + k, A1);
            }
            if (dv != sv) A.fail(c.row0 + dr, B2F_CODE_COPY);
          }
        } else if (c.kind == T_INIT) {
          if (lane < 24) {  // v12 = IV4 ^ t0, v13 = IV5 ^ t1, v14 = IV6 ^ fmask
            const uint32_t a = lane >> 3, k = (lane >> 1) & 3u, op = lane & 1u;
            const uint32_t dr = 140 + 8 * a + 2 * k;
            const uint32_t sr = op == 0 ? 108 + 4 * (4 + a) + k : (a < 2 ? 96 + 4 * a + k : 104 + k);
            if (T.at(op ? A4 : A3, dr) != T.at(A2, sr)) A.fail(c.row0 + dr, B2F_CODE_COPY);
          }
        } else if (c.kind == T_FINAL && qlane) {  // h' = h ^ v_i ^ v_{i+8}
          const uint32_t a = lane >> 1;
#pragma unroll
          for (int kk2 = 0; kk2 < 2; kk2++) {
            const uint32_t k = 2 * (lane & 1u) + kk2, dr = 8 * a + 2 * k;
            uint32_t cv = 0, cu = 0;
            const uint32_t vs = state_src(a, k, 1, 2 * c.rounds, cv);
            const uint32_t us = state_src(a + 8, k, 1, 2 * c.rounds, cu);
            uint32_t sh = spread16(limb(P.w[0], k));
            uint32_t sv = spread16(limb(prod[a], k));
            uint32_t su = spread16(limb(prod[a + 8], k));
            if (MODE & FZ_INJECT) {
              sh ^= inj_at(inj, c.off + 4 * a + k, A2);
              sv ^= inj_at(inj, c.off + vs, cv);
              su ^= inj_at(inj, c.off + us, cu);
            }
            if (T.at(A3, dr) != sh) A.fail(c.row0 + dr, B2F_CODE_COPY);
            if (T.at(A4, dr) != sv) A.fail(c.row0 + dr, B2F_CODE_COPY);
            if (T.at(A5, dr) != su) A.fail(c.row0 + dr, B2F_CODE_COPY);
          }
        }
      }
      // the staging is rewritten by the next tile: its reads above must be done first
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      c = cn;
      P = Pn;
    }
  }
  __syncthreads();
  flush_report(A, rep, tid);
}

// Per-tile descriptors {instance, tile index inside it, rounds, first state index}: thread per
// instance, 2 rounds + 2 tiles each (init, half-rounds, final).
__global__ void tile_desc_kernel(const uint64_t* __restrict__ off, const b2f_input* __restrict__ in,
                                 uint32_t n, TileDesc* __restrict__ desc, const int* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || *status) return;
  const uint32_t rounds = in[i].rounds;
  const uint64_t st = 2 * ((off[i] - (uint64_t)FIXED_ROWS * i) / ROUND_ROWS) + i;
  const uint64_t t0 = st + i;
  for (uint32_t j = 0; j <= 2 * rounds + 1; j++) {
    TileDesc d;
    d.inst = i;
    d.j = j;
    d.rounds = rounds;
    d.st = (uint32_t)st;
    desc[t0 + j] = d;
  }
}

// Gates of selector rows the fused kernel deferred (their gate reads rows past the tile that
// assigned them), on the written trace: all selector bits of each listed row.
__global__ void deferred_gates_kernel(const uint32_t* __restrict__ adv, const uint32_t* __restrict__ fixed,
                                      uint64_t total_rows, const uint64_t* __restrict__ defer,
                                      uint32_t defer_cap, b2f_eval_report* __restrict__ rep,
                                      const int* __restrict__ status) {
  if (*status) return;
  const uint64_t cnt = defer[0] < defer_cap ? defer[0] : defer_cap;
  for (uint64_t k = threadIdx.x; k < cnt; k += blockDim.x) {
    const uint64_t row = defer[1 + k];
    const uint32_t k0 = fixed[row], sel = k0 & 0xffffu;
    const GlobalRows G{adv, total_rows, row};
    uint32_t failed;
    if (sel == (1u << S_CONST)) failed = G.at(A1, 0) == (k0 >> 16) ? 0u : sel;
    else failed = row_gates(G, sel, 0, adv[(uint64_t)A9 * total_rows + row], k0);
    for (uint32_t m = failed; m; m &= m - 1)
      atomicAdd((unsigned long long*)&rep->gate_failures[__builtin_ctz(m)], 1ull);
    if (failed)
      atomicMin((unsigned long long*)&rep->first_failure,
                (unsigned long long)((row << 8) | (uint32_t)__builtin_ctz(failed)));
  }
}

constexpr uint32_t DEFER_CAP = 4096;

}  // namespace

namespace b2f {

// Scratch of the fused path: tile descriptors for `tiles` instance tiles and the deferred row
// list (count + DEFER_CAP rows).
size_t fused_scratch_bytes(uint64_t tiles) { return tiles * sizeof(TileDesc) + 8 * (1 + DEFER_CAP); }
// Instance tiles of a batch of n instances in at most total_rows rows (an upper bound).
uint64_t fused_instance_tiles(uint64_t total_rows, uint64_t n) {
  return (total_rows - (uint64_t)FIXED_ROWS * n) / 208 + 2 * n;
}

// Launch the fused path (b2f_fill_eval_dev) after the record kernel: tile descriptors, the
// fused kernel, the deferred gates. `scratch` holds fused_scratch_bytes(tiles).
hipError_t launch_fill_eval(const b2f_input* d_in, uint32_t n, const uint64_t* d_off,
                            uint64_t total_rows, const uint64_t* rec, uint32_t* d_adv,
                            uint32_t* d_fixed, void* scratch, uint64_t tiles,
                            b2f_eval_report* d_rep, const int* d_status, uint64_t inj_row,
                            uint32_t inj_col, uint32_t inj_mask, int mode, int cu_count,
                            hipStream_t s) {
  TileDesc* desc = reinterpret_cast<TileDesc*>(scratch);
  uint64_t* defer = reinterpret_cast<uint64_t*>(desc + tiles);
  hipError_t e = hipMemsetAsync(defer, 0, 8, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(tile_desc_kernel, dim3((n + 255) / 256), dim3(256), 0, s, d_off, d_in, n, desc, d_status);
  Inject inj;
  inj.row = inj_row;
  inj.col = inj_col;
  inj.mask = inj_mask;
#ifndef B2F_DIAG
  mode = FZ_FULL;  // the product library launches the full kernel only
#endif
  if (inj_row != ~0ull) mode |= FZ_INJECT;
  // persistent grid: the workgroups that are resident at once (VGPRs and LDS bound them)
  static int per_cu = 0;
  if (!per_cu) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fused_kernel<FZ_FULL>, FW * WAVES, 0) !=
            hipSuccess || nb < 1)
      nb = 2;
    per_cu = nb;
  }
  const uint32_t grid = (uint32_t)(cu_count * per_cu);
  switch (mode) {
#define B2F_FUSED(M)                                                                          \
  case M:                                                                                     \
    hipLaunchKernelGGL(fused_kernel<M>, dim3(grid), dim3(FW * WAVES), 0, s, d_in, n, d_off,   \
                       total_rows, rec, d_adv, d_fixed, desc, d_rep, d_status, inj, defer,    \
                       DEFER_CAP);                                                            \
    break;
#ifdef B2F_DIAG
    B2F_FUSED(0) B2F_FUSED(2) B2F_FUSED(3) B2F_FUSED(10) B2F_FUSED(18) B2F_FUSED(8) B2F_FUSED(16)
#endif
    B2F_FUSED(FZ_FULL | FZ_INJECT)
    default: B2F_FUSED(FZ_FULL)
#undef B2F_FUSED
  }
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(deferred_gates_kernel, dim3(1), dim3(256), 0, s, d_adv, d_fixed, total_rows,
                     defer, DEFER_CAP, d_rep, d_status);
  return hipGetLastError();
}

}  // namespace b2f

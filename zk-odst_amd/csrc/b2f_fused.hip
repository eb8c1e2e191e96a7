// b2f_fused.hip -- the fused witness fill + constraint evaluation (b2f_fill_eval_dev).
//
// The launches assign every cell of a batch (the fill kernel's work) and check the trace they
// assign (the eval kernel's work) before the cells leave the CU: each cell is written to HBM
// once and never read back. The result is the same trace, h' and verdict as b2f_fill_dev
// followed by b2f_eval_dev -- MockProver::run (synthesize, blake2f.rs:301) then verify (:302)
// over the same assignment -- at the HBM cost of the fill alone.
//
// Work layout: the WAVE is the unit; a tile is a block-aligned piece of one instance, assigned
// lane = quad, staged in the wave's own LDS region, stored (16-byte non-temporal column stores,
// each 128-byte line by one store instruction) and checked out of LDS: lookups per row, every
// canonical gate block, every copy constraint whose operand cell lies in the tile, the fixed
// column against the keygen structure. No workgroup barrier: waves never share data.
//   fused_hr_kernel: the half-round tiles (4 G's = 52 quads, 96 % of the rows). A wave takes
//     whole instances and walks their half-rounds in order, carrying the state in LDS: the G
//     outputs of its previous tile are this tile's state words and the copy sources of its
//     state-word cells, so no tile reads a recorded state (the record kernel writes only the
//     two states per instance the edge launch reads).
//   fused_edge_kernel: per instance the init region (41 quads) and the final region (16
//     quads) in one wave tile, then 64-quad tiles of the zero rows past the last instance; the
//     final region's copy sources in the last half-round are recomputed from the recorded state
//     at its start (four otherwise idle lanes).
// Checks are 32-bit identities that assume the ranges the other checks of the same pass
// establish, so a clean pass proves a clean tile; a flagged tile is re-checked exactly (the
// eval kernel's counters, first failing row). A selector row whose gate would read past the
// tile (only a corrupted fixed column has one) goes to a short list that a follow-up kernel
// evaluates on the written trace (deferred_gates_kernel).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>

#include "../../include/b2f.h"
#include "b2f_common.h"

typedef int32_t b2f_i32x4 __attribute__((ext_vector_type(4)));
// the raw buffer store intrinsic (declared as CK's amd_buffer_addressing.hpp does)
__device__ void b2f_raw_buffer_store_v4(b2f_i32x4 data, b2f_i32x4 rsrc, int voffset, int soffset,
                                        int aux) __asm("llvm.amdgcn.raw.buffer.store.v4i32");

namespace {

using i32x4 = b2f_i32x4;
constexpr int FW = 64;            // lanes per wave
constexpr int WAVES = 4;          // waves per workgroup
constexpr int STR = 208;          // staged rows per column (a half-round tile)
// the half-round launches' staging column: HPRE rows in front of the tile's 208 (the previous
// tile's last seven quads, which the fused kernel stores with its own: line ownership), so a
// column is HSTR = 236 words apart and row -HPRE .. -1 of column c is column c - 1's rows 208 ..
constexpr int HPRE = 28, HSTR = STR + HPRE;
constexpr uint32_t HR_Q = 52, INIT_Q = 41, FINAL_Q = 16, PAD_Q = 64;
constexpr int NSTAGE = 11;        // staged columns a_0 .. a_9 and the fixed column
constexpr int FXC = 10;           // staging column of the fixed cells

// per-wave LDS region (words): a_0..a_9, fixed [11][STR], the 16 producer words (u64), a
// per-quad flag "the quad's selector bits are the keygen structure's" (init / final tiles)
constexpr int S_PROD = NSTAGE * STR;
constexpr int S_CANON = S_PROD + 32;
constexpr int WAVE_WORDS = S_CANON + INIT_Q + 3;
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
template <int ST>
struct WaveTileS {
  const uint32_t* S;
  __device__ __forceinline__ uint32_t at(int c, uint32_t r) const { return S[c * ST + r]; }
  __device__ __forceinline__ uint4 quad(int c, uint32_t r) const {
    return *reinterpret_cast<const uint4*>(S + c * ST + r);
  }
};
using WaveTile = WaveTileS<STR>;   // the edge path's staging
using HrTile = WaveTileS<HSTR>;    // the half-round launches' staging

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

union TileDesc {  // 16 B, written by eval_desc_kernel
  struct {
    uint32_t inst, j, rounds, st;
  } f;
  uint4 v;
};

// A tile as the wave sees it (wave-uniform).
struct Ctx {
  uint32_t kind, inst, rounds, hr, nq;
  uint64_t off, st, row0;  // instance offset, its first state index, first row of the tile
};

// Operand words of one lane for a tile, loaded one tile ahead of their use. Every lane loads
// all seven words unconditionally from a per-lane address (a harmless in-bounds word where the
// lane has no use for one) and nothing is derived from them here: a conditional load or a use
// right after the load would make the wave wait for its outstanding stores (vmcnt retires
// loads and stores in order). Roles:
//   quad lanes: half-round: its G's a b c d at the half-round start, message words x y;
//     init: the input word the quad decomposes (h / m / t, the `rounds | f << 32` word);
//     final: h_i, v_i, v_{i+8}
//   producer lanes (the four lanes after the quads of half-round and final tiles): the
//     previous half-round's G operands (its outputs are this tile's state-word copy sources),
//     or for the first half-round / a 0-round final: h_g, h_{g+4}, -, the t / f word of v_{g+12}
//   w[6] (half-round lanes < 32): the message word of the lane's message-copy check
struct Ops {
  uint64_t w[7];
};

__device__ __forceinline__ Ops load_ops(const Ctx& c, uint32_t lane, const b2f_input* __restrict__ in,
                                        const uint64_t* __restrict__ rec, const uint8_t* Sg) {
  const b2f_input* x = in + (c.kind == T_PAD ? 0u : c.inst);
  const uint64_t* fw = reinterpret_cast<const uint64_t*>(&x->rounds);  // rounds | f << 32
  const uint64_t* p[7] = {fw, fw, fw, fw, fw, fw, fw};
  const uint32_t npq = c.kind == T_HR ? HR_Q : FINAL_Q;
  const uint64_t* st0 = rec + 16ull * c.st;
  if (c.kind == T_INIT) {
    if (lane < 26) p[0] = lane < 8 ? x->h + lane : (lane < 24 ? x->m + (lane - 8) : x->t + (lane - 24));
    else if (lane >= 35 && ((lane - 35) >> 1) < 2) p[0] = x->t + ((lane - 35) >> 1);
  } else if (c.kind == T_HR || c.kind == T_FINAL) {
    const bool prodl = lane >= npq && lane < npq + 4;
    const uint32_t gg = prodl ? lane - npq : lane / G_QUADS;
    const bool first = c.kind == T_HR ? c.hr == 0 : c.rounds == 0;
    if (c.kind == T_FINAL && !prodl) {
      const uint32_t a = (lane >> 1) & 7u;
      const uint64_t* fin = st0 + 16ull * (2ull * c.rounds);
      p[0] = x->h + a;
      p[1] = fin + a;
      p[2] = fin + a + 8;
    } else if (prodl && first) {
      p[0] = x->h + gg;
      p[1] = x->h + gg + 4;
      p[3] = gg < 2 ? x->t + gg : fw;
    } else if (lane < npq + 4) {
      const uint32_t h = prodl ? (c.kind == T_HR ? c.hr - 1 : 2 * c.rounds - 1) : c.hr;
      const uint32_t g = (gg & 3u) + 4 * (h & 1u);
      const uint64_t* s = st0 + 16ull * h;
      const uint32_t gi = gidx_word(g);
      const uint8_t* sg = Sg + 16 * ((h >> 1) % 10) + 2 * g;
      p[0] = s + (gi & 15u);
      p[1] = s + ((gi >> 8) & 15u);
      p[2] = s + ((gi >> 16) & 15u);
      p[3] = s + ((gi >> 24) & 15u);
      p[4] = x->m + sg[0];
      p[5] = x->m + sg[1];
    }
    if (c.kind == T_HR && lane < 32)
      p[6] = x->m + Sg[16 * ((c.hr >> 1) % 10) + 2 * ((lane >> 3) + 4 * (c.hr & 1u)) + ((lane >> 2) & 1u)];
  }
  Ops o;
#pragma unroll
  for (int k = 0; k < 7; k++) o.w[k] = *p[k];
  return o;
}

// The producer lanes' outputs: the four words of G g as the previous half-round ends (its
// chain a2 b2 c2 d2), or the initial work vector words of column G g, into the wave's prod.
__device__ __forceinline__ void producer_words(uint64_t* prod, const Ops& P, uint32_t pg, bool first,
                                               uint32_t hp, const uint64_t* IV) {
  uint64_t o0, o1, o2, o3;
  uint32_t g = pg;
  if (first) {
    o0 = P.w[0];
    o1 = P.w[1];
    o2 = IV[pg];
    const uint64_t tw = pg < 2 ? P.w[3] : (pg == 2 ? ((P.w[3] >> 32) ? ~0ull : 0ull) : 0ull);
    o3 = IV[pg + 4] ^ tw;
  } else {
    g = pg + 4 * (hp & 1u);
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

// MODE (diagnostics; the product launches FZ_FULL, with FZ_INJECT only under the test hook)
#ifndef B2F_FUSED_WAVES
// minimum waves per SIMD the half-round kernel is compiled for: 2, i.e. a VGPR ceiling of 256.
// The kernel allocates 159 VGPRs, which leaves room for 3 waves per SIMD, and the launch runs
// B2F_FUSED_HR_PER_CU = 3 workgroups (of 4 waves) per CU: 3 waves per SIMD. (Forcing a budget
// of 3 per SIMD at compile time is not needed while the allocation stays <= 168.)
#define B2F_FUSED_WAVES 2
#endif
#ifndef B2F_FUSED_HR_PER_CU
#define B2F_FUSED_HR_PER_CU 3  // half-round launch: workgroups per CU (at most what fits)
#endif
enum { FZ_LOOKUP = 1, FZ_STORE = 2, FZ_INJECT = 4, FZ_GATES = 8, FZ_COPIES = 16, FZ_FULL = 27,
       FZ_CLOCK = 128 };  // per-phase s_memtime totals per wave slot (diagnostics, b2f_debug_clock)

// Stores of a tile: raw buffer stores through a per-tile, per-column buffer resource whose
// range is the tile's quads, so every lane of the wave issues the same store instructions and
// the lanes past the tile's last quad are dropped by the range check. Straight-line stores keep
// the compiler's vmcnt bookkeeping exact: a branch that might skip a tile's stores would make
// every later wait for an older load wait for those stores too (vmcnt is in order).
#ifndef B2F_BUF_POLICY
#define B2F_BUF_POLICY 2  // non-temporal: at 3 workgroups per CU with line-owned stores 10.93 vs
                          // 11.24 ms (default write-back) / 11.27 (sc0), profiles/r03t_*; at 2 per
                          // CU before line ownership the default had been 2.9 % faster
#endif
constexpr int BUF_NT = B2F_BUF_POLICY;  // gfx94x/gfx950 cache-policy bits: 1 sc0, 2 non-temporal
#ifndef B2F_EDGE_BUF_POLICY
#define B2F_EDGE_BUF_POLICY 2  // the edge launch's region stores: non-temporal (690 vs 763 us)
#endif
constexpr int EDGE_NT = B2F_EDGE_BUF_POLICY;
__device__ __forceinline__ void tile_store(uint32_t* base, uint32_t nq, uint32_t lane, uint4 v) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const i32x4 rsrc = {(int32_t)(uint32_t)a, (int32_t)(uint32_t)(a >> 32), (int32_t)(nq * 16u), 0x00020000};
  b2f_raw_buffer_store_v4(i32x4{(int32_t)v.x, (int32_t)v.y, (int32_t)v.z, (int32_t)v.w}, rsrc,
                      (int)(16 * lane), 0, BUF_NT);
}

// One column of a quad at LDS word pointer `p`: the test-only injection, then staged.
template <int MODE>
__device__ __forceinline__ void emit_at(uint32_t* p, int col, uint64_t qrow, uint32_t v0, uint32_t v1,
                                        uint32_t v2, uint32_t v3, const Inject& inj) {
  if (MODE & FZ_INJECT) {
    if ((inj.row >> 2) == (qrow >> 2) && inj.col == (uint32_t)col) {
      const uint32_t j = (uint32_t)inj.row & 3u;
      v0 ^= j == 0 ? inj.mask : 0u;
      v1 ^= j == 1 ? inj.mask : 0u;
      v2 ^= j == 2 ? inj.mask : 0u;
      v3 ^= j == 3 ? inj.mask : 0u;
    }
  }
  *reinterpret_cast<uint4*>(p) = make_uint4(v0, v1, v2, v3);
}

// One column of this lane's quad: the test-only injection, then staged (wave LDS) or stored
// (16-byte non-temporal store; column 10 = the fixed column).
template <int MODE>
__device__ __forceinline__ void emit(uint32_t* S, int col, uint32_t lane, uint64_t qrow, uint32_t v0,
                                     uint32_t v1, uint32_t v2, uint32_t v3, uint32_t* adv,
                                     uint32_t* fixed, uint64_t total_rows, const Inject& inj,
                                     bool stage) {
  if (MODE & FZ_INJECT) {
    if ((inj.row >> 2) == (qrow >> 2) && inj.col == (uint32_t)col) {
      const uint32_t j = (uint32_t)inj.row & 3u;
      v0 ^= j == 0 ? inj.mask : 0u;
      v1 ^= j == 1 ? inj.mask : 0u;
      v2 ^= j == 2 ? inj.mask : 0u;
      v3 ^= j == 3 ? inj.mask : 0u;
    }
  }
  *reinterpret_cast<uint4*>(S + col * STR + 4 * lane) = make_uint4(v0, v1, v2, v3);
}

// Wait for the next tile's operand words here, before this tile's stores are issued: they were
// loaded at the top of the iteration, and the only older vector memory operations still in
// flight are the previous tile's stores, issued a whole tile ago. Waited on later (at their
// first use in the next iteration) they would also wait for this tile's stores (vmcnt is in
// order, and the compiler cannot count stores across the tile kinds' branches).
__device__ __forceinline__ void settle(const Ops& P) {
  asm volatile("" ::"v"(P.w[0]), "v"(P.w[1]), "v"(P.w[2]), "v"(P.w[3]), "v"(P.w[4]), "v"(P.w[5]),
               "v"(P.w[6]));
}

// The staged tile to HBM (every lane; see tile_store). Issued only after every use of the
// loaded operand words: a use after a store would wait for the store (vmcnt is in order).
template <int MODE>
__device__ __forceinline__ void store_staged(const uint32_t* S, uint32_t lane, uint32_t nq, uint64_t row0,
                                             uint32_t* adv, uint32_t* fixed, uint64_t total_rows) {
  if (!(MODE & FZ_STORE)) return;

  const uint32_t l = lane < nq ? lane : 0;
  // one column at a time (read, store): measured faster than reading 4, 6 or all 11 columns
  // ahead of their stores, whose burstier store stream wrote slower (same-process A/B)
#pragma unroll
  for (int col = 0; col < NSTAGE; col++)
    tile_store((col < 10 ? adv + (uint64_t)col * total_rows : fixed) + row0, nq, lane,
               *reinterpret_cast<const uint4*>(S + col * STR + 4 * l));
}

// A built quad (init / final / zero rows): every column emitted.
template <int MODE>
__device__ __forceinline__ void emit_quad(uint32_t* S, uint32_t lane, uint64_t qrow, const Quad& Q,
                                          uint32_t* adv, uint32_t* fixed, uint64_t total_rows,
                                          const Inject& inj, bool stage) {
#pragma unroll
  for (int cc = 0; cc < 10; cc++)
    emit<MODE>(S, cc, lane, qrow, Q.c[cc][0], Q.c[cc][1], Q.c[cc][2], Q.c[cc][3], adv, fixed, total_rows, inj, stage);
  emit<MODE>(S, FXC, lane, qrow, Q.fx[0], Q.fx[1], Q.fx[2], Q.fx[3], adv, fixed, total_rows, inj, stage);
}

// Lookups on the quad's four rows.
__device__ __forceinline__ void check_lookups(EvalAcc& A, uint4 q0, uint4 q1, uint4 q2, uint64_t qrow) {
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint32_t tg = comp(q0, j), de = comp(q1, j), sp = comp(q2, j);
    if (!(de < 65536u && tg == tag16(de) && sp == spread16(de & 0xffffu))) A.fail(qrow + j, B2F_CODE_LOOKUP);
  }
}

// The quad's fixed cells against the keygen structure.
__device__ __forceinline__ void check_fixed(EvalAcc& A, uint4 fx, uint4 xf, uint64_t qrow) {
  if ((fx.x ^ xf.x) | (fx.y ^ xf.y) | (fx.z ^ xf.z) | (fx.w ^ xf.w)) {
#pragma unroll
    for (int j = 0; j < 4; j++)
      if (comp(fx, j) != comp(xf, j)) A.fail(qrow + j, B2F_CODE_FIXED);
  }
}

// The selector rows of a quad whose selector bits are not the keygen structure's (only a
// corrupted fixed column, i.e. the test hook, has one): their gates -- every selector bit of
// the row, as the eval's per-quad path evaluates them -- go to the deferred list and are
// evaluated on the written trace after the kernel (deferred_gates_kernel).
__device__ __forceinline__ void defer_rows(uint4 fx, uint64_t qrow, uint64_t* defer, uint32_t defer_cap) {
#pragma unroll
  for (int j = 0; j < 4; j++) {
    if (!(comp(fx, j) & 0xffffu)) continue;
    const uint64_t slot = atomicAdd((unsigned long long*)defer, 1ull);
    if (slot < defer_cap) defer[1 + slot] = qrow + j;
  }
}

// An init or final tile, whole (about 4 % of the quads). The caller has settled the next
// tile's loads, so the stores here wait for nothing.
template <int MODE>
__device__ __forceinline__ void edge_tile(uint32_t* S, uint32_t* accw, const uint64_t* IV, const Inject inj,
                                       uint32_t* adv, uint32_t* fixed, uint64_t total_rows,
                                       uint64_t* defer, uint32_t defer_cap, const Ctx c, const Ops P,
                                       uint32_t lane) {
  EvalAcc A{accw};
  const WaveTile T{S};
  uint64_t* prod = reinterpret_cast<uint64_t*>(S + S_PROD);
  const uint32_t nq = c.nq;
  const bool qlane = lane < nq;
  const uint64_t qrow = c.row0 + 4ull * lane;
    // ---- the init region (h, m, t, fmask, IV, v12..v14) or the final XOR3 blocks
    Quad Q;
    zero(Q);
    if (c.kind == T_INIT) {
      QuadOps qo;
      qo.w[0] = P.w[0];
#pragma unroll
      for (int k = 1; k < 6; k++) qo.w[k] = 0;
      qo.lq = qlane ? lane : 0;
      qo.rounds = c.rounds;
      quad_cells_ops(Q, qo, IV);
    } else {
      q_xor3(Q, P.w[0], P.w[1], P.w[2], lane & 1u);
    }
    if (qlane) emit_quad<MODE>(S, lane, qrow, Q, adv, fixed, total_rows, inj, true);
    if (c.kind == T_FINAL && lane >= FINAL_Q && lane < FINAL_Q + 4)  // the final state
      producer_words(prod, P, lane - FINAL_Q, c.rounds == 0, 2 * c.rounds - 1, IV);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if ((MODE & FZ_COPIES) && c.kind == T_FINAL && qlane) {
      // h' = h ^ v_i ^ v_{i+8}: sources h (INW, the loaded word: before the stores) and the
      // final state words
      const uint32_t a = lane >> 1;
#pragma unroll
      for (int kk2 = 0; kk2 < 2; kk2++) {
        const uint32_t k = 2 * (lane & 1u) + kk2, dr = 8 * a + 2 * k;
        uint32_t sh = spread16(limb(P.w[0], k));
        uint32_t sv = spread16(limb(prod[a], k));
        uint32_t su = spread16(limb(prod[a + 8], k));
        if (MODE & FZ_INJECT) {
          uint32_t cv = 0, cu = 0;
          const uint32_t vs = state_src(a, k, 1, 2 * c.rounds, cv);
          const uint32_t us = state_src(a + 8, k, 1, 2 * c.rounds, cu);
          sh ^= inj_at(inj, c.off + 4 * a + k, A2);
          sv ^= inj_at(inj, c.off + vs, cv);
          su ^= inj_at(inj, c.off + us, cu);
        }
        if (T.at(A3, dr) != sh) A.fail(c.row0 + dr, B2F_CODE_COPY);
        if (T.at(A4, dr) != sv) A.fail(c.row0 + dr, B2F_CODE_COPY);
        if (T.at(A5, dr) != su) A.fail(c.row0 + dr, B2F_CODE_COPY);
      }
    }
    store_staged<MODE>(S, lane, nq, c.row0, adv, fixed, total_rows);
    if (qlane) {
      const uint4 fx = T.quad(FXC, 4 * lane);
      if (MODE & FZ_LOOKUP) check_lookups(A, T.quad(A0, 4 * lane), T.quad(A1, 4 * lane), T.quad(A2, 4 * lane), qrow);
      if (MODE & FZ_GATES) {
        const QuadInfo d = decode_quad((uint32_t)((qrow - c.off) >> 2), c.rounds);
        const uint4 xf = fixed_of_quad(d, d.kind == K_CONST ? IV[d.a & 7u] : 0ull);
        check_fixed(A, fx, xf, qrow);
        const bool canon = ((fx.x ^ xf.x) & 0xffffu) == 0 && ((fx.y ^ xf.y) & 0xffffu) == 0 &&
                           ((fx.z ^ xf.z) & 0xffffu) == 0 && ((fx.w ^ xf.w) & 0xffffu) == 0;
        S[S_CANON + lane] = canon ? 1u : 0u;
        if (!canon) defer_rows(fx, qrow, defer, defer_cap);
      }
    }
    if (MODE & FZ_GATES) {
      // the canonical init / final blocks, one kind per pass (LAYOUT.md §5 row map)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      const uint32_t* cq = S + S_CANON;
      if (c.kind == T_INIT) {
        if (lane < 26 && cq[lane] && !gate_ok(T, S_ABCD, 4 * lane, 0u, 0u))  // h, m, t words
          A.fail_gates(c.row0 + 4 * lane, 1u << S_ABCD);
        if (lane == 26 && cq[26] && !gate_ok(T, S_FMASK, 104, 0u, 0u))
          A.fail_gates(c.row0 + 104, 1u << S_FMASK);
        if (lane < 32 && cq[27 + (lane >> 2)]) {  // IV limbs: a_1 = k_0 on every CONST row
          const uint32_t r = 108 + lane;
          if (T.at(A1, r) != (T.at(FXC, r) >> 16)) A.fail_gates(c.row0 + r, 1u << S_CONST);
        }
        if (lane < 3 && cq[35 + 2 * lane] && !g_xor(T, 140 + 8 * lane, false))  // v12..v14
          A.fail_gates(c.row0 + 140 + 8 * lane, 1u << S_XOR);
      } else if (lane < 8 && cq[2 * lane]) {  // h'_i: XOR3 + digest
        const uint32_t r = 8 * lane;
        const uint32_t f = (g_xor(T, r, true) ? 0u : 1u << S_XOR3) | (g_digest(T, r) ? 0u : 1u << S_DIGEST);
        if (f) A.fail_gates(c.row0 + r, f);
      }
    }
    if (MODE & FZ_COPIES) {
      if (c.kind == T_INIT) {
        if (lane < 24) {  // v12 = IV4 ^ t0, v13 = IV5 ^ t1, v14 = IV6 ^ fmask
          const uint32_t a = lane >> 3, k = (lane >> 1) & 3u, op = lane & 1u;
          const uint32_t dr = 140 + 8 * a + 2 * k;
          const uint32_t sr = op == 0 ? 108 + 4 * (4 + a) + k : (a < 2 ? 96 + 4 * a + k : 104 + k);
          if (T.at(op ? A4 : A3, dr) != T.at(A2, sr)) A.fail(c.row0 + dr, B2F_CODE_COPY);
        }
      }
    }
}

// message words (the last use of the loaded operands): a1 (x) at +0 and a2 (y) at +28 of
// every G, lanes 0..31
template <int MODE, bool REC>
__device__ __forceinline__ void hr_msg_copies(Fails<REC>& F, const HrTile& T, uint32_t lane,
                                              const Ctx& c, uint64_t mw, const uint8_t* Sg,
                                              const Inject& inj) {
  if ((MODE & FZ_COPIES) && lane < 32) {
    const uint32_t mg = lane >> 3, which = (lane >> 2) & 1u, k = lane & 3u;
    const uint32_t dr = 52 * mg + (which ? 28u : 0u) + k;
    uint32_t sv = limb(mw, k);
    if (MODE & FZ_INJECT) {
      const uint32_t g = mg + 4 * (c.hr & 1u);
      const uint32_t mj = Sg[16 * ((c.hr >> 1) % 10) + 2 * g + which];
      sv ^= inj_at(inj, c.off + 32 + 4 * mj + k, A1);
    }
    F.fail(T.at(A5, dr) != sv, c.row0 + dr, B2F_CODE_COPY);
  }
}

// lookups, the fixed column, the canonical gate passes and the copies of a half-round tile.
// `ct`: the HrChecks entries of the tile's parity; `state(w, k, spread)`: limb k of state word w
// as its producer assigned it (dense or spread).
template <int MODE, bool REC, class StateLimb>
__device__ __forceinline__ void hr_checks(Fails<REC>& F, const HrTile& T, uint32_t lane,
                                          const Ctx& c, const uint32_t* ct, const StateLimb& state,
                                          const Inject& inj, uint64_t* defer, uint32_t defer_cap) {
  const uint32_t nq = c.nq;
  const bool qlane = lane < nq;
  const uint64_t qrow = c.row0 + 4ull * lane;
  const uint32_t gg = lane / G_QUADS, p = lane - G_QUADS * gg;
  if (qlane) {
    const uint4 fx = T.quad(FXC, 4 * lane);
    const uint32_t xs = expected_sel(p);
    if (MODE & FZ_LOOKUP) {
      const uint4 q0 = T.quad(A0, 4 * lane), q1 = T.quad(A1, 4 * lane), q2 = T.quad(A2, 4 * lane);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t tg = comp(q0, j), de = comp(q1, j), sp = comp(q2, j);
        F.fail(!(de < 65536u && tg == tag16(de) && sp == spread16(de & 0xffffu)), qrow + j, B2F_CODE_LOOKUP);
      }
    }
    if (MODE & FZ_GATES) {
      if (REC) {
        const bool canon = (fx.x & 0xffffu) == xs && ((fx.y | fx.z | fx.w) & 0xffffu) == 0;
        check_fixed(F.A, fx, make_uint4(xs, 0, 0, 0), qrow);
        if (!canon) defer_rows(fx, qrow, defer, defer_cap);
      } else {
        F.bad |= ((fx.x ^ xs) | fx.y | fx.z | fx.w) != 0;  // any fixed cell off the structure
      }
    }
  }
  if (MODE & FZ_GATES) {
    // canonical blocks, one kind per pass so each pass is one evaluator: the adds
    // (lanes 0-15: a1 +0, c1 +12, a2 +28, c2 +40 of G lane / 4), the XORs (lanes 0-7:
    // d1 +4, d2 +32 of G lane / 2), XOR24 limbs (lanes 0-15: b1 + efgh at +16, limb
    // lane % 4, OR-combined over the DPP quad) and XOR63 limbs (b2 + ijkl at +44)
    const uint32_t w4 = lane & 3u;
    auto canon_block = [&](uint32_t r, uint32_t want) {
      const uint4 bf = T.quad(FXC, r);  // the block's first quad
      return (bf.x & 0xffffu) == want && ((bf.y | bf.z | bf.w) & 0xffffu) == 0;
    };
    if (lane < 16) {
      const uint32_t r = 52 * (lane >> 2) + (w4 == 0 ? 0u : w4 == 1 ? 12u : w4 == 2 ? 28u : 40u);
      const uint32_t want = 1u << (w4 == 0 ? S_A1 : w4 == 1 ? S_C1 : w4 == 2 ? S_A2 : S_C2);
      F.gates(canon_block(r, want) && !g_add(T, r, T.at(A9, r), (w4 & 1u) == 0), c.row0 + r, want);
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < 8) {
      const uint32_t r = 52 * (lane >> 1) + ((lane & 1u) ? 32u : 4u);
      const uint32_t want = 1u << ((lane & 1u) ? S_D2 : S_D1);
      F.gates(canon_block(r, want) && !g_xor(T, r, false), c.row0 + r, want);
    }
    __builtin_amdgcn_wave_barrier();
    {
      const uint32_t r = 52 * ((lane >> 2) & 3u) + 16;
      const uint32_t want = (1u << S_B1) | (1u << S_EFGH);
      const bool take = lane < 16 && canon_block(r, want);
      const uint32_t qb = quad_or(take ? g_xor24_limb(T, r, w4) : 0u);
      F.gates(take && w4 == 0 && qb, c.row0 + r,
              ((qb & 1u) ? 1u << S_B1 : 0u) | ((qb & 2u) ? 1u << S_EFGH : 0u));
    }
    __builtin_amdgcn_wave_barrier();
    {
      const uint32_t r = 52 * ((lane >> 2) & 3u) + 44;
      const uint32_t want = (1u << S_B2) | (1u << S_IJKL);
      const bool take = lane < 16 && canon_block(r, want);
      const uint32_t qb = quad_or(take ? g_xor63_limb(T, r, w4) : 0u);
      F.gates(take && w4 == 0 && qb, c.row0 + r,
              ((qb & 1u) ? 1u << S_B2 : 0u) | ((qb & 2u) ? 1u << S_IJKL : 0u));
    }
  }
  if (MODE & FZ_COPIES) {
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
        sv = state(w, k, sp);
        if (MODE & FZ_INJECT) {
          uint32_t col = 0;
          const uint32_t sr = state_src(w, k, sp, c.hr, col);
          sv ^= inj_at(inj, c.off + sr, col);
        }
      }
      F.fail(dv != sv, c.row0 + dr, B2F_CODE_COPY);
    }
  }
}

// The first tile of wave wv of workgroup b in a persistent grid of `grid` workgroups that takes
// WAVES * grid consecutive tiles per round. XCD-aware: workgroups are dispatched to the 8 XCDs
// round-robin (b % 8), so XCD x takes the x-th eighth of every round as one contiguous run --
// neighbouring tiles (which share boundary cache lines, the previous half-round's state cells and
// the instance's message rows) sit behind the same L2.
__device__ __forceinline__ uint64_t first_tile(uint32_t b, uint32_t wv, uint32_t grid) {
  if (grid % 8 == 0) return ((uint64_t)(b % 8) * (grid / 8) + b / 8) * WAVES + wv;
  return (uint64_t)b * WAVES + wv;
}

// ============================================================================================
// The half-round launch (fused_hr_kernel): a lane's quad position p inside its G never
// changes from tile to tile, so everything that depends on p alone -- which bytes of which
// operand word land in every cell, which cells every check reads -- is resolved once per lane
// before the tile loop (v_perm_b32 byte selectors and LDS byte addresses in registers). Per tile:
//   1. lanes 0-15 copy the tile's 16 state words in G order out of OUT (the wave's previous tile's
//      G outputs, or the initial work vector at an instance's first tile), lanes 16-23 its 8
//      message words out of the instance record in LDS;
//   2. every lane runs the G chain of its G; one lane per G publishes the chain
//      (a d c b a1 d1 c1 b1 a2 d2 c2 mx my 0), so a quad's operands X = s[step], Y = s[step+3]
//      and M are three LDS reads instead of select chains, and writes its G's outputs into the
//      other OUT slot (the next tile's state); G 3's chain also goes to the other GP slot (the
//      next tile's tail lanes, which recompute this tile's last seven quads); every lane builds
//      one (word, limb) entry of the limb table the copy checks read, from this tile's OUT slot;
//   3. cells: a_1 rows and every operand slot by v_perm byte selection, spreads and tags, staged;
//   4. stores: 11 raw buffer stores per tile, each covering whole 128-byte lines (line ownership,
//      see the store loop);
//   5. fast checks, every one a 32-bit bitwise accumulation (acc |= lhs ^ rhs): lookups, the
//      fixed column, all XOR/XOR24/XOR63 limb identities in ONE pass (64 lanes = 64 limb items),
//      the 16 additions as carry chains, the 256 + 32 copies as pure LDS compares. They assume
//      what the other checks of the same pass establish (every checked cell in its range); a
//      cell out of range fails its own check, so a clean pass proves a clean tile, and a flagged
//      tile is re-checked exactly (hr_checks<REC = true>, the eval kernel's bookkeeping).
// The staging columns a_9 and fixed are written last in a tile, so their rows hold the tile's
// transient words (steps 1-2) until then.
namespace hr2 {
constexpr uint32_t PZ = 0x0c0c0c0cu;  // v_perm_b32 selector: four zero bytes
constexpr uint32_t psel(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3) {
  return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
}
constexpr uint32_t limb_sel(uint32_t k) { return psel(2 * k, 2 * k + 1, 12, 12); }  // on (hi, lo)

// The ADD block each lane checks in the fast checks (every lane checks one of the tile's 16 ADD
// blocks, i = 4 G + kind). ds_read_b128 serves a wave in four 16-lane groups, a lane's 16 bytes on
// banks (a / 4) mod 64 .. +3; the blocks' first rows mod 64 are 0 12 28 40 | 52 0 16 28 | 40 52 4 16
// | 28 40 56 4, so one lane per block within a group is up to 4-way conflicted. Instead each group
// reads four blocks whose bank ranges are disjoint, each by four lanes (the same address:
// broadcast): {0 16 28 52} {0 16 40 52} {4 12 28 40} {4 28 40 56} by first row mod 64.
struct AddBlk {
  uint32_t b[64];
};
constexpr AddBlk make_add_blk() {
  AddBlk T{};
  const uint32_t sets[4][4] = {{0, 6, 2, 4}, {5, 11, 3, 9}, {10, 1, 7, 8}, {15, 12, 13, 14}};
  // ds_read_b128 lane groups, in lane order
  const uint32_t grp[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                               {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                               {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                               {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
  for (uint32_t g = 0; g < 4; g++)
    for (uint32_t k = 0; k < 16; k++) T.b[grp[g][k]] = sets[g][k & 3u];
  return T;
}
constexpr bool add_blk_ok() {  // every block covered; bank ranges disjoint inside each group
  const AddBlk T = make_add_blk();
  uint32_t seen = 0;
  for (uint32_t l = 0; l < 64; l++) seen |= 1u << T.b[l];
  if (seen != 0xffffu) return false;
  const uint32_t off[4] = {0, 12, 28, 40};
  const uint32_t sets[4][4] = {{0, 6, 2, 4}, {5, 11, 3, 9}, {10, 1, 7, 8}, {15, 12, 13, 14}};
  for (uint32_t g = 0; g < 4; g++)
    for (uint32_t a = 0; a < 4; a++)
      for (uint32_t b = a + 1; b < 4; b++) {
        const uint32_t ra = (52 * (sets[g][a] >> 2) + off[sets[g][a] & 3u]) % 64;
        const uint32_t rb = (52 * (sets[g][b] >> 2) + off[sets[g][b] & 3u]) % 64;
        if (ra < rb + 4 && rb < ra + 4) return false;
      }
  return true;
}
static_assert(add_blk_ok(), "ADD block lane map: all 16 blocks, conflict-free groups");
__constant__ AddBlk c_add_blk = make_add_blk();

// Per quad position p: the byte selectors of every cell of the quad (LAYOUT.md §4, the same
// recipes as make_rows / quad_round).
struct QuadProg {
  uint32_t selL[4], selH[4];  // a_1 of row j = perm(O_lo, T_lo, selL) | perm(O_hi, T_hi, selH)
  uint32_t slot[4];           // a_3..a_8 of row j = perm(slot B, slot A, slot) (ADD: limb j of (hi, lo))
  uint32_t slA, slB;          // limb selectors of the operand slots on (hi, lo)
  uint32_t flags;             // bit 0 ADD, 1 XOR63, 2 XOR24 | XOR63 (w cells), 3 XOR24
  uint32_t fx0;               // fixed cell of row 0 (keygen selectors; rows 1-3 are 0)
};
struct QuadProgs {
  QuadProg q[G_QUADS];
};
constexpr QuadProgs make_qprogs() {
  QuadProgs P{};
  const RowTable R = make_rows();
  for (uint32_t p = 0; p < G_QUADS; p++) {
    QuadProg& g = P.q[p];
    const uint32_t st = step_of_quad(p);
    const bool add = st % 2 == 0, x24 = st == 3, x63 = st == 7;
    for (uint32_t j = 0; j < 4; j++) {
      const uint32_t e = R.r[p][j];
      const uint32_t k = e & 3u, src = (e >> 2) & 3u, sh8 = (e >> 4) & 1u, mcode = (e >> 5) & 3u;
      const uint32_t b0 = 2 * k + sh8, half = b0 >> 2, bb = b0 & 3u, so = src == 2 ? 4u : 0u;
      const uint32_t sel = psel(bb + so, mcode == 1 ? 12u : bb + 1 + so, 12, 12);
      g.selL[j] = half == 0 ? sel : PZ;
      g.selH[j] = half == 1 ? sel : PZ;
    }
    const uint32_t sd = R.slot[p];
    const uint32_t jA = sd & 3u, kA = (sd >> 2) & 3u, vA = (sd >> 4) & 1u;
    const uint32_t jB = (sd >> 5) & 3u, kB = (sd >> 7) & 3u, vB = (sd >> 9) & 1u;
    g.slA = limb_sel(kA);
    g.slB = limb_sel(kB);
    for (uint32_t j = 0; j < 4; j++)
      g.slot[j] = add ? limb_sel(j) : (vA && jA == j) ? 0x03020100u : (vB && jB == j) ? 0x07060504u : PZ;
    g.flags = (add ? 1u : 0u) | (x63 ? 2u : 0u) | ((x24 || x63) ? 4u : 0u) | (x24 ? 8u : 0u);
    g.fx0 = expected_sel(p);
  }
  return P;
}
// The recipes the selectors assume: a_1 sources are S (ADD), Z / O (XOR family); 0x7fff
// masks only on XOR63's Z rows (applied to T), 0xff fields only in XOR24; no field crosses a
// 32-bit half.
constexpr bool qprogs_ok() {
  const RowTable R = make_rows();
  for (uint32_t p = 0; p < G_QUADS; p++) {
    const uint32_t st = step_of_quad(p);
    for (uint32_t j = 0; j < 4; j++) {
      const uint32_t e = R.r[p][j], src = (e >> 2) & 3u, mcode = (e >> 5) & 3u;
      if (st % 2 == 0 && src != 0) return false;
      if (st % 2 == 1 && src == 0) return false;
      if (mcode == 2 && !(st == 7 && src == 1)) return false;
      if (st == 7 && src == 1 && mcode != 2) return false;
      if (mcode == 1 && st != 3) return false;
      if (mcode == 3) return false;
    }
  }
  return true;
}
static_assert(qprogs_ok(), "quad programs match the row recipes");
__constant__ QuadProgs c_qprogs = make_qprogs();

// wave LDS (words), relative to S = row 0 of staging column a_0: staging [11][HSTR] from row -HPRE
// (the region starts HPRE words before S); limb table LT: [0, 64) dense, [64, 128) spread limb k
// of state word w at 4 w + k; MW: the tile's 8 message words (u64, 2 gg + i).
constexpr int H_LT = NSTAGE * HSTR - HPRE;
constexpr int H_MW = H_LT + 128;
// carried from tile to tile by the half-round launch (a wave walks an instance's half-rounds in
// order): OUT [2][16] u64 -- by parity, the G outputs of the wave's previous tile in its G order
// (the state as this tile starts, and the copy sources of its state-word cells); GP [2][16] u64 --
// by parity, the previous tile's G 3 chain record (the tail lanes'); IN [27] u64 -- the
// instance's input record (h, m, t, rounds | f)
constexpr int H_OUT = H_MW + 16;
constexpr int H_GP = H_OUT + 64;
constexpr int H_IN = H_GP + 64;
constexpr int HW_WORDS = HPRE + H_IN + 56;  // the region
// transient, inside staging columns a_9 and fixed: WD 56 u64 ([0, 16) state words of the tile
// in G order, [16, 24) the producers' message words, [24, 40) previous state words in G order,
// [40, 56) scratch), GS 4 x 16 u64 (the published chains), PG 16 u64 (producer outputs, G order),
// GP 16 u64 (the chain of the previous half-round's G 3, published by producer lane HR_Q + 3 for
// the tail lanes TAIL0 .. TAIL0 + 6, which recompute its quads 6-12 into rows -28 .. -1)
constexpr int T_WD = A9 * HSTR;
constexpr int T_GS = T_WD + 112;
constexpr int T_PG = T_GS + 128;
constexpr int T_GP = T_PG + 32;
constexpr int TAIL0 = 56;
static_assert(T_GP + 32 <= H_LT, "transient words inside columns a_9 and fixed");
static_assert(HSTR % 4 == 0 && HPRE == 4 * 7, "16-byte quads; seven tail quads in front");
// workgroup LDS (words)
constexpr int H_ACC = 0, H_IV = 24, H_SG = H_IV + 16, H_WAVE = H_SG + 40;
constexpr int H_WORDS = H_WAVE + WAVES * HW_WORDS;
static_assert(H_WAVE % 4 == 0 && HW_WORDS % 4 == 0 && T_WD % 4 == 0 && T_GS % 4 == 0 && T_PG % 4 == 0 &&
                  T_GP % 4 == 0 && H_OUT % 4 == 0 && H_GP % 4 == 0 && H_IN % 4 == 0,
              "16-byte aligned carve");
static_assert(H_WORDS * 4 * 3 <= 160 * 1024, "three workgroups per CU");
static_assert(4 * H_WORDS < 65536, "LDS byte addresses fit 16 bits");
// the quad whose program a lane holds: its own (lanes 0-51), the previous tile's quads 45-51 (the
// tail lanes), quads 0-3 / 11 again (the producer lanes, lane 63: duplicate checks)
__host__ __device__ constexpr uint32_t lane_quad(uint32_t lane) {
  return lane < HR_Q ? lane : (lane >= TAIL0 && lane < TAIL0 + 7) ? lane - (TAIL0 - (HR_Q - 7)) : lane - HR_Q;
}
static_assert(lane_quad(TAIL0) == HR_Q - 7 && lane_quad(TAIL0 + 6) == HR_Q - 1, "tail lanes: quads 45-51");

// LDS accesses by byte address (a VGPR holding the address, the offset immediates folded in)
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) uint32_t l32;
typedef __attribute__((address_space(3))) uint16_t l16;
typedef __attribute__((address_space(3))) uint64_t l64;
typedef __attribute__((address_space(3))) u32x4_t l128;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wint-to-pointer-cast"
__device__ __forceinline__ uint32_t lds_byte(const uint32_t* p) {
  return (uint32_t)(uintptr_t)(const l32*)p;
}
__device__ __forceinline__ uint32_t ld32(uint32_t a) { return *(const l32*)a; }
__device__ __forceinline__ uint32_t ld16(uint32_t a) { return *(const l16*)a; }
__device__ __forceinline__ uint64_t ld64(uint32_t a) { return *(const l64*)a; }
__device__ __forceinline__ uint4 ld128(uint32_t a) {
  const u32x4_t v = *(const l128*)a;
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st32(uint32_t a, uint32_t v) { *(l32*)a = v; }
__device__ __forceinline__ void st64(uint32_t a, uint64_t v) { *(l64*)a = v; }
__device__ __forceinline__ void st128(uint32_t a, uint4 v) {
  const u32x4_t w = {v.x, v.y, v.z, v.w};
  *(l128*)a = w;
}
#pragma clang diagnostic pop
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}
__device__ __forceinline__ uint32_t lo32(uint64_t v) { return (uint32_t)v; }
__device__ __forceinline__ uint32_t hi32(uint64_t v) { return (uint32_t)(v >> 32); }
__device__ __forceinline__ uint64_t mk64(uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); }
// tag of a 16-bit value (0: < 2^8, 1: < 2^15, 2: otherwise), branch-free
__device__ __forceinline__ uint32_t tag_of(uint32_t x) { return ((x + 0xff00u) >> 16) + (x >> 15); }
__device__ __forceinline__ uint32_t sel32(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }
// A tile as the wave sees it (wave-uniform).
struct HCtx {
  uint32_t inst, rounds, hr, st;
  uint64_t off, row0;
};
__device__ __forceinline__ HCtx hctx(const uint4& raw) {
  HCtx c;
  c.inst = __builtin_amdgcn_readfirstlane(raw.x);
  const uint32_t j = __builtin_amdgcn_readfirstlane(raw.y);
  c.rounds = __builtin_amdgcn_readfirstlane(raw.z);
  c.st = __builtin_amdgcn_readfirstlane(raw.w);
  c.hr = j ? j - 1 : 0;  // past the last tile: a valid in-bounds context (its loads are never used)
  c.off = 20ull * c.inst + 208ull * c.st;
  c.row0 = c.off + INIT_ROWS + 208ull * c.hr;
  return c;
}

// The per-lane constants of the tile loop (resolved once).
struct Lane {
  // assignment
  uint32_t selL[4], selH[4], slot[4], slA, slB;
  uint32_t madd, mzm, mhz, mhw, mswap, rsh, fx0;
  uint32_t aWD, aAB, aMX, aGS, aXY, aM, aPG, aLTs, aLTd, ltsh;
  uint32_t oW;  // lanes 0-15: byte offsets in an OUT slot of the state word (hr 0 | even | odd)
  // checks
  uint32_t aQ;                        // the lane's quad (lane_quad), column a_0
  uint32_t gb, ge, gf, gsel, gm24, gm63, gnl, grs, gsF, gsH;  // XOR-family limb item
  uint32_t ar, m3;                    // ADD block
  uint32_t ce[2][4], cm;              // copies (dst | src << 16), message copy
};

__device__ __forceinline__ Lane make_lane(uint32_t lane, uint32_t Sb) {
  Lane L;
  const uint32_t lq = lane_quad(lane);
  const uint32_t gg = lq / G_QUADS, p = lq - G_QUADS * gg;
  const QuadProg& Q = c_qprogs.q[p];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    L.selL[j] = Q.selL[j];
    L.selH[j] = Q.selH[j];
    L.slot[j] = Q.slot[j];
  }
  L.slA = Q.slA;
  L.slB = Q.slB;
  const uint32_t fl = Q.flags;
  L.madd = (fl & 1u) ? ~0u : 0u;
  L.mzm = (fl & 2u) ? 0x7fff7fffu : ~0u;
  L.mhz = (fl & 2u) ? ~0u : 0u;
  L.mhw = (fl & 4u) ? ~0u : 0u;
  L.mswap = (fl & 2u) ? ~0u : 0u;
  L.rsh = (fl & 2u) ? 31u : 24u;
  L.fx0 = Q.fx0;
  const uint32_t st = step_of_quad(p), mi = st == 0 ? 11u : st == 4 ? 12u : 13u;
  // gathers
  L.aWD = lane < 16 ? Sb + 4 * T_WD + 8 * lane : lane < 24 ? Sb + 4 * H_MW + 8 * (lane - 16)
                                                            : Sb + 4 * T_WD + 8 * (lane - 8);
  if (lane < HR_Q) {
    L.aAB = Sb + 4 * T_WD + 32 * gg;
    L.aMX = Sb + 4 * H_MW + 16 * gg;
  } else if (lane < HR_Q + 4) {
    const uint32_t pg = lane - HR_Q;
    L.aAB = Sb + 4 * T_WD + 8 * (24 + 4 * pg);
    L.aMX = Sb + 4 * T_WD + 8 * (16 + 2 * pg);
  } else {
    L.aAB = Sb + 4 * T_WD + 8 * 40;
    L.aMX = Sb + 4 * T_WD + 8 * 40;
  }
  L.aGS = Sb + 4 * T_GS + 128 * gg;
  L.aXY = L.aGS + 8 * st;
  L.aM = Sb + 4 * T_GS + 128 * gg + 8 * mi;
  if (lane >= TAIL0 && lane < TAIL0 + 7) {  // the previous tile's G 3 chain record (GP slot 0)
    L.aXY = Sb + 4 * H_GP + 8 * st;
    L.aM = Sb + 4 * H_GP + 8 * mi;
  }
  {  // state word (a, b, c, d)[role] of G gl, in the previous tile's G order q = (hr - 1) & 1:
     // natural word w = 4 role + j is output (G (j - role q) & 3, role) of the previous half-round
    const uint32_t gl = (lane >> 2) & 3u, role = lane & 3u;
    const uint32_t i0 = 4 * gl + role;                           // hr 0: the initial vector, q = 0
    const uint32_t i1 = 4 * ((gl - role) & 3u) + role;           // hr even: w = 4 role + gl, q = 1
    const uint32_t i2 = 4 * ((gl + role) & 3u) + role;           // hr odd: w = 4 role + (gl + role), q = 0
    L.oW = 8 * i0 | (8 * i1) << 8 | (8 * i2) << 16;
  }
  L.aPG = Sb + 4 * T_PG + 32 * (lane - HR_Q);  // producer lanes only
  {  // limb table entry lane = 4 w + k, read from the producer outputs in G order (parity 0 / 1)
    const uint32_t w = lane >> 2, k = lane & 3u, role = w >> 2, pos = w & 3u;
    const uint32_t i0 = 4 * pos + role, i1 = 4 * ((pos - role) & 3u) + role;
    const uint32_t a0 = Sb + 4 * H_OUT + 8 * i0 + 4 * (k >> 1), a1 = Sb + 4 * H_OUT + 8 * i1 + 4 * (k >> 1);
    L.aLTs = a0 | (a1 << 16);
    L.ltsh = 16 * (k & 1u);
    L.aLTd = Sb + 4 * H_LT + 4 * lane;
  }
  L.aQ = Sb + 16 * lq;
  {  // XOR-family limb item `lane`: 0-31 XOR (d1 at +4, d2 at +32), 32-47 XOR24, 48-63 XOR63
    const uint32_t k = lane & 3u;
    uint32_t b, E, F, kind;
    if (lane < 32) {
      const uint32_t blk = lane >> 2, r = 52 * (blk >> 1) + ((blk & 1u) ? 32u : 4u);
      b = r + 2 * k;
      E = A1 * HSTR + b;
      F = A1 * HSTR + b;
      kind = 0;
    } else if (lane < 48) {
      const uint32_t r = 52 * ((lane - 32) >> 2) + 16;
      b = r + 3 * k;
      E = A1 * HSTR + r + 3 * ((k + 1) & 3u) + 1;
      F = A1 * HSTR + r + 3 * ((k + 2) & 3u);
      kind = 1;
    } else {
      const uint32_t r = 52 * ((lane - 48) >> 2) + 44;
      b = r + 2 * k;
      E = A6 * HSTR + r + 2 * ((k + 3) & 3u);
      F = A1 * HSTR + b;
      kind = 2;
    }
    L.gb = Sb + 4 * b;
    L.ge = Sb + 4 * E;
    L.gf = Sb + 4 * F;
    L.gsel = kind == 1 ? psel(12, 12, 0, 1) : PZ;  // XOR24: s2[b+1] << 16
    L.gm24 = kind == 1 ? ~0u : 0u;
    L.gm63 = kind == 2 ? ~0u : 0u;
    L.gnl = kind == 1 ? ~0u : kind == 2 ? ~1u : 0u;  // side cells: XOR24 == 0, XOR63 <= 1
    L.grs = kind ? ~0u : 0u;
    L.gsF = kind == 1 ? 8u : 1u;
    L.gsH = kind == 1 ? 16u : 2u;
  }
  {  // ADD block i = c_add_blk[lane] (a1 +0, c1 +12, a2 +28, c2 +40 of G i >> 2): every
     // ds_read_b128 lane group reads 4 blocks whose 16-byte bank ranges are disjoint, each by 4
     // lanes (one address: a broadcast) -- conflict-free
    const uint32_t i = c_add_blk.b[lane], w4 = i & 3u;
    const uint32_t r = 52 * (i >> 2) + (w4 == 0 ? 0u : w4 == 1 ? 12u : w4 == 2 ? 28u : 40u);
    L.ar = Sb + 4 * r;
    L.m3 = (w4 & 1u) ? 0u : ~0u;  // ADD3: a_5 is an operand
  }
#pragma unroll
  for (int par = 0; par < 2; par++)
#pragma unroll
    for (int it = 0; it < HR_CHECKS / FW; it++) {
      const uint32_t e = c_hr_checks.e[par][it * FW + lane];
      const uint32_t dr = e & 255u, dc = (e >> 8) & 3u;
      const uint32_t dst = Sb + 4 * ((A3 + dc) * HSTR + dr);
      uint32_t src;
      if (!((e >> 10) & 1u)) {
        src = Sb + 4 * (wcol((e >> 19) & 3u) * HSTR + ((e >> 11) & 255u));
      } else {
        const uint32_t w = (e >> 11) & 15u, k = (e >> 15) & 3u, sp = (e >> 17) & 1u;
        src = Sb + 4 * (H_LT + 64 * sp + 4 * w + k);
      }
      L.ce[par][it] = dst | (src << 16);
    }
  {  // message copy (lanes 32-63 repeat lanes 0-31)
    const uint32_t l = lane & 31u, mg = l >> 3, which = (l >> 2) & 1u, k = l & 3u;
    const uint32_t dr = 52 * mg + (which ? 28u : 0u) + k;
    L.cm = (Sb + 4 * (A5 * HSTR + dr)) | ((Sb + 4 * H_MW + 8 * (2 * mg + which) + 2 * k) << 16);
  }
  return L;
}

}  // namespace hr2

// The fast checks of a staged half-round tile (see the half-round launch's comment): lookups, the fixed
// column, every canonical gate block, the 256 state-word / in-tile copies (sources: the staging
// and the limb table), the lane's message copy against `msrc` (the message limb its producer or
// the trace holds, read where it is used). Returns the OR of every identity's lhs ^ rhs: 0 iff all hold (given the
// ranges the other checks of the pass establish).
template <int MODE, class MsgSrc>
__device__ __forceinline__ uint32_t hr_fast_checks(const hr2::Lane& K, uint32_t hr, const MsgSrc& msrc) {
  using namespace hr2;
  uint32_t acc = 0;
  if (MODE & (FZ_LOOKUP | FZ_GATES)) {
    const uint4 q0 = ld128(K.aQ + 4 * A0 * HSTR), q1 = ld128(K.aQ + 4 * A1 * HSTR), q2 = ld128(K.aQ + 4 * A2 * HSTR);
    const uint4 fx = ld128(K.aQ + 4 * FXC * HSTR);
    if (MODE & FZ_LOOKUP) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t de = comp(q1, j);
        acc |= (de & 0xffff0000u) | (tag_of(de) ^ comp(q0, j)) | (spread16(de) ^ comp(q2, j));
      }
    }
    if (MODE & FZ_GATES) acc |= (fx.x ^ K.fx0) | fx.y | fx.z | fx.w;
  }
  if (MODE & FZ_GATES) {
    {  // XOR / XOR24 / XOR63 limb item
      const uint32_t gb = K.gb;
      const uint32_t x3 = ld32(gb + 4 * A3 * HSTR), x4 = ld32(gb + 4 * A4 * HSTR);
      const uint32_t s0 = ld32(gb + 4 * A2 * HSTR), s1v = ld32(gb + 4 * (A2 * HSTR + 1)), s2v = ld32(gb + 4 * (A2 * HSTR + 2));
      const uint32_t z6 = ld32(gb + 4 * A6 * HSTR), t0 = ld32(gb), t1 = ld32(gb + 4);
      const uint32_t w7 = ld32(gb + 4 * A7 * HSTR), w8 = ld32(gb + 4 * A8 * HSTR);
      const uint32_t E = ld32(K.ge), E2 = ld32(K.ge + 4 * (A2 - A1) * HSTR);
      const uint32_t F = ld32(K.gf), H = ld32(K.gf + 4 * (A2 - A1) * HSTR);
      const uint32_t R = s0 + perm(0u, s1v, K.gsel) + ((z6 << 30) & K.gm63) + 2 * sel32(K.gm24, s2v, s1v);
      acc |= (x3 + x4) ^ R;
      acc |= (t0 | (t1 & K.gm24) | (z6 & K.gm63)) & K.gnl;
      const uint32_t G = sel32(K.gm24, E2, E);
      acc |= (((E + (F << K.gsF)) ^ w7) | ((G + (H << K.gsH)) ^ w8)) & K.grs;
    }
    {  // ADD block (lanes 16-63 repeat lanes 0-15)
      const uint4 s = ld128(K.ar + 4 * A1 * HSTR), x = ld128(K.ar + 4 * A3 * HSTR);
      const uint4 y = ld128(K.ar + 4 * A4 * HSTR), z = ld128(K.ar + 4 * A5 * HSTR);
      const uint32_t a9 = ld32(K.ar + 4 * A9 * HSTR);
      int32_t cy = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        cy += (int32_t)(comp(x, k) + comp(y, k) + (comp(z, k) & K.m3) - comp(s, k));
        acc |= (uint32_t)cy & 0xffffu;
        cy >>= 16;
      }
      acc |= (uint32_t)cy ^ a9;
    }
  }
  if (MODE & FZ_COPIES) {
    const bool odd = hr & 1u;
#pragma unroll
    for (int it = 0; it < HR_CHECKS / FW; it++) {
      const uint32_t e = odd ? K.ce[1][it] : K.ce[0][it];
      acc |= ld32(e & 0xffffu) ^ ld32(e >> 16);
    }
    acc |= ld32(K.cm & 0xffffu) ^ msrc();
  }
  return acc;
}

#ifndef B2F_EDGE_SEPARATE
#define B2F_EDGE_SEPARATE 0  // 1 (diagnostics): the edge tiles in their own launch after this one
#endif
#ifndef B2F_FUSED_DYN
#define B2F_FUSED_DYN 1  // 0 (variant): instances dealt statically to the waves (round 5)
#endif
#ifndef B2F_FUSED_EDGE_DYN
// 1: the edge tiles claimed from a counter too, B2F_FUSED_EDGE_CHUNK consecutive tiles per claim.
// One tile per claim was 11.62 vs 9.38 ms (2^18 x 12) and 8.53 vs 6.62 ({1,4,12},
// profiles/r06k_ab_dyn_*.txt): an edge tile is 9 KB of work, and 2^18 claims within the launch's
// last half-millisecond serialise on the one counter. 16 per claim: 9.49 vs 9.56 dealt, 5.25 vs
// 5.33; 64 per claim 9.56 / 5.32 (profiles/r06m_ab_edge_*.txt); another box, 8 / 16 / 32 per claim
// and dealt: 9.77 / 9.79 / 9.80 / 9.84 ms and 4.96 / 4.98 / 4.99 / 5.07 (profiles/r06n_ab_*.txt)
#define B2F_FUSED_EDGE_DYN 1
#endif
#ifndef B2F_FUSED_EDGE_CHUNK
#define B2F_FUSED_EDGE_CHUNK 8
#endif
template <int MODE>
__device__ __forceinline__ void edge_walk(uint32_t* S, uint32_t lane, uint64_t t_first, uint64_t W,
                                          const uint64_t* IV, const uint8_t* Sg, EvalAcc& A,
                                          const b2f_input* __restrict__ in, uint32_t n,
                                          const uint64_t* __restrict__ off, uint64_t total_rows,
                                          const uint64_t* __restrict__ rec, uint32_t* __restrict__ adv,
                                          uint32_t* __restrict__ fixed, uint32_t* __restrict__ redo,
                                          const Inject& inj, uint64_t* __restrict__ defer,
                                          uint32_t defer_cap, unsigned* __restrict__ ectr);
template <int MODE>
__global__ void __launch_bounds__(FW * WAVES, B2F_FUSED_WAVES)
fused_hr_kernel(const b2f_input* __restrict__ in, uint32_t n, const uint64_t* __restrict__ off,
                uint64_t total_rows, const uint64_t* __restrict__ rec, uint32_t* __restrict__ adv,
                uint32_t* __restrict__ fixed, unsigned* __restrict__ ictr,
                b2f_eval_report* __restrict__ rep, const int* __restrict__ status, Inject inj,
                uint64_t* __restrict__ defer, uint32_t defer_cap, unsigned long long* __restrict__ clk,
                const uint64_t* __restrict__ seg, uint64_t seg_cap, uint32_t* __restrict__ redo) {
  using namespace hr2;
  __shared__ __attribute__((aligned(16))) uint32_t L[H_WORDS];
  uint64_t ck[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tp = 0;
  auto tick = [&](int k) {
    if (MODE & FZ_CLOCK) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      if (k >= 0) ck[k] += now - tp;
      tp = now;
    }
  };
  const int tid = threadIdx.x;
  const uint32_t lane = (uint32_t)tid & 63u, wv = (uint32_t)tid >> 6;
  if (tid < 22) L[H_ACC + tid] = 0;
  if (tid == 22) *reinterpret_cast<uint64_t*>(L + H_ACC + 20) = ~0ull;
  if (tid < 16) L[H_IV + tid] = reinterpret_cast<const uint32_t*>(c_iv)[tid];
  if (tid < 40) L[H_SG + tid] = reinterpret_cast<const uint32_t*>(c_sigma)[tid];
  __syncthreads();
  EvalAcc A{L + H_ACC};
  const uint64_t* IV = reinterpret_cast<const uint64_t*>(L + H_IV);
  const uint8_t* Sg = reinterpret_cast<const uint8_t*>(L + H_SG);
  uint32_t* S = L + H_WAVE + wv * HW_WORDS + HPRE;  // this wave's staging (row 0 of column a_0)
  const uint32_t Sb = lds_byte(S);
  const Lane K = make_lane(lane, Sb);
  const bool qlane = lane < HR_Q, p0 = qlane && (lane % G_QUADS) == 0;
  const bool tlane = lane >= TAIL0 && lane < TAIL0 + 7;

  if (*status == 0) {  // the record kernel accepted the layout
    // Instances dealt to waves (XCD-aware, first_tile), each walked half-round by half-round:
    // the state a tile starts from is the G outputs of the wave's previous tile (OUT), so no
    // tile reads a recorded state. The next instance's input record is loaded one instance
    // ahead, a word per lane (27 lanes), every tile (the same address: L2 after the first) and
    // settled inside the tile like every other load.
    const uint64_t W = (uint64_t)gridDim.x * WAVES;
    uint64_t* const INW = reinterpret_cast<uint64_t*>(S + H_IN);
    const uint32_t aIN = Sb + 4 * H_IN;
    auto rec_word = [&](uint32_t i) -> uint64_t {  // lane's word of instance i's input record
      const uint64_t* x = reinterpret_cast<const uint64_t*>(in + (i < n ? i : 0));
      return x[lane < 27 ? lane : 26];
    };
#if B2F_FUSED_DYN
    // Instances are claimed from the launch's counter (a wave holds the one it walks and the next
    // one, whose record it loads ahead): the waves finish within one instance of each other
    // whatever the rounds mix. Dealt statically (wave w: instances w, w + W, ...) a {1,4,12}
    // batch gave each wave 85 instances of 2 / 8 / 24 half-round tiles at random, i.e. per-wave
    // work spread by +-9 % and the launch ended with its slowest wave (round 6, config 5).
    auto next_inst = [&](uint32_t) -> uint32_t {
      uint32_t i;
      do {
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(ictr, 1u);
        i = __builtin_amdgcn_readfirstlane(v);
      } while (i < n && in[i].rounds == 0);
      return i < n ? i : n;
    };
    const uint64_t w0 = first_tile(blockIdx.x, __builtin_amdgcn_readfirstlane(wv), gridDim.x);
    uint32_t inst = next_inst(0);
#else
    (void)ictr;
    // the instance after `i` in this wave's sequence that has half-rounds (scalar loads)
    auto next_inst = [&](uint32_t i) -> uint32_t {
      uint64_t j = (uint64_t)i + W;
      while (j < n && in[j].rounds == 0) j += W;
      return j < n ? (uint32_t)j : n;
    };
    const uint64_t w0 = first_tile(blockIdx.x, __builtin_amdgcn_readfirstlane(wv), gridDim.x);
    uint32_t inst = w0 < n ? (in[w0].rounds ? (uint32_t)w0 : next_inst((uint32_t)w0)) : n;
#endif
    uint64_t Pi = rec_word(inst);  // the current instance's record word
    // settled before the loop: otherwise the compiler cannot prove at the loop header that Pi is
    // never pending and waits for vmcnt(0) -- every store in flight -- at its first use
    asm volatile("" ::"v"(Pi));
    HCtx c;
    uint32_t ninst = 0, hr_end = 0;
    uint64_t qs = w0;  // this wave's next entry of the segment list (after its instances)
    bool fresh = true;
    c.hr = 0;
    for (;;) {
      tick(-1);
      if (fresh && inst < n) {  // an instance's first tile: its context, its record into IN, the
                                // initial work vector (h, IV, IV ^ (t0, t1, fmask)) into OUT slot 0
                                // in column-G order; its first SEG_HR half-rounds
        const uint64_t o = off[inst];
        c.inst = inst;
        c.rounds = in[inst].rounds;
        c.st = (uint32_t)((o - 20ull * inst) / 208);
        c.off = o;
        c.hr = 0;
        hr_end = 2 * c.rounds < SEG_HR ? 2 * c.rounds : SEG_HR;
        ninst = next_inst(inst);
        if (lane < 27) st64(aIN + 8 * lane, Pi);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (lane < 16) {
          const uint32_t g = lane >> 2, k = lane & 3u;
          const uint64_t fw = INW[26];
          const uint64_t tw = g < 2 ? INW[24 + g] : (g == 2 ? ((fw >> 32) ? ~0ull : 0ull) : 0ull);
          const uint64_t v = k == 0 ? INW[g] : k == 1 ? INW[g + 4] : k == 2 ? IV[g] : (IV[g + 4] ^ tw);
          st64(Sb + 4 * H_OUT + 8 * lane, v);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        fresh = false;
      } else if (fresh) {  // a later segment m of a long instance (the list, after the instances):
                           // half-rounds h0 = m SEG_HR .. from the recorded states h0 - 1 and h0
        if (qs >= (seg[0] < seg_cap ? seg[0] : seg_cap)) break;  // an overflow raised B2F_ERR_CHECK
        const uint64_t e = seg[1 + qs];
        qs += W;
        const uint32_t i = __builtin_amdgcn_readfirstlane((uint32_t)(e >> 32));
        const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)e);
        const uint64_t o = off[i];
        c.inst = i;
        c.rounds = in[i].rounds;
        c.st = (uint32_t)((o - 20ull * i) / 208);
        c.off = o;
        c.hr = m * SEG_HR;
        hr_end = 2 * c.rounds < (m + 1) * SEG_HR ? 2 * c.rounds : (m + 1) * SEG_HR;
        ninst = n;
        const uint64_t* sp = rec + 16ull * ((uint64_t)c.st + c.hr);  // state at h0, natural order
        const uint32_t ob0 = 128u * (c.hr & 1u);
        const uint64_t rw = rec_word(i);
        // OUT: the state at h0 in the previous half-round's G order (its G outputs as the walk
        // would have left them); the lanes' words settle before the LDS writes
        const uint32_t gs = (lane >> 2) & 3u, kk = lane & 3u;
        const uint32_t gw = gidx_word(gs + 4 * ((c.hr - 1) & 1u));
        const uint64_t vs = sp[(gw >> (8 * kk)) & 15u];
        if (lane < 27) st64(aIN + 8 * lane, rw);
        if (lane < 16) st64(Sb + 4 * H_OUT + ob0 + 8 * lane, vs);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) {  // GP: the chain of half-round h0 - 1's G 3 (the tail lanes' quads)
          const uint32_t hp = c.hr - 1, g3 = 3 + 4 * (hp & 1u);
          const uint64_t* pp = rec + 16ull * ((uint64_t)c.st + hp);
          const uint32_t gi = gidx_word(g3);
          const uint64_t a = pp[gi & 15u], b = pp[(gi >> 8) & 15u], cc = pp[(gi >> 16) & 15u], d = pp[gi >> 24];
          const uint8_t* sg = Sg + 16 * ((hp >> 1) % 10) + 2 * g3;
          const uint64_t mx = INW[8 + sg[0]], my = INW[8 + sg[1]];
          const uint64_t a1 = a + b + mx, d1 = rotr64(d ^ a1, 32), c1 = cc + d1, b1 = rotr64(b ^ c1, 24);
          const uint64_t a2 = a1 + b1 + my, d2 = rotr64(d1 ^ a2, 16), c2 = c1 + d2;
          const uint32_t gp = Sb + 4 * H_GP + ob0;
          st128(gp, make_uint4(lo32(a), hi32(a), lo32(d), hi32(d)));
          st128(gp + 16, make_uint4(lo32(cc), hi32(cc), lo32(b), hi32(b)));
          st128(gp + 32, make_uint4(lo32(a1), hi32(a1), lo32(d1), hi32(d1)));
          st128(gp + 48, make_uint4(lo32(c1), hi32(c1), lo32(b1), hi32(b1)));
          st128(gp + 64, make_uint4(lo32(a2), hi32(a2), lo32(d2), hi32(d2)));
          st128(gp + 80, make_uint4(lo32(c2), hi32(c2), lo32(mx), hi32(mx)));
          st128(gp + 96, make_uint4(lo32(my), hi32(my), 0u, 0u));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        fresh = false;
      }
      c.row0 = c.off + INIT_ROWS + 208ull * c.hr;
      const uint32_t ob = 128u * (c.hr & 1u), nb = 128u - ob;  // this tile's OUT / GP slot, the next's
      const uint64_t Pn = rec_word(ninst);  // the next instance's record word (past the end: harmless)
      // ---- 1. the tile's words into the wave's LDS: the state words (lanes 0-15) from OUT, the
      // message words (16-23) from IN
      {
        const uint32_t h = c.hr;
        const uint32_t sh = h == 0 ? 0u : (h & 1u) ? 16u : 8u;
        const uint32_t gm = (lane >> 1) & 3u, i = lane & 1u;
        const uint32_t sidx = Sg[16 * ((h >> 1) % 10) + 2 * (gm + 4 * (h & 1u)) + i];
        const uint32_t src = lane < 16 ? Sb + 4 * H_OUT + ob + ((K.oW >> sh) & 255u) : aIN + 8 * (8 + sidx);
        if (lane < 24) st64(K.aWD, ld64(src));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      tick(0);
      // ---- 2. chains: quad lanes their G of half-round hr
      const uint4 ab = ld128(K.aAB), cd = ld128(K.aAB + 16), mm = ld128(K.aMX);
      const uint64_t a = mk64(ab.x, ab.y), b = mk64(ab.z, ab.w), cc = mk64(cd.x, cd.y), d = mk64(cd.z, cd.w);
      const uint64_t mx = mk64(mm.x, mm.y), my = mk64(mm.z, mm.w);
      const uint64_t a1 = a + b + mx;
      const uint64_t d1 = rotr64(d ^ a1, 32);
      const uint64_t c1 = cc + d1;
      const uint64_t b1 = rotr64(b ^ c1, 24);
      const uint64_t a2 = a1 + b1 + my;
      const uint64_t d2 = rotr64(d1 ^ a2, 16);
      const uint64_t c2 = c1 + d2;
      if (p0) {
        const uint32_t g = K.aGS;  // this G's chain record
        const uint4 r0 = make_uint4(lo32(a), hi32(a), lo32(d), hi32(d));
        const uint4 r1 = make_uint4(lo32(cc), hi32(cc), lo32(b), hi32(b));
        const uint4 r2 = make_uint4(lo32(a1), hi32(a1), lo32(d1), hi32(d1));
        const uint4 r3 = make_uint4(lo32(c1), hi32(c1), lo32(b1), hi32(b1));
        const uint4 r4 = make_uint4(lo32(a2), hi32(a2), lo32(d2), hi32(d2));
        const uint4 r5 = make_uint4(lo32(c2), hi32(c2), lo32(mx), hi32(mx));
        const uint4 r6 = make_uint4(lo32(my), hi32(my), 0u, 0u);
        st128(g, r0);
        st128(g + 16, r1);
        st128(g + 32, r2);
        st128(g + 48, r3);
        st128(g + 64, r4);
        st128(g + 80, r5);
        st128(g + 96, r6);
        // the next tile's state / copy sources: this G's outputs into the other OUT slot
        const uint64_t o1 = rotr64(b1 ^ c2, 63);
        const uint32_t go = Sb + 4 * H_OUT + nb + 32 * (lane / G_QUADS);
        st128(go, make_uint4(lo32(a2), hi32(a2), lo32(o1), hi32(o1)));
        st128(go + 16, make_uint4(lo32(c2), hi32(c2), lo32(d2), hi32(d2)));
        if (lane == 3 * G_QUADS) {  // G 3's chain record for the next tile's tail lanes
          const uint32_t gp = Sb + 4 * H_GP + nb;
          st128(gp, r0);
          st128(gp + 16, r1);
          st128(gp + 32, r2);
          st128(gp + 48, r3);
          st128(gp + 64, r4);
          st128(gp + 80, r5);
          st128(gp + 96, r6);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      tick(1);
      // ---- 3. operands of the lane's quad, the lane's limb-table entry
      const uint32_t gofs = tlane ? ob : 0u;  // tail lanes: the previous tile's G 3 (GP slot)
      const uint64_t X = ld64(K.aXY + gofs), Y = ld64(K.aXY + gofs + 24), M = ld64(K.aM + gofs);
      const uint32_t par = c.hr ? ((c.hr & 1u) ^ 1u) : 0u;  // G order of the previous tile's outputs
      const uint32_t pv = ld32((par ? K.aLTs >> 16 : K.aLTs & 0xffffu) + ob);
      const uint32_t lv = (pv >> K.ltsh) & 0xffffu;
      st32(K.aLTd, lv);
      st32(K.aLTd + 256, spread16(lv));
      // ---- 4. the cells
      const uint64_t s1 = X + Y, Sm = s1 + M;
      const uint32_t carry = (uint32_t)(s1 < X) + (uint32_t)(Sm < s1);
      const uint64_t Z = X ^ Y, O = X & Y;
      const uint32_t Tl = sel32(K.madd, lo32(Sm), lo32(Z) & K.mzm), Th = sel32(K.madd, hi32(Sm), hi32(Z) & K.mzm);
      const uint32_t Ol = lo32(O), Oh = hi32(O);
      // w = rotr(z, 24) (XOR24) or rotr(z, 63) (XOR63)
      const uint32_t zu = sel32(K.mswap, lo32(Z), hi32(Z)), zv = sel32(K.mswap, hi32(Z), lo32(Z));
      const uint32_t Wl = __builtin_amdgcn_alignbit(zu, zv, K.rsh), Wh = __builtin_amdgcn_alignbit(zv, zu, K.rsh);
      uint32_t v[4];
#pragma unroll
      for (int j = 0; j < 4; j++) v[j] = perm(Ol, Tl, K.selL[j]) | perm(Oh, Th, K.selH[j]);
      // operand slots
      const uint32_t xA = perm(hi32(X), lo32(X), K.slA), xB = perm(hi32(X), lo32(X), K.slB);
      const uint32_t yA = perm(hi32(Y), lo32(Y), K.slA), yB = perm(hi32(Y), lo32(Y), K.slB);
      const uint32_t wA = perm(Wh, Wl, K.slA) & K.mhw, wB = perm(Wh, Wl, K.slB) & K.mhw;
      const uint32_t zA = (perm(hi32(Z), lo32(Z), K.slA) >> 15) & K.mhz;
      const uint32_t zB = (perm(hi32(Z), lo32(Z), K.slB) >> 15) & K.mhz;
      const uint32_t P3 = sel32(K.madd, hi32(X), spread16(xB)), Q3 = sel32(K.madd, lo32(X), spread16(xA));
      const uint32_t P4 = sel32(K.madd, hi32(Y), spread16(yB)), Q4 = sel32(K.madd, lo32(Y), spread16(yA));
      const uint32_t swA = spread16(wA), swB = spread16(wB);
      if (qlane || tlane) {  // tail lanes: the previous tile's quads 45-51, into rows -28 .. -1
        const uint64_t qrow = qlane ? c.row0 + 4ull * lane : c.row0 - HPRE + 4ull * (lane - TAIL0);
        uint32_t* const q = S + 4 * (qlane ? (int)lane : (int)lane - (TAIL0 + 7));  // rows -28 ..
        auto put = [&](int col, uint32_t v0, uint32_t v1, uint32_t v2, uint32_t v3) {
          emit_at<MODE>(q + col * HSTR, col, qrow, v0, v1, v2, v3, inj);
        };
        put(A0, tag_of(v[0]), tag_of(v[1]), tag_of(v[2]), tag_of(v[3]));
        put(A1, v[0], v[1], v[2], v[3]);
        put(A2, spread16(v[0]), spread16(v[1]), spread16(v[2]), spread16(v[3]));
        put(A3, perm(P3, Q3, K.slot[0]), perm(P3, Q3, K.slot[1]), perm(P3, Q3, K.slot[2]),
            perm(P3, Q3, K.slot[3]));
        put(A4, perm(P4, Q4, K.slot[0]), perm(P4, Q4, K.slot[1]), perm(P4, Q4, K.slot[2]),
            perm(P4, Q4, K.slot[3]));
        put(A5, perm(hi32(M), lo32(M), limb_sel(0)), perm(hi32(M), lo32(M), limb_sel(1)),
            perm(hi32(M), lo32(M), limb_sel(2)), perm(hi32(M), lo32(M), limb_sel(3)));
        put(A6, perm(zB, zA, K.slot[0]), perm(zB, zA, K.slot[1]), perm(zB, zA, K.slot[2]),
            perm(zB, zA, K.slot[3]));
        put(A7, perm(wB, wA, K.slot[0]), perm(wB, wA, K.slot[1]), perm(wB, wA, K.slot[2]),
            perm(wB, wA, K.slot[3]));
        put(A8, perm(swB, swA, K.slot[0]), perm(swB, swA, K.slot[1]), perm(swB, swA, K.slot[2]),
            perm(swB, swA, K.slot[3]));
        // last: these two columns hold the transient words until here
        put(A9, carry & K.madd, 0u, 0u, 0u);
        put(FXC, K.fx0, 0u, 0u, 0u);
      }
      tick(2);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's staging is complete
      __builtin_amdgcn_wave_barrier();
      // ---- 5. stores, then the wait for the next tile's word: vmcnt counts loads and stores
      // in issue order, so placed after this tile's 11 stores it is vmcnt(11) -- the load and
      // the PREVIOUS tile's stores, issued a tile ago -- never a wait for these stores
      tick(3);
      // Line ownership: a 208-row tile is 832 bytes per column, so tile boundaries fall inside
      // 128-byte lines, and a line written half by one wave and half by another was measured
      // 15-25 % slower to store (tools/store_probe.hip, profiles/r03i_store_probe_align.jsonl).
      // Each tile but an instance's first therefore also stores the previous tile's last kc
      // quads (the head of the line its first row sits in, kc = 0..7 per column, rows -4 kc ..), and
      // each tile but an instance's last leaves its last tc quads (the head of the line the next
      // tile starts in) to the next tile: every line inside the instance's half-rounds is
      // written by one store instruction of one wave.
      const bool own_head = c.hr != 0, own_tail = c.hr + 1 == 2 * c.rounds;
      const uint32_t r4 = 4u * (uint32_t)c.row0, tr4 = 4u * (uint32_t)total_rows;
      const uint32_t adv_lo = (uint32_t)reinterpret_cast<uintptr_t>(adv) + r4;
      const uint32_t fix_lo = (uint32_t)reinterpret_cast<uintptr_t>(fixed) + r4;
      auto store_col = [&](int col) {
        uint32_t* base = (col < 10 ? adv + (uint64_t)col * total_rows : fixed) + c.row0;
        // the line offset needs only the address's low bits
        const uint32_t ba = col < 10 ? adv_lo + (uint32_t)col * tr4 : fix_lo;
        const uint32_t kc = own_head ? (ba >> 4) & 7u : 0u;
        const uint32_t tc = own_tail ? 0u : ((ba + 16u * HR_Q) >> 4) & 7u;
        const int32_t sq = (int32_t)lane - (int32_t)kc;  // the staged quad this lane stores
        const uint32_t* src = S + col * HSTR + 4 * sq;  // sq < 0: the rows in front
        const uint4 v = *reinterpret_cast<const uint4*>(src);
        if (MODE & FZ_STORE) tile_store(base - 4 * kc, HR_Q + kc - tc, lane, v);
      };
#pragma unroll
      for (int col = 0; col < NSTAGE; col++) store_col(col);
      // the lookup and fixed checks read the lane's quad (lane_quad: its K program)
      const uint32_t ls = lane_quad(lane);
      const uint4 cq0 = *reinterpret_cast<const uint4*>(S + A0 * HSTR + 4 * ls);
      const uint4 cq1 = *reinterpret_cast<const uint4*>(S + A1 * HSTR + 4 * ls);
      const uint4 cq2 = *reinterpret_cast<const uint4*>(S + A2 * HSTR + 4 * ls);
      const uint4 cfx = *reinterpret_cast<const uint4*>(S + FXC * HSTR + 4 * ls);
      // ---- 6. fast checks: acc |= (every identity's lhs ^ rhs) -- hr_fast_checks, kept inline
      // here: called as a function it moved the register allocation (hot-loop spill reloads)
      uint32_t acc = 0;
      if (MODE & FZ_LOOKUP) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t de = comp(cq1, j);
          acc |= (de & 0xffff0000u) | (tag_of(de) ^ comp(cq0, j)) | (spread16(de) ^ comp(cq2, j));
        }
      }
      tick(4);
      asm volatile("" ::"v"(Pn));
      tick(7);
      if (MODE & FZ_GATES) {
        {  // XOR / XOR24 / XOR63 limb item
          const uint32_t gb = K.gb;
          const uint32_t x3 = ld32(gb + 4 * A3 * HSTR), x4 = ld32(gb + 4 * A4 * HSTR);
          const uint32_t s0 = ld32(gb + 4 * A2 * HSTR), s1v = ld32(gb + 4 * (A2 * HSTR + 1)), s2v = ld32(gb + 4 * (A2 * HSTR + 2));
          const uint32_t z6 = ld32(gb + 4 * A6 * HSTR), t0 = ld32(gb), t1 = ld32(gb + 4);
          const uint32_t w7 = ld32(gb + 4 * A7 * HSTR), w8 = ld32(gb + 4 * A8 * HSTR);
          const uint32_t E = ld32(K.ge), E2 = ld32(K.ge + 4 * (A2 - A1) * HSTR);
          const uint32_t F = ld32(K.gf), H = ld32(K.gf + 4 * (A2 - A1) * HSTR);
          const uint32_t R = s0 + perm(0u, s1v, K.gsel) + ((z6 << 30) & K.gm63) + 2 * sel32(K.gm24, s2v, s1v);
          acc |= (x3 + x4) ^ R;
          acc |= (t0 | (t1 & K.gm24) | (z6 & K.gm63)) & K.gnl;
          const uint32_t G = sel32(K.gm24, E2, E);
          acc |= (((E + (F << K.gsF)) ^ w7) | ((G + (H << K.gsH)) ^ w8)) & K.grs;
        }
        {  // ADD block (c_add_blk: each lane one of the 16, 4 lanes per block)
          const uint4 s = ld128(K.ar + 4 * A1 * HSTR), x = ld128(K.ar + 4 * A3 * HSTR);
          const uint4 y = ld128(K.ar + 4 * A4 * HSTR), z = ld128(K.ar + 4 * A5 * HSTR);
          const uint32_t a9 = ld32(K.ar + 4 * A9 * HSTR);
          int32_t cy = 0;
#pragma unroll
          for (int k = 0; k < 4; k++) {
            cy += (int32_t)(comp(x, k) + comp(y, k) + (comp(z, k) & K.m3) - comp(s, k));
            acc |= (uint32_t)cy & 0xffffu;
            cy >>= 16;
          }
          acc |= (uint32_t)cy ^ a9;
        }
      }
      if (MODE & FZ_GATES) acc |= (cfx.x ^ K.fx0) | cfx.y | cfx.z | cfx.w;
      if (MODE & FZ_COPIES) {
        const bool odd = c.hr & 1u;
#pragma unroll
        for (int it = 0; it < HR_CHECKS / FW; it++) {
          const uint32_t e = odd ? K.ce[1][it] : K.ce[0][it];
          acc |= ld32(e & 0xffffu) ^ ld32(e >> 16);
        }
        acc |= ld32(K.cm & 0xffffu) ^ ld16(K.cm >> 16);
      }
      bool bad = acc != 0;
      if (MODE & FZ_INJECT)  // the test hook: its instance is checked exactly
        bad |= inj.row >= c.off && inj.row < c.off + FIXED_ROWS + (uint64_t)ROUND_ROWS * c.rounds;
      tick(5);
      if (__builtin_amdgcn_ballot_w64(bad)) {  // rare: a failure in this tile, record it exactly
        Ctx c1;
        c1.kind = T_HR;
        c1.inst = c.inst;
        c1.rounds = c.rounds;
        c1.hr = c.hr;
        c1.nq = HR_Q;
        c1.off = c.off;
        c1.st = c.st;
        c1.row0 = c.row0;
        const HrTile T{S};
        const uint32_t* LT = S + H_LT;
        const uint64_t* MW = reinterpret_cast<const uint64_t*>(S + H_MW);
        auto state = [&](uint32_t w, uint32_t k, uint32_t sp) { return LT[64 * sp + 4 * w + k]; };
        Fails<true> Rf{A, false};
        hr_msg_copies<MODE, true>(Rf, T, lane, c1, MW[2 * ((lane >> 3) & 3u) + ((lane >> 2) & 1u)], Sg, inj);
        hr_checks<MODE, true>(Rf, T, lane, c1, &c_hr_checks.e[c.hr & 1u][0], state, inj, defer, defer_cap);
      }
      // the staging is rewritten by the next tile: keep the compiler from hoisting those writes
      // above this tile's reads (the wave's LDS operations execute in order)
      asm volatile("" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      tick(6);
      if (c.hr + 1 < hr_end) {
        c.hr++;
      } else {  // the unit (an instance's first segment, or a listed segment) is done
        fresh = true;
        inst = ninst;
        Pi = Pn;
      }
    }
    if (!B2F_EDGE_SEPARATE)  // then the edge tiles, in the wave's whole region
      edge_walk<MODE>(L + H_WAVE + wv * HW_WORDS, lane, w0, W, IV, Sg, A, in, n, off, total_rows, rec,
                      adv, fixed, redo, inj, defer, defer_cap,
                      B2F_FUSED_DYN && B2F_FUSED_EDGE_DYN ? ictr + 1 : nullptr);
  }
  if ((MODE & FZ_CLOCK) && lane == 0) {
#pragma unroll
    for (int k = 0; k < 8; k++) atomicAdd(&clk[8 * wv + k], (unsigned long long)ck[k]);
  }
  __syncthreads();
  flush_report(A, rep, tid);
}

// ============================================================================================
// The edge launch (fused_edge_kernel): ONE wave tile per instance holds both of its edge
// regions -- the init region on lanes 0-40 (INW h / m / t, FMASK, CONST IV, XOR v12..v14) and the
// final region on lanes 41-56 (XOR3 + digest), so the init region's h cells (the XOR3 H operands'
// copy sources) are staged in the same tile; lanes 57-60 recompute the final state from the last
// half-round (the XOR3 V / U operands' producer values). The zero rows past the last instance
// follow as 64-quad tiles. Fast 32-bit checks as in the half-round launch; a flagged tile is done
// again, region by region, by the exact edge path (edge_tile: assignment, stores, exact checks).
namespace edge2 {
constexpr uint32_t NQ_I = INIT_Q, NQ_F = FINAL_Q, NQ = INIT_Q + FINAL_Q;  // 41, 16, 57
constexpr int STR_E = 232;  // staged rows per column: init rows 0-163, final rows 164-227
static_assert(4 * NQ_I == INIT_ROWS && 4 * NQ <= (uint32_t)STR_E && STR_E % 4 == 0, "lane = quad, rows 4 lane");
enum : uint32_t { E_INW = 1, E_FMASK = 2, E_CONST = 4, E_XOR = 8, E_XOR3 = 16 };
struct EdgeProg {
  uint32_t selL[4], selH[4];  // a_1 of row j = perm(O_lo, T_lo, selL) | perm(O_hi, T_hi, selH)
  uint32_t kind, qq, a;       // block kind, quad inside an XOR / XOR3 block, word index
};
struct EdgeProgs {
  EdgeProg e[NQ];
};
constexpr EdgeProgs make_edge_progs() {
  EdgeProgs P{};
  for (uint32_t l = 0; l < NQ; l++) {
    EdgeProg& g = P.e[l];
    uint32_t kind = 0, qq = 0, a = 0;
    if (l < 26) {
      kind = E_INW;
      a = l;
    } else if (l == 26) {
      kind = E_FMASK;
    } else if (l < 35) {
      kind = E_CONST;
      a = l - 27;
    } else if (l < NQ_I) {
      kind = E_XOR;
      a = (l - 35) >> 1;
      qq = (l - 35) & 1u;
    } else {
      kind = E_XOR3;
      a = (l - NQ_I) >> 1;
      qq = (l - NQ_I) & 1u;
    }
    g.kind = kind;
    g.qq = qq;
    g.a = a;
    for (uint32_t j = 0; j < 4; j++) {
      const bool xr = kind & (E_XOR | E_XOR3);
      const uint32_t k = xr ? 2 * qq + (j >> 1) : j, so = (xr && (j & 1u)) ? 4u : 0u;  // XOR: rows 2h z/e, 2h+1 o/maj
      const uint32_t half = k >> 1, bb = 2 * (k & 1u);
      const uint32_t sel = hr2::psel(bb + so, bb + 1 + so, 12, 12);
      g.selL[j] = half == 0 ? sel : hr2::PZ;
      g.selH[j] = half == 1 ? sel : hr2::PZ;
    }
  }
  return P;
}
__constant__ EdgeProgs c_eprogs = make_edge_progs();

// Copy checks of an edge tile (120): the init XORs' operands (IV_4..6 from the CONST blocks, t0 /
// t1 / fmask from their INW / FMASK blocks) and the XOR3 operands (H from the INW h blocks, V and
// U from the final state's producer values). Entry: dst row (bits 0-7), dst column a_3 + c
// (8-9), source kind (10: 0 staged a_2 cell at row bits 11-18, 1 limb-table entry bits 11-16).
constexpr int E_CHECKS = 120;
struct EdgeChecks {
  uint32_t e[128];
};
constexpr EdgeChecks make_edge_checks() {
  EdgeChecks T{};
  uint32_t n = 0;
  for (uint32_t a = 0; a < 3; a++)
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t row = 140 + 8 * a + 2 * k;
      T.e[n++] = row | (0u << 8) | ((108 + 4 * (4 + a) + k) << 11);
      T.e[n++] = row | (1u << 8) | ((a < 2 ? 96 + 4 * a + k : 104 + k) << 11);
    }
  for (uint32_t i = 0; i < 8; i++)
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t row = INIT_ROWS + 8 * i + 2 * k;
      T.e[n++] = row | (0u << 8) | ((4 * i + k) << 11);
      T.e[n++] = row | (1u << 8) | (1u << 10) | ((4 * i + k) << 11);
      T.e[n++] = row | (2u << 8) | (1u << 10) | ((4 * (i + 8) + k) << 11);
    }
  for (uint32_t i = n; i < 128; i++) T.e[i] = T.e[i - n];  // duplicates fill the last lanes
  if (n != E_CHECKS) T.e[0] = 0xffffffffu;
  return T;
}
static_assert(make_edge_checks().e[0] != 0xffffffffu, "120 edge copy checks");
__constant__ EdgeChecks c_echecks = make_edge_checks();

// wave LDS (words): staging [11][STR_E], limb table (spread limbs of the final state, 4 w + k),
// producer outputs (16 u64 by word). The exact edge path (edge_tile, in edge_redo_kernel) reuses the same words with
// its own carve (staging [11][208], prod, canonical flags), inside this one.
constexpr int E_LT = NSTAGE * STR_E;
constexpr int E_PROD = E_LT + 64;
constexpr int EW_WORDS = E_PROD + 32;
static_assert(EW_WORDS >= WAVE_WORDS, "the exact edge path's carve fits");
static_assert(EW_WORDS <= hr2::HW_WORDS, "the half-round launch's wave region holds an edge tile");
constexpr int E_ACC = 0, E_IV = 24, E_SG = E_IV + 16, E_WAVE = E_SG + 40;
constexpr int E_WORDS = E_WAVE + WAVES * EW_WORDS;
static_assert(E_WAVE % 4 == 0 && EW_WORDS % 4 == 0 && E_PROD % 2 == 0, "aligned carve");
static_assert(4 * E_WORDS < 65536, "LDS byte addresses fit 16 bits");

// store of one region of an edge tile: lane `lane` writes quad lane - q0 of the region
__device__ __forceinline__ void region_store(uint32_t* base, uint32_t nq, uint32_t lane, uint32_t q0, uint4 v) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const i32x4 rsrc = {(int32_t)(uint32_t)a, (int32_t)(uint32_t)(a >> 32), (int32_t)(nq * 16u), 0x00020000};
  b2f_raw_buffer_store_v4(i32x4{(int32_t)v.x, (int32_t)v.y, (int32_t)v.z, (int32_t)v.w}, rsrc,
                          (int)(16u * (lane - q0)), 0, EDGE_NT);  // lanes outside: past the range
}

struct ECtx {
  uint32_t inst, rounds;
  uint64_t off, st;
};
}  // namespace edge2

// One column of an edge tile's quad into the staging (STR_E rows per column), the test-only
// injection applied as emit applies it.
template <int MODE>
__device__ __forceinline__ void stage_e(uint32_t* S, int col, uint32_t lane, uint64_t qrow, uint32_t v0,
                                        uint32_t v1, uint32_t v2, uint32_t v3, const Inject& inj) {
  if (MODE & FZ_INJECT) {
    if ((inj.row >> 2) == (qrow >> 2) && inj.col == (uint32_t)col) {
      const uint32_t j = (uint32_t)inj.row & 3u;
      v0 ^= j == 0 ? inj.mask : 0u;
      v1 ^= j == 1 ? inj.mask : 0u;
      v2 ^= j == 2 ? inj.mask : 0u;
      v3 ^= j == 3 ? inj.mask : 0u;
    }
  }
  *reinterpret_cast<uint4*>(S + col * edge2::STR_E + 4 * lane) = make_uint4(v0, v1, v2, v3);
}


// Per-lane constants of an edge tile (lane = quad of the init region 0-40 / final region 41-56;
// lanes >= 57 check a repeat of quads 0-6).
struct ELane {
  uint32_t selL[4], selH[4];
  uint32_t kind, qq, a;
  uint32_t mINW, mFM, mCONST, mX3, mXOR, m78, mDG;
  uint4 fxq;          // the keygen fixed cells of the quad
  uint32_t aQ, aQn;   // the quad's and the next quad's staged rows (column a_0)
  uint32_t ce[2];     // copy checks (dst | src << 16)
};
__device__ __forceinline__ ELane make_elane(uint32_t lane, uint32_t Sb, const uint64_t* IV) {
  using namespace edge2;
  ELane E;
  const uint32_t lq = lane < NQ ? lane : lane - NQ;
  const EdgeProg& G = c_eprogs.e[lq];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    E.selL[j] = G.selL[j];
    E.selH[j] = G.selH[j];
  }
  E.kind = G.kind;
  E.qq = G.qq;
  E.a = G.a;
  const uint32_t kind = G.kind, qq = G.qq;
  E.mINW = kind == E_INW ? ~0u : 0u;
  E.mFM = kind == E_FMASK ? ~0u : 0u;
  E.mCONST = kind == E_CONST ? ~0u : 0u;
  E.mX3 = kind == E_XOR3 ? ~0u : 0u;
  E.mXOR = (kind & (E_XOR | E_XOR3)) ? ~0u : 0u;
  E.m78 = E.mINW | (qq == 0 ? E.mX3 : 0u);
  E.mDG = qq == 0 ? E.mX3 : 0u;
  uint4 fxq = make_uint4(0, 0, 0, 0);
  if (kind == E_INW) fxq.x = 1u << S_ABCD;
  if (kind == E_FMASK) fxq.x = 1u << S_FMASK;
  if (kind == E_XOR && qq == 0) fxq.x = 1u << S_XOR;
  if (kind == E_XOR3 && qq == 0) fxq.x = (1u << S_XOR3) | (1u << S_DIGEST);
  if (kind == E_CONST) {
    const uint64_t w = IV[G.a];
    fxq = make_uint4((1u << S_CONST) | ((uint32_t)(w & 0xffffu) << 16), (1u << S_CONST) | ((uint32_t)((w >> 16) & 0xffffu) << 16),
                     (1u << S_CONST) | ((uint32_t)((w >> 32) & 0xffffu) << 16), (1u << S_CONST) | ((uint32_t)(w >> 48) << 16));
  }
  E.fxq = fxq;
  E.aQ = Sb + 16 * lq;
  E.aQn = Sb + 16 * (lq + 1);
#pragma unroll
  for (int it = 0; it < 2; it++) {
    const uint32_t e = c_echecks.e[it * FW + lane];
    const uint32_t dst = Sb + 4 * ((A3 + ((e >> 8) & 3u)) * STR_E + (e & 255u));
    const uint32_t src = (e >> 10) & 1u ? Sb + 4 * (E_LT + ((e >> 11) & 63u)) : Sb + 4 * (A2 * STR_E + ((e >> 11) & 255u));
    E.ce[it] = dst | (src << 16);
  }
  return E;
}

// The fast checks of a staged edge tile: lookups, the fixed column, the INW / FMASK / CONST /
// XOR / XOR3 / digest identities of each lane's quad, the 120 copies (staging and limb table).
template <int MODE>
__device__ __forceinline__ uint32_t edge_fast_checks(const ELane& E) {
  using namespace hr2;
  using namespace edge2;
  uint32_t acc = 0;
  {
    const uint4 q0 = ld128(E.aQ + 4 * A0 * STR_E), q1 = ld128(E.aQ + 4 * A1 * STR_E), q2 = ld128(E.aQ + 4 * A2 * STR_E);
    const uint4 q3 = ld128(E.aQ + 4 * A3 * STR_E), q4 = ld128(E.aQ + 4 * A4 * STR_E), q5 = ld128(E.aQ + 4 * A5 * STR_E);
    const uint4 q7 = ld128(E.aQ + 4 * A7 * STR_E), q8 = ld128(E.aQ + 4 * A8 * STR_E), fx = ld128(E.aQ + 4 * FXC * STR_E);
    const uint4 n1 = ld128(E.aQn + 4 * A1 * STR_E);
    if (MODE & FZ_LOOKUP) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t de = comp(q1, j);
        acc |= (de & 0xffff0000u) | (tag_of(de) ^ comp(q0, j)) | (spread16(de) ^ comp(q2, j));
      }
    }
    if (MODE & FZ_GATES) {
      acc |= (fx.x ^ E.fxq.x) | (fx.y ^ E.fxq.y) | (fx.z ^ E.fxq.z) | (fx.w ^ E.fxq.w);
      // INW: a_7 = a_1@0 + 2^16 a_1@1, a_8 = a_1@2 + 2^16 a_1@3
      acc |= ((q7.x ^ (q1.x + (q1.y << 16))) | (q8.x ^ (q1.z + (q1.w << 16)))) & E.mINW;
      // FMASK: a_5 in {0, 1}, a_1@k = 65535 a_5
      const uint32_t fm = (0u - q5.x) & 0xffffu;
      acc |= ((q5.x >> 1) | (q1.x ^ fm) | (q1.y ^ fm) | (q1.z ^ fm) | (q1.w ^ fm)) & E.mFM;
      // CONST: a_1 = k_0 on every row
      acc |= ((q1.x ^ (fx.x >> 16)) | (q1.y ^ (fx.y >> 16)) | (q1.z ^ (fx.z >> 16)) | (q1.w ^ (fx.w >> 16))) & E.mCONST;
      // XOR / XOR3 limbs of the quad (rows 0 and 2)
      acc |= (((q3.x + q4.x + (q5.x & E.mX3)) ^ (q2.x + 2 * q2.y)) | ((q3.z + q4.z + (q5.z & E.mX3)) ^ (q2.z + 2 * q2.w))) & E.mXOR;
      // digest: a_7 = a_1@0 + 2^16 a_1@2, a_8 = a_1@4 + 2^16 a_1@6 (the next quad's rows 0, 2)
      acc |= ((q7.x ^ (q1.x + (q1.z << 16))) | (q8.x ^ (n1.x + (n1.z << 16)))) & E.mDG;
    }
  }
  if (MODE & FZ_COPIES) {
#pragma unroll
    for (int it = 0; it < 2; it++) acc |= ld32(E.ce[it] & 0xffffu) ^ ld32(E.ce[it] >> 16);
  }
  return acc;
}

// The edge tiles t_first, t_first + W, ... of a batch (one per instance, then the zero rows past
// the last instance) on this wave, staged in the wave region S (EW_WORDS words): the body of the
// edge launch, and the last phase of the half-round launch (each wave walks edge tiles once its
// instances and listed segments are done, so the edge work fills the half-round launch's tail
// instead of waiting for it).
template <int MODE>
__device__ __forceinline__ void edge_walk(uint32_t* S, uint32_t lane, uint64_t t_first, uint64_t W,
                                          const uint64_t* IV, const uint8_t* Sg, EvalAcc& A,
                                          const b2f_input* __restrict__ in, uint32_t n,
                                          const uint64_t* __restrict__ off, uint64_t total_rows,
                                          const uint64_t* __restrict__ rec, uint32_t* __restrict__ adv,
                                          uint32_t* __restrict__ fixed, uint32_t* __restrict__ redo,
                                          const Inject& inj, uint64_t* __restrict__ defer,
                                          uint32_t defer_cap, unsigned* __restrict__ ectr) {
  using namespace hr2;
  using namespace edge2;
  const uint32_t Sb = lds_byte(S);
  uint64_t* prod = reinterpret_cast<uint64_t*>(S + E_PROD);
  // per-lane constants
  const ELane E = make_elane(lane, Sb, IV);
  const uint32_t kind = E.kind, qq = E.qq, wa = E.a;
  const uint32_t mFM = E.mFM, mX3 = E.mX3, mXOR = E.mXOR, m78 = E.m78;
  const uint4 fxq = E.fxq;
  const bool plane = lane >= NQ && lane < NQ + 4;
  const uint32_t pg = lane - NQ;

  {
    const uint64_t used_rows = off[n];
    const uint64_t n_pad = ((total_rows - used_rows) / 4 + PAD_Q - 1) / PAD_Q;
    const uint64_t t_all = (uint64_t)n + n_pad;
    // edge tiles t, t + W, ... from t_first, or (ectr) claimed from the launch's counter: a wave
    // holds the tile it works on and the next two, whose context it loads ahead
    // (B2F_FUSED_EDGE_CHUNK consecutive tiles per claim)
    uint32_t cleft = 0;
    uint64_t cbase = 0;
    auto claim = [&]() -> uint64_t {
      if (cleft == 0) {
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(ectr, (unsigned)B2F_FUSED_EDGE_CHUNK);
        cbase = __builtin_amdgcn_readfirstlane(v);
        cleft = B2F_FUSED_EDGE_CHUNK;
      }
      cleft--;
      return cbase++;
    };
    uint64_t t = ectr ? claim() : t_first;
    uint64_t t1 = ectr ? claim() : t + W;
    auto ectx = [&](uint64_t tt) {
      ECtx c;
      const uint32_t i = tt < n ? (uint32_t)tt : 0u;
      c.inst = i;
      c.off = off[i];
      c.rounds = in[i].rounds;
      c.st = 2 * ((c.off - (uint64_t)FIXED_ROWS * i) / ROUND_ROWS) + i;
      return c;
    };
    // the words of one tile: init lanes their block's word, final lanes h_i and the final state's
    // v_i, v_{i+8}; producer lanes the last half-round's G operands (or the initial words at 0 rounds)
    auto words = [&](const ECtx& c) {
      const b2f_input* x = in + c.inst;
      const uint64_t* fw = reinterpret_cast<const uint64_t*>(&x->rounds);  // rounds | f << 32
      const uint64_t* p[6] = {fw, fw, fw, fw, fw, fw};
      if (lane < 26) {
        p[0] = lane < 8 ? x->h + lane : lane < 24 ? x->m + (lane - 8) : x->t + (lane - 24);
      } else if (lane >= 35 && lane < NQ_I) {
        const uint32_t a = (lane - 35) >> 1;
        p[0] = a < 2 ? x->t + a : fw;
      } else if (lane >= NQ_I && lane < NQ) {
        const uint32_t i = (lane - NQ_I) >> 1;
        const uint64_t* fin = rec + 16ull * (c.st + 2ull * c.rounds);
        p[0] = x->h + i;
        p[1] = fin + i;
        p[2] = fin + i + 8;
      } else if (plane) {
        if (c.rounds == 0) {
          p[0] = x->h + pg;
          p[1] = x->h + pg + 4;
          p[3] = pg < 2 ? x->t + pg : fw;
        } else {
          const uint32_t hp = 2 * c.rounds - 1, g = pg + 4;  // the last half-round: diagonal G's
          const uint64_t* s = rec + 16ull * (c.st + hp);
          const uint32_t gi = gidx_word(g);
          const uint8_t* sg = Sg + 16 * ((hp >> 1) % 10) + 2 * g;
          p[0] = s + (gi & 15u);
          p[1] = s + ((gi >> 8) & 15u);
          p[2] = s + ((gi >> 16) & 15u);
          p[3] = s + ((gi >> 24) & 15u);
          p[4] = x->m + sg[0];
          p[5] = x->m + sg[1];
        }
      }
      Ops o;
#pragma unroll
      for (int k = 0; k < 6; k++) o.w[k] = *p[k];
      o.w[6] = 0;
      return o;
    };
    ECtx c = ectx(t);
    Ops P = words(c);  // past the instances: instance 0's words (harmless, unused)
    settle(P);
    ECtx cn = ectx(t1);
    while (t < t_all) {
      const uint64_t t2 = ectr ? claim() : t1 + W;
      const ECtx cnn = ectx(t2);  // scalar loads, two tiles ahead
      const Ops Pn = words(cn);         // unconditional: the compiler counts vmcnt exactly
      if (t < n) {
        // ---- one instance's init + final regions
        const uint64_t row_i = c.off, row_f = c.off + INIT_ROWS + (uint64_t)ROUND_ROWS * c.rounds;
        const uint64_t qrow = lane < NQ_I ? row_i + 4ull * lane : row_f + 4ull * (lane - NQ_I);
        const uint64_t w0 = P.w[0];
        const bool fbit = (w0 >> 32) != 0;
        uint64_t X = 0, Y = 0, U = 0, T, O = 0;
        if (kind == E_CONST) {
          T = IV[wa];
        } else if (kind == E_FMASK) {
          T = fbit ? ~0ull : 0ull;
        } else if (kind == E_XOR) {
          X = IV[4 + wa];
          Y = wa < 2 ? w0 : (fbit ? ~0ull : 0ull);
          T = X ^ Y;
          O = X & Y;
        } else if (kind == E_XOR3) {
          X = w0;
          Y = P.w[1];
          U = P.w[2];
          T = X ^ Y ^ U;
          O = (X & Y) | (X & U) | (Y & U);
        } else {
          T = w0;
        }
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] = perm(lo32(O), lo32(T), E.selL[j]) | perm(hi32(O), hi32(T), E.selH[j]);
        const uint32_t sl0 = limb_sel(2 * qq), sl1 = limb_sel(2 * qq + 1);
        const uint32_t sx0 = spread16(perm(hi32(X), lo32(X), sl0)) & mXOR, sx1 = spread16(perm(hi32(X), lo32(X), sl1)) & mXOR;
        const uint32_t sy0 = spread16(perm(hi32(Y), lo32(Y), sl0)) & mXOR, sy1 = spread16(perm(hi32(Y), lo32(Y), sl1)) & mXOR;
        const uint32_t su0 = spread16(perm(hi32(U), lo32(U), sl0)) & mX3, su1 = spread16(perm(hi32(U), lo32(U), sl1)) & mX3;
        const uint32_t a5r0 = (su0 & mX3) | ((fbit ? 1u : 0u) & mFM);
        if (lane < NQ) {
          stage_e<MODE>(S, A0, lane, qrow, tag_of(v[0]), tag_of(v[1]), tag_of(v[2]), tag_of(v[3]), inj);
          stage_e<MODE>(S, A1, lane, qrow, v[0], v[1], v[2], v[3], inj);
          stage_e<MODE>(S, A2, lane, qrow, spread16(v[0]), spread16(v[1]), spread16(v[2]), spread16(v[3]), inj);
          stage_e<MODE>(S, A3, lane, qrow, sx0, 0u, sx1, 0u, inj);
          stage_e<MODE>(S, A4, lane, qrow, sy0, 0u, sy1, 0u, inj);
          stage_e<MODE>(S, A5, lane, qrow, a5r0, 0u, su1, 0u, inj);
          stage_e<MODE>(S, A6, lane, qrow, 0u, 0u, 0u, 0u, inj);
          stage_e<MODE>(S, A7, lane, qrow, lo32(T) & m78, 0u, 0u, 0u, inj);
          stage_e<MODE>(S, A8, lane, qrow, hi32(T) & m78, 0u, 0u, 0u, inj);
          stage_e<MODE>(S, A9, lane, qrow, 0u, 0u, 0u, 0u, inj);
          stage_e<MODE>(S, FXC, lane, qrow, fxq.x, fxq.y, fxq.z, fxq.w, inj);
        }
        if (plane) producer_words(prod, P, pg, c.rounds == 0, 2 * c.rounds - 1, IV);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        {  // limb table: spread limb (lane & 3) of final state word lane >> 2
          const uint32_t lv = limb(prod[lane >> 2], lane & 3u);
          S[E_LT + lane] = spread16(lv);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        // ---- stores: the init region (lanes 0-40) and the final region (lanes 41-56)
        if (MODE & FZ_STORE) {
          const uint32_t l = lane < NQ ? lane : 0;
#pragma unroll
          for (int col = 0; col < NSTAGE; col++) {
            const uint4 cv = *reinterpret_cast<const uint4*>(S + col * STR_E + 4 * l);
            uint32_t* base = col < 10 ? adv + (uint64_t)col * total_rows : fixed;
            region_store(base + row_i, NQ_I, lane, 0, cv);
            region_store(base + row_f, NQ_F, lane, NQ_I, cv);
          }
        }
        asm volatile("" ::"v"(Pn.w[0]), "v"(Pn.w[1]), "v"(Pn.w[2]), "v"(Pn.w[3]), "v"(Pn.w[4]), "v"(Pn.w[5]));
        // ---- fast checks
        const uint32_t acc = edge_fast_checks<MODE>(E);
        bool bad = acc != 0;
        if (MODE & FZ_INJECT)  // the test hook: its instance is checked exactly
          bad |= inj.row >= c.off && inj.row < c.off + FIXED_ROWS + (uint64_t)ROUND_ROWS * c.rounds;
        // rare: the instance goes to the redo list (edge_redo_kernel: the exact edge path,
        // exact bookkeeping); a list slot per instance, so it cannot overflow
        if (__builtin_amdgcn_ballot_w64(bad) && lane == 0) {
          const uint32_t slot = atomicAdd(redo, 1u);
          redo[1 + slot] = c.inst;
        }
      } else {
        // ---- the zero rows past the last instance: written and checked from registers (a
        // selector here can only come from the test hook, and its gate is deferred)
        const uint64_t row0 = used_rows + (uint64_t)PAD_Q * 4 * (t - n);
        const uint64_t left = row0 < total_rows ? (total_rows - row0) >> 2 : 0;
        const uint32_t nq = (uint32_t)(left < PAD_Q ? left : PAD_Q);
        const uint64_t qrow = row0 + 4ull * lane;
        Quad Q;
        zero(Q);
        if (MODE & FZ_INJECT) {
          if ((inj.row >> 2) == (qrow >> 2)) {
            const uint32_t j = (uint32_t)inj.row & 3u;
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
#pragma unroll
              for (int cc = 0; cc < 10; cc++)
                if ((uint32_t)cc == inj.col && (uint32_t)jj == j) Q.c[cc][jj] ^= inj.mask;
              if (inj.col == 10 && (uint32_t)jj == j) Q.fx[jj] ^= inj.mask;
            }
          }
        }
        if (MODE & FZ_STORE) {
#pragma unroll
          for (int cc = 0; cc < 11; cc++)
            tile_store((cc < 10 ? adv + (uint64_t)cc * total_rows : fixed) + row0, nq, lane,
                       cc < 10 ? make_uint4(Q.c[cc][0], Q.c[cc][1], Q.c[cc][2], Q.c[cc][3])
                               : make_uint4(Q.fx[0], Q.fx[1], Q.fx[2], Q.fx[3]));
        }
        asm volatile("" ::"v"(Pn.w[0]), "v"(Pn.w[1]), "v"(Pn.w[2]), "v"(Pn.w[3]), "v"(Pn.w[4]), "v"(Pn.w[5]));
        if (lane < nq) {
          const uint4 fx = make_uint4(Q.fx[0], Q.fx[1], Q.fx[2], Q.fx[3]);
          if (MODE & FZ_LOOKUP)
            check_lookups(A, make_uint4(Q.c[A0][0], Q.c[A0][1], Q.c[A0][2], Q.c[A0][3]),
                          make_uint4(Q.c[A1][0], Q.c[A1][1], Q.c[A1][2], Q.c[A1][3]),
                          make_uint4(Q.c[A2][0], Q.c[A2][1], Q.c[A2][2], Q.c[A2][3]), qrow);
          if (MODE & FZ_GATES) {
            check_fixed(A, fx, make_uint4(0, 0, 0, 0), qrow);
            defer_rows(fx, qrow, defer, defer_cap);
          }
        }
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      c = cn;
      cn = cnn;
      P = Pn;
      t = t1;
      t1 = t2;
    }
    }
}

#ifndef B2F_EDGE_WAVES
#define B2F_EDGE_WAVES 3  // waves per SIMD the edge kernel is compiled for (VGPR budget)
#endif
template <int MODE>
__global__ void __launch_bounds__(FW * WAVES, B2F_EDGE_WAVES)
fused_edge_kernel(const b2f_input* __restrict__ in, uint32_t n, const uint64_t* __restrict__ off,
                  uint64_t total_rows, const uint64_t* __restrict__ rec, uint32_t* __restrict__ adv,
                  uint32_t* __restrict__ fixed, uint32_t* __restrict__ redo,
                  b2f_eval_report* __restrict__ rep, const int* __restrict__ status, Inject inj,
                  uint64_t* __restrict__ defer, uint32_t defer_cap, unsigned long long* __restrict__ clk) {
  using namespace hr2;
  using namespace edge2;
  (void)clk;
  __shared__ __attribute__((aligned(16))) uint32_t L[E_WORDS];
  const int tid = threadIdx.x;
  const uint32_t lane = (uint32_t)tid & 63u, wv = (uint32_t)tid >> 6;
  if (tid < 22) L[E_ACC + tid] = 0;
  if (tid == 22) *reinterpret_cast<uint64_t*>(L + E_ACC + 20) = ~0ull;
  if (tid < 16) L[E_IV + tid] = reinterpret_cast<const uint32_t*>(c_iv)[tid];
  if (tid < 40) L[E_SG + tid] = reinterpret_cast<const uint32_t*>(c_sigma)[tid];
  __syncthreads();
  EvalAcc A{L + E_ACC};
  const uint64_t* IV = reinterpret_cast<const uint64_t*>(L + E_IV);
  const uint8_t* Sg = reinterpret_cast<const uint8_t*>(L + E_SG);
  uint32_t* S = L + E_WAVE + wv * EW_WORDS;

  if (*status == 0)
    edge_walk<MODE>(S, lane, first_tile(blockIdx.x, __builtin_amdgcn_readfirstlane(wv), gridDim.x),
                    (uint64_t)gridDim.x * WAVES, IV, Sg, A, in, n, off, total_rows, rec, adv, fixed,
                    redo, inj, defer, defer_cap, nullptr);
  __syncthreads();
  flush_report(A, rep, tid);
}

// The edge regions of the instances the edge launch flagged, done again by the exact edge
// path (assignment and stores repeated with the same values, every check recorded exactly).
template <int MODE>
__global__ void __launch_bounds__(FW * WAVES)
edge_redo_kernel(const b2f_input* __restrict__ in, const uint64_t* __restrict__ off,
                 uint64_t total_rows, const uint64_t* __restrict__ rec, uint32_t* __restrict__ adv,
                 uint32_t* __restrict__ fixed, const uint32_t* __restrict__ redo,
                 b2f_eval_report* __restrict__ rep, const int* __restrict__ status, Inject inj,
                 uint64_t* __restrict__ defer, uint32_t defer_cap) {
  __shared__ __attribute__((aligned(16))) uint32_t L[L_WAVE + WAVES * WAVE_WORDS];
  const int tid = threadIdx.x;
  const uint32_t lane = (uint32_t)tid & 63u, wv = (uint32_t)tid >> 6;
  if (tid < 22) L[L_ACC + tid] = 0;
  if (tid == 22) *reinterpret_cast<uint64_t*>(L + L_ACC + 20) = ~0ull;
  if (tid < 16) L[L_IV + tid] = reinterpret_cast<const uint32_t*>(c_iv)[tid];
  if (tid < 40) L[L_SG + tid] = reinterpret_cast<const uint32_t*>(c_sigma)[tid];
  __syncthreads();
  const uint64_t* IV = reinterpret_cast<const uint64_t*>(L + L_IV);
  const uint8_t* Sg = reinterpret_cast<const uint8_t*>(L + L_SG);
  uint32_t* S = L + L_WAVE + wv * WAVE_WORDS;
  if (*status == 0) {
    const uint32_t cnt = redo[0];
    for (uint32_t k = blockIdx.x * WAVES + wv; k < cnt; k += gridDim.x * WAVES) {
      const uint32_t i = __builtin_amdgcn_readfirstlane(redo[1 + k]);
#pragma unroll 1
      for (int part = 0; part < 2; part++) {
        Ctx c;
        c.inst = i;
        c.rounds = in[i].rounds;
        c.off = off[i];
        c.st = 2 * ((c.off - (uint64_t)FIXED_ROWS * i) / ROUND_ROWS) + i;
        c.kind = part ? T_FINAL : T_INIT;
        c.hr = 0;
        c.nq = part ? FINAL_Q : INIT_Q;
        c.row0 = part ? c.off + INIT_ROWS + (uint64_t)ROUND_ROWS * c.rounds : c.off;
        const Ops P = load_ops(c, lane, in, rec, Sg);
        settle(P);
        edge_tile<MODE>(S, L + L_ACC, IV, inj, adv, fixed, total_rows, defer, defer_cap, c, P, lane);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
      }
    }
  }
  __syncthreads();
  EvalAcc A{L + L_ACC};
  flush_report(A, rep, tid);
}

// ============================================================================================
// The eval's fast clean-check pass (b2f_eval_dev): the same wave tiles, lane programs and fast
// checks as the fused path, on a GIVEN trace -- the tile's cells are loaded instead of assigned,
// and every copy source is the source cell in the trace (the state words' canonical cells at the
// half-round start, the message words' INW cells, the final state's canonical cells), gathered
// into the limb table. A pass that finds nothing proves the trace clean: the report
// report_init_kernel wrote is the verdict. Anything it flags (a failure, or a range a check
// assumes) sets `dirty`, and the exact eval kernel then evaluates the whole trace and writes the
// report (MockProver's counters and first failing row).

// half-round tile descriptors from the row map alone (the eval has no input records): a thread
// per tile T, whose instance is the last i with 2 R_i <= T (R_i = (off_i - 228 i) / 416, the
// rounds before instance i; instances without rounds own no tile). One search over the row map
// per wave (its first tile), then the wave loads 2 R of the next 64 instances (one
// coalesced load) and each lane finds its instance among them by a 6-step shuffle search; a lane
// whose tile lies past them (possible only after runs of zero-round instances) searches the row
// map itself. The descriptors go out as whole lines. (Round 5: a thread per instance wrote its
// 2 rounds descriptors 384 bytes apart from its neighbours', 73 us per 2^18 x 12 call; a thread
// per tile with its own 18-step search over the row map, 96 us; the per-wave search starts from the
// interpolated instance, so a uniform batch needs two row-map loads per wave.)
__global__ void __launch_bounds__(256) eval_desc_kernel(const uint64_t* __restrict__ off, uint32_t n,
                                                        TileDesc* __restrict__ desc,
                                                        const int* __restrict__ status) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t T = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, T0 = T - lane;
  if (*status) return;
  auto R2 = [&](uint32_t i) { return 2 * ((off[i] - (uint64_t)FIXED_ROWS * i) / ROUND_ROWS); };
  const uint64_t tiles = R2(n);
  if (T0 >= tiles) return;
  auto search = [&](uint64_t t) {  // last i < n with R2(i) <= t (R2(0) = 0 <= t < R2(n))
    // the bracket [lo, hi) around the interpolated guess t n / tiles (exact for uniform rounds),
    // widened by doubling steps, then bisected
    uint32_t g = (uint32_t)((double)t / (double)tiles * (double)n);
    g = g < n ? g : n - 1;
    uint32_t lo, hi;
    if (R2(g) <= t) {
      lo = g;
      uint32_t step = 1;
      hi = g + 1;
      while (hi < n && R2(hi) <= t) {
        lo = hi;
        hi = n - hi > step ? hi + step : n;
        step *= 2;
      }
    } else {
      hi = g;
      uint32_t step = 1;
      lo = g > step ? g - step : 0;
      while (lo > 0 && R2(lo) > t) {
        hi = lo;
        step *= 2;
        lo = lo > step ? lo - step : 0;
      }
    }
    while (hi - lo > 1) {
      const uint32_t mid = lo + (hi - lo) / 2;
      if (R2(mid) <= t) lo = mid;
      else hi = mid;
    }
    return lo;
  };
  const uint32_t i0 = __builtin_amdgcn_readfirstlane(search(T0));
  const uint32_t il = i0 + lane;
  const uint64_t r2 = il <= n ? R2(il) : ~0ull;  // nondecreasing over the lanes
  uint32_t k = 0;
#pragma unroll
  for (uint32_t step = 32; step > 0; step >>= 1) {
    const uint64_t v = ((uint64_t)(uint32_t)__shfl((int)(r2 >> 32), (int)(k + step) & 63, 64) << 32) |
                       (uint32_t)__shfl((int)(uint32_t)r2, (int)(k + step) & 63, 64);
    if (k + step < 64 && v <= T) k += step;
  }
  const uint64_t rn_sh = ((uint64_t)(uint32_t)__shfl((int)(r2 >> 32), (int)(k + 1) & 63, 64) << 32) |
                         (uint32_t)__shfl((int)(uint32_t)r2, (int)(k + 1) & 63, 64);
  if (T >= tiles) return;
  uint32_t i = i0 + k;
  uint64_t r0, r1;
  if (k < 63) {  // instance i0 + k and the next one are among the wave's 64
    r0 = ((uint64_t)(uint32_t)__shfl((int)(r2 >> 32), (int)k, 64) << 32) | (uint32_t)__shfl((int)(uint32_t)r2, (int)k, 64);
    r1 = rn_sh;
  } else {  // past them
    i = search(T);
    r0 = R2(i);
    r1 = R2(i + 1);
  }
  desc[T].v = make_uint4(i, (uint32_t)(T - r0) + 1, (uint32_t)((r1 - r0) / 2), (uint32_t)(r0 + i));
}

// The loads of one eval tile (see eval_hr_kernel): the tile's 11 cells of the lane's quad, the
// lane's limb-table entry (dense, spread) and its message-copy source. Named members, no array:
// a register array carried across the tile loop was kept in scratch by the compiler.
// (loaded non-temporally -- __builtin_nontemporal_load -- the pass ran 13 % slower: 11.00 vs
// 9.70 ms same process, profiles/r03v_ab_eval.txt)
__device__ __forceinline__ uint4 ev_ld(const uint32_t* p) { return *reinterpret_cast<const uint4*>(p); }
struct EvCells {
  uint4 c0, c1, c2, c3, c4, c5, c6, c7, c8, c9, c10;
  uint32_t d, sp, mc;
};
__device__ __forceinline__ EvCells ev_load(const hr2::HCtx& c, uint32_t lane, uint32_t lq, uint32_t mg, uint32_t mwh,
                                           uint32_t mk, const uint32_t* __restrict__ adv,
                                           const uint32_t* __restrict__ fixed, uint64_t total_rows, const uint8_t* Sg,
                                           bool gath) {
  EvCells v;
  const uint32_t* p = adv + c.row0 + 4 * lq;
  v.c0 = ev_ld(p);
  v.c1 = ev_ld(p + total_rows);
  v.c2 = ev_ld(p + 2 * total_rows);
  v.c3 = ev_ld(p + 3 * total_rows);
  v.c4 = ev_ld(p + 4 * total_rows);
  v.c5 = ev_ld(p + 5 * total_rows);
  v.c6 = ev_ld(p + 6 * total_rows);
  v.c7 = ev_ld(p + 7 * total_rows);
  v.c8 = ev_ld(p + 8 * total_rows);
  v.c9 = ev_ld(p + 9 * total_rows);
  v.c10 = ev_ld(fixed + c.row0 + 4 * lq);
  // the limb-table gather only when the previous half-round's tile is not the wave's previous tile
  // (otherwise a read of the tile's own first cells: lines this wave loads anyway, value unused)
#ifdef B2F_EV_NOGATHER  // diagnostics (verdict wrong): no limb-table or message gathers, to bound their traffic
  (void)gath;
  (void)Sg;
  (void)mg;
  (void)mwh;
  (void)mk;
  v.d = v.c0.x;
  v.sp = v.c1.y;
  v.mc = v.c2.z;
#else
  const Canon cs = canon_state(lane >> 2, c.hr);
  const uint64_t r = gath ? c.off + cs.row(lane & 3u) : c.row0 + 4 * lq;
  v.d = adv[(uint64_t)(gath ? cs.dcol : (uint32_t)A1) * total_rows + r];
  v.sp = adv[(uint64_t)(gath ? cs.scol : (uint32_t)A2) * total_rows + r];
  const uint32_t j = Sg[16 * ((c.hr >> 1) % 10) + 2 * (mg + 4 * (c.hr & 1u)) + mwh];
  v.mc = adv[(uint64_t)A1 * total_rows + c.off + 32 + 4 * j + mk];
#endif
  return v;
}

// The eval's edge tiles (one per instance: its init and final regions; then the zero rows as
// PAD_Q-quad tiles) dealt from tile t0 with stride W, in the wave's region S: the fast checks of
// the fused edge launch on the loaded trace. Returns whether any tile was flagged.
template <int MODE>
__device__ __forceinline__ bool eval_edge_walk(uint32_t* S, uint32_t lane, uint64_t t0, uint64_t W,
                                               const uint64_t* IV, const uint32_t* __restrict__ adv,
                                               const uint32_t* __restrict__ fixed, uint32_t n,
                                               const uint64_t* __restrict__ off, uint64_t total_rows) {
  using namespace hr2;
  using namespace edge2;
  const ELane E = make_elane(lane, lds_byte(S), IV);
  const uint64_t used_rows = off[n];
  const uint64_t n_pad = ((total_rows - used_rows) / 4 + PAD_Q - 1) / PAD_Q;
  const uint64_t t_all = (uint64_t)n + n_pad;
  bool bad = false;
  for (uint64_t t = t0; t < t_all; t += W) {
    if (t < n) {
      const uint32_t i = (uint32_t)t;
      const uint64_t o = off[i];
      const uint32_t rounds = (uint32_t)((off[i + 1] - o - FIXED_ROWS) / ROUND_ROWS);
      const uint64_t row_f = o + INIT_ROWS + (uint64_t)ROUND_ROWS * rounds;
      const uint64_t row = lane < NQ_I ? o + 4 * lane : lane < NQ ? row_f + 4 * (lane - NQ_I) : o;
      uint4 cv[NSTAGE];
#pragma unroll
      for (int col = 0; col < NSTAGE; col++)
        cv[col] = *reinterpret_cast<const uint4*>((col < 10 ? adv + (uint64_t)col * total_rows : fixed) + row);
      // limb table: the spread canonical cell of final state word lane / 4, limb lane % 4
      const Canon cs = canon_state(lane >> 2, 2 * rounds);
      const uint32_t sp = adv[(uint64_t)cs.scol * total_rows + o + cs.row(lane & 3u)];
      if (lane < NQ) {
#pragma unroll
        for (int col = 0; col < NSTAGE; col++) *reinterpret_cast<uint4*>(S + col * STR_E + 4 * lane) = cv[col];
      }
      S[E_LT + lane] = sp;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      bad |= edge_fast_checks<MODE>(E) != 0;
      asm volatile("" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    } else {  // the zero rows: valid lookups, no selector
      const uint64_t row0 = used_rows + (uint64_t)PAD_Q * 4 * (t - n);
      const uint64_t left = row0 < total_rows ? (total_rows - row0) >> 2 : 0;
      const uint32_t nq = (uint32_t)(left < PAD_Q ? left : PAD_Q);
      if (lane < nq) {
        const uint64_t r = row0 + 4ull * lane;
        const uint4 q0 = *reinterpret_cast<const uint4*>(adv + r), q1 = *reinterpret_cast<const uint4*>(adv + total_rows + r);
        const uint4 q2 = *reinterpret_cast<const uint4*>(adv + 2 * total_rows + r), fx = *reinterpret_cast<const uint4*>(fixed + r);
        uint32_t acc = fx.x | fx.y | fx.z | fx.w;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t de = comp(q1, j);
          acc |= (de & 0xffff0000u) | (tag_of(de) ^ comp(q0, j)) | (spread16(de) ^ comp(q2, j));
        }
        bad |= acc != 0;
      }
    }
  }
  return bad;
}

#ifndef B2F_EVAL_WAVES_HR
#define B2F_EVAL_WAVES_HR 3  // waves per SIMD of the eval fast pass (the prefetched tile's registers)
#endif
#ifndef B2F_EVAL_DYN
// 1 (variant): bands claimed from a counter -- 9.77 vs 9.64 ms (2^18 x 12), 5.26 vs 5.17 (mix),
// profiles/r06k_ab_dyn_*.txt: the load-bound pass balances itself
#define B2F_EVAL_DYN 0
#endif
#ifndef B2F_EVAL_HR_BAND
#define B2F_EVAL_HR_BAND 24  // consecutive half-round tiles per wave visit (1: one tile, every limb table gathered)
#endif
constexpr uint32_t EV_BAND = B2F_EVAL_HR_BAND;
// LDS byte addresses (dense | spread << 16) of limb k = lane % 4 of state word lane / 4 in the staged
// PREVIOUS half-round tile, for that tile's parity `par` (0: column G's, 1: diagonal G's): where the
// limb table of a tile comes from when the wave has just checked the instance's previous half-round
__device__ __forceinline__ uint32_t carry_addr(uint32_t lane, uint32_t Sb, uint32_t par) {
  const Canon cs = canon_state(lane >> 2, 1 + par);  // rows of half-round par of round 0
  const uint32_t ri = cs.row(lane & 3u) - INIT_ROWS - 208 * par;
  return (Sb + 4 * (cs.dcol * HSTR + ri)) | ((Sb + 4 * (cs.scol * HSTR + ri)) << 16);
}
template <int MODE>
__global__ void __launch_bounds__(FW * WAVES, B2F_EVAL_WAVES_HR)
eval_hr_kernel(const uint32_t* __restrict__ adv, const uint32_t* __restrict__ fixed, uint32_t n,
               const uint64_t* __restrict__ off, uint64_t total_rows, const TileDesc* __restrict__ desc,
               uint32_t* __restrict__ dirty, unsigned* __restrict__ bctr, const int* __restrict__ status) {
  using namespace hr2;
  __shared__ __attribute__((aligned(16))) uint32_t L[H_WORDS];
  const int tid = threadIdx.x;
  const uint32_t lane = (uint32_t)tid & 63u, wv = (uint32_t)tid >> 6;
  if (tid < 40) L[H_SG + tid] = reinterpret_cast<const uint32_t*>(c_sigma)[tid];
  if (tid < 16) L[H_IV + tid] = reinterpret_cast<const uint32_t*>(c_iv)[tid];
  __syncthreads();
  if (*status) return;  // a rejected row map: the eval kernel reports it
  const uint8_t* Sg = reinterpret_cast<const uint8_t*>(L + H_SG);
  uint32_t* S = L + H_WAVE + wv * HW_WORDS + HPRE;
  const Lane K = make_lane(lane, lds_byte(S));
  const bool qlane = lane < HR_Q;
  const uint32_t lq = qlane ? lane : 0;
  const uint32_t m32 = lane & 31u, mg = m32 >> 3, mwh = (m32 >> 2) & 1u, mk = m32 & 3u;
  const uint64_t used_rows = off[n];
  const uint64_t n_hr = (used_rows - (uint64_t)FIXED_ROWS * n) / 208;
  const uint64_t W = (uint64_t)gridDim.x * WAVES;
#if B2F_EVAL_DYN
  // (variant) bands of EV_BAND consecutive tiles per wave visit, claimed from the launch's counter
  // (one band ahead, when the band's last tile prefetches the next one's first)
  auto claim = [&]() -> uint64_t {
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(bctr, 1u);
    return __builtin_amdgcn_readfirstlane(v);
  };
  uint64_t b = claim();
#else
  (void)bctr;
  // bands of EV_BAND consecutive tiles per wave visit, dealt like single tiles (first_tile)
  uint64_t b = first_tile(blockIdx.x, __builtin_amdgcn_readfirstlane(wv), gridDim.x);
#endif
  uint64_t t = b * EV_BAND;
  uint32_t j = 0;
  const uint32_t cA0 = carry_addr(lane, lds_byte(S), 0), cA1 = carry_addr(lane, lds_byte(S), 1);
  auto raw_desc = [&](uint64_t tt) -> uint4 { return desc[tt].v; };
  // per tile: its cells (lane = quad), its limb-table entry (the canonical dense / spread cell of
  // state word lane / 4, limb lane % 4, as the half-round starts: gathered at a band's first tile
  // and at an instance's first half-round, otherwise read from the previous tile's staging) and its
  // message-copy source (message word SIGMA[..] limb, a_1 of its INW block), loaded one tile ahead
  HCtx c = hctx(raw_desc(t < n_hr ? t : 0));
  EvCells cur = ev_load(c, lane, lq, mg, mwh, mk, adv, fixed, total_rows, Sg, true);
  while (t < n_hr) {
    uint64_t tn = t + 1, bn = b;
    uint32_t jn = j + 1;
    if (jn == EV_BAND || tn >= n_hr) {
#if B2F_EVAL_DYN
      bn = claim();
#else
      bn = b + W;
#endif
      tn = bn * EV_BAND;
      jn = 0;
    }
    const HCtx cn = hctx(raw_desc(tn < n_hr ? tn : 0));
    const EvCells nxt = ev_load(cn, lane, lq, mg, mwh, mk, adv, fixed, total_rows, Sg, jn == 0 || cn.hr == 0);
    uint32_t ltd = cur.d, lts = cur.sp;
    if (j != 0 && c.hr != 0) {  // the staging holds half-round hr - 1 of this instance
      const uint32_t a = ((c.hr - 1) & 1u) ? cA1 : cA0;
      ltd = ld32(a & 0xffffu);
      lts = ld32(a >> 16);
    }
    asm volatile("" ::: "memory");  // read before the tile's cells overwrite the staging
    if (qlane) {
      uint4* q = reinterpret_cast<uint4*>(S + 4 * lane);
      q[0 * HSTR / 4] = cur.c0;
      q[1 * HSTR / 4] = cur.c1;
      q[2 * HSTR / 4] = cur.c2;
      q[3 * HSTR / 4] = cur.c3;
      q[4 * HSTR / 4] = cur.c4;
      q[5 * HSTR / 4] = cur.c5;
      q[6 * HSTR / 4] = cur.c6;
      q[7 * HSTR / 4] = cur.c7;
      q[8 * HSTR / 4] = cur.c8;
      q[9 * HSTR / 4] = cur.c9;
      q[10 * HSTR / 4] = cur.c10;
    }
    S[H_LT + lane] = ltd;
    S[H_LT + 64 + lane] = lts;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const uint32_t mc = cur.mc;
    const uint32_t acc = hr_fast_checks<MODE>(K, c.hr, [&] { return mc; });
    if (__builtin_amdgcn_ballot_w64(acc != 0) && lane == 0) *dirty = 1u;
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    c = cn;
    cur = nxt;
    t = tn;
    j = jn;
    b = bn;
  }
  // then the edge tiles, in the wave's whole region (as the fused launch
  // does since round 4, the edge work fills this launch's tail instead of a launch after it)
  if (!B2F_EDGE_SEPARATE) {
    const uint64_t* IV = reinterpret_cast<const uint64_t*>(L + H_IV);
    const bool bad = eval_edge_walk<MODE>(L + H_WAVE + wv * HW_WORDS, lane,
                                          first_tile(blockIdx.x, __builtin_amdgcn_readfirstlane(wv), gridDim.x),
                                          W, IV, adv, fixed, n, off, total_rows);
    if (__builtin_amdgcn_ballot_w64(bad) && lane == 0) *dirty = 1u;
  }
}

// The edge walk as its own launch after the half-round pass (diagnostics: B2F_EDGE_SEPARATE = 1
// builds this form; the product runs the walk as eval_hr_kernel's last phase)
template <int MODE>
__global__ void __launch_bounds__(FW * WAVES, 3)
eval_edge_kernel(const uint32_t* __restrict__ adv, const uint32_t* __restrict__ fixed, uint32_t n,
                 const uint64_t* __restrict__ off, uint64_t total_rows, uint32_t* __restrict__ dirty,
                 const int* __restrict__ status) {
  using namespace hr2;
  using namespace edge2;
  __shared__ __attribute__((aligned(16))) uint32_t L[E_WORDS];
  const int tid = threadIdx.x;
  const uint32_t lane = (uint32_t)tid & 63u, wv = (uint32_t)tid >> 6;
  if (tid < 16) L[E_IV + tid] = reinterpret_cast<const uint32_t*>(c_iv)[tid];
  __syncthreads();
  if (*status) return;
  const uint64_t* IV = reinterpret_cast<const uint64_t*>(L + E_IV);
  const bool bad = eval_edge_walk<MODE>(L + E_WAVE + wv * EW_WORDS, lane,
                                        first_tile(blockIdx.x, __builtin_amdgcn_readfirstlane(wv), gridDim.x),
                                        (uint64_t)gridDim.x * WAVES, IV, adv, fixed, n, off, total_rows);
  if (__builtin_amdgcn_ballot_w64(bad) && lane == 0) *dirty = 1u;
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
// + the edge launch's redo list (count + one slot per instance; tiles >= instances)
size_t fused_scratch_bytes(uint64_t tiles) {
  // + the eval's band counter and dirty word
  return tiles * sizeof(TileDesc) + 8 * (1 + DEFER_CAP) + 4 * (2 + tiles) + 16;
}

// The eval's fast clean-check pass (see eval_hr_kernel) into the fused scratch; returns the
// device word the exact eval kernel is gated on (0: clean, the report stands).
hipError_t launch_eval_fast(const uint32_t* d_adv, const uint32_t* d_fixed, const uint64_t* d_off, uint32_t n,
                            uint64_t total_rows, void* scratch, uint64_t tiles, const int* d_status,
                            int cu_count, hipStream_t s, const uint32_t** gate, int mode) {
#ifndef B2F_DIAG
  mode = FZ_FULL;  // the product library runs the full pass only
#endif
  TileDesc* desc = reinterpret_cast<TileDesc*>(scratch);
  uint32_t* dirty = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(scratch) + fused_scratch_bytes(tiles) - 8);
  unsigned* bctr = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(scratch) + fused_scratch_bytes(tiles) - 16);
  hipError_t e = hipMemsetAsync(bctr, 0, 16, s);  // the band counter and the dirty word
  if (e != hipSuccess) return e;
  // tiles (an upper bound on the half-round tiles) >= 2 sum(rounds): every tile has its thread
  hipLaunchKernelGGL(eval_desc_kernel, dim3((uint32_t)((tiles + 255) / 256)), dim3(256), 0, s, d_off, n, desc, d_status);
  static int per_cu[2] = {0, 0};
  if (!per_cu[0]) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, eval_hr_kernel<FZ_FULL>, FW * WAVES, 0) != hipSuccess || nb < 1) nb = 2;
    per_cu[0] = nb;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, eval_edge_kernel<FZ_FULL>, FW * WAVES, 0) != hipSuccess || nb < 1) nb = 2;
    per_cu[1] = nb;
  }
  const uint64_t edge_tiles = (uint64_t)n + ((total_rows / 4) + PAD_Q - 1) / PAD_Q;
  const uint64_t edge_wgs = (edge_tiles + WAVES - 1) / WAVES;
  const uint32_t grid_e = (uint32_t)(edge_wgs < (uint64_t)cu_count * per_cu[1] ? edge_wgs : (uint64_t)cu_count * per_cu[1]);
  // 2 workgroups per CU (the fused half-round launch runs 3): for this load-bound pass a
  // narrower front of tiles in flight reads faster than every workgroup that fits
  // (same-process A/B 9.77 vs 9.87 ms)
  int ev_per_cu = per_cu[0] < 2 ? per_cu[0] : 2;
#ifdef B2F_DIAG  // diagnostics: workgroups per CU of the half-round pass
  if (const char* v = getenv("B2F_EVAL_PERCU")) {
    const int k = atoi(v);
    if (k >= 1 && k <= per_cu[0]) ev_per_cu = k;
  }
#endif
  switch (mode) {
#define B2F_EVFAST(M)                                                                              \
  case M:                                                                                          \
    hipLaunchKernelGGL(eval_hr_kernel<M>, dim3(cu_count * ev_per_cu), dim3(FW * WAVES), 0, s, d_adv, d_fixed, n, \
                       d_off, total_rows, desc, dirty, bctr, d_status);                            \
    if (B2F_EDGE_SEPARATE)                                                                         \
      hipLaunchKernelGGL(eval_edge_kernel<M>, dim3(grid_e), dim3(FW * WAVES), 0, s, d_adv, d_fixed, n, d_off, \
                         total_rows, dirty, d_status);                                             \
    break;
#ifdef B2F_DIAG
    B2F_EVFAST(0) B2F_EVFAST(1) B2F_EVFAST(8) B2F_EVFAST(16)
#endif
    default: B2F_EVFAST(FZ_FULL)
#undef B2F_EVFAST
  }
  *gate = dirty;
  return hipGetLastError();
}
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
                            unsigned long long* clk, const uint64_t* seg, uint64_t seg_cap,
                            hipStream_t s) {
  TileDesc* desc = reinterpret_cast<TileDesc*>(scratch);
  uint64_t* defer = reinterpret_cast<uint64_t*>(desc + tiles);
  uint32_t* redo = reinterpret_cast<uint32_t*>(defer + 1 + DEFER_CAP);
  // the half-round launch's instance and edge-tile counters: the first two words of the
  // tile-descriptor area (only the eval's fast pass uses descriptors)
  unsigned* ictr = reinterpret_cast<unsigned*>(desc);
  hipError_t e = hipMemsetAsync(defer, 0, 8, s);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(ictr, 0, 8, s);  // the instance and the edge-tile counters
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(redo, 0, 4, s);
  if (e != hipSuccess) return e;
  Inject inj;
  inj.row = inj_row;
  inj.col = inj_col;
  inj.mask = inj_mask;
#ifndef B2F_DIAG
  mode = FZ_FULL;  // the product library launches the full kernel only
#endif
  if (inj_row != ~0ull) mode |= FZ_INJECT;
  // persistent grid: the workgroups that are resident at once (VGPRs and LDS bound them)
  static int per_cu[2] = {0, 0};
  if (!per_cu[0]) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fused_hr_kernel<FZ_FULL>, FW * WAVES, 0) !=
            hipSuccess || nb < 1)
      nb = 2;
    per_cu[0] = nb;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fused_edge_kernel<FZ_FULL>, FW * WAVES, 0) !=
            hipSuccess || nb < 1)
      nb = 2;
    per_cu[1] = nb;
  }
  // the edge tiles (one per instance) plus the zero rows; no more workgroups than they fill
  // (the zero-row count here is an upper bound)
  const uint64_t edge_tiles = (uint64_t)n + ((total_rows / 4) + PAD_Q - 1) / PAD_Q;
  const uint64_t edge_wgs = (edge_tiles + WAVES - 1) / WAVES;
  // Fewer half-round workgroups than fit: 3 per CU (12 waves) write the trace faster than 2 or 4
  // per CU (same-process A/B 11.48 vs 12.89 / 12.91 ms, profiles/r03o_ab_percu.txt): enough
  // waves to overlap one tile's stores with another's compute, a narrow front of tiles in flight
  int hr_per_cu = per_cu[0] < B2F_FUSED_HR_PER_CU ? per_cu[0] : B2F_FUSED_HR_PER_CU;
#ifdef B2F_DIAG  // diagnostics: workgroups per CU of the half-round launch
  if (const char* v = getenv("B2F_FUSED_PERCU")) {
    const int k = atoi(v);
    if (k >= 1 && k <= per_cu[0]) hr_per_cu = k;
  }
#endif
  const uint32_t grid = (uint32_t)(cu_count * hr_per_cu);
  int e_per_cu = per_cu[1];
#ifdef B2F_DIAG  // diagnostics: workgroups per CU of the edge launch
  if (const char* v = getenv("B2F_EDGE_PERCU")) {
    const int k = atoi(v);
    if (k >= 1 && k <= per_cu[1]) e_per_cu = k;
  }
#endif
  const uint32_t grid_e = (uint32_t)(edge_wgs < (uint64_t)cu_count * e_per_cu ? edge_wgs : (uint64_t)cu_count * e_per_cu);
  switch (mode) {
#define B2F_FUSED(M)                                                                               \
  case M:                                                                                          \
    hipLaunchKernelGGL(fused_hr_kernel<M>, dim3(grid), dim3(FW * WAVES), 0, s, d_in, n, d_off,     \
                       total_rows, rec, d_adv, d_fixed, ictr, d_rep, d_status, inj, defer, DEFER_CAP, \
                       clk, seg, seg_cap, redo);                                                   \
    if (B2F_EDGE_SEPARATE)                                                                         \
      hipLaunchKernelGGL(fused_edge_kernel<M>, dim3(grid_e), dim3(FW * WAVES), 0, s, d_in, n, d_off, \
                         total_rows, rec, d_adv, d_fixed, redo, d_rep, d_status, inj, defer,       \
                         DEFER_CAP, clk);                                                          \
    hipLaunchKernelGGL(edge_redo_kernel<M>, dim3(cu_count), dim3(FW * WAVES), 0, s, d_in, d_off,   \
                       total_rows, rec, d_adv, d_fixed, redo, d_rep, d_status, inj, defer,         \
                       DEFER_CAP);                                                                 \
    break;
#ifdef B2F_DIAG
    B2F_FUSED(0) B2F_FUSED(2) B2F_FUSED(3) B2F_FUSED(10) B2F_FUSED(18) B2F_FUSED(8) B2F_FUSED(16)
    B2F_FUSED(FZ_FULL | FZ_CLOCK) B2F_FUSED(2 | FZ_CLOCK) B2F_FUSED(0 | FZ_CLOCK)
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

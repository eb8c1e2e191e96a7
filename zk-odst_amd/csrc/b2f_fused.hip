// b2f_fused.hip -- the fused witness fill + constraint evaluation (b2f_fill_eval_dev).
//
// One persistent kernel assigns every cell of a batch (the fill_kernel's work) and checks the
// trace it assigns (the eval_kernel's work) before the cells leave the CU: each cell is written
// to HBM once and never read back. The result is the same trace, h' and verdict as
// b2f_fill_dev followed by b2f_eval_dev -- MockProver::run (synthesize, blake2f.rs:301) then
// verify (:302) over the same assignment -- at the HBM cost of the fill alone.
//
// Work layout
//   * Workgroups walk bands of `band` consecutive 1024-row tiles (band k -> workgroup
//     k mod grid). Thread = quad: it builds its 4 rows x 11 columns in registers from operand
//     words prefetched during the previous tile (half-round states, message words, init
//     words), stores them (16-byte non-temporal column stores, 1 KiB per wave per column) and
//     stages them into LDS.
//   * The checks lag the cells by 16 rows: LDS coordinate u = row - (tile0 - 16), computed
//     rows sit at u in [16, 1040), u in [0, 16) are the previous tile's last four quads,
//     carried in LDS. Every gate is evaluated in the tile that holds the last row it reads
//     (blocks are <= 12 rows), so no tile ever needs rows of the next one; lookups and copy
//     constraints (sources always precede their operand cells) are checked in the tile that
//     holds their row.
//   * The 384-row history window of the four canonical columns (every copy source) is the
//     previous tile's tail, moved in LDS by the threads that overwrite it; only the first tile
//     of a band recomputes it (100 extra quads). The init-region cache of the tile's first
//     instance is recomputed when that instance changes.
//   * The gate / copy machinery is the eval kernel's (G table one tile ahead, canonical round
//     blocks by kind per wave, 72 copy checks per G spread over the workgroup, per-quad paths
//     for init/final blocks and non-canonical selector rows), on the shifted coordinates.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "../../include/b2f.h"
#include "b2f_common.h"

namespace {

constexpr int SHIFT = 16;                         // check rows lag computed rows by 4 quads
constexpr int NQ = BLOCK + SHIFT / 4;             // 260 quads of u coordinates
constexpr int F_HALO = 16;                        // zero rows past u = 1040 (last tile only)
constexpr int F_TS = SHIFT + TILE_ROWS + F_HALO;  // 1056
constexpr int F_WS = HIST + F_TS;                 // 1440
constexpr int U_END = SHIFT + TILE_ROWS;          // 1040
constexpr int F_MAX_G = 24;                       // G starts in [tile0 - 51, tile0 + 1023]: <= 21
constexpr int F_GT_WORDS = 8;
constexpr int FS_GT = 0, FS_QM = F_MAX_G * F_GT_WORDS, FS_NG = FS_QM + (NQ + 3) / 4;
constexpr int FSET = (FS_NG + 1 + 3) & ~3;
constexpr int HIST_QUADS = (HIST + SHIFT) / 4;    // 100 quads recomputed at a band start

// LDS carve (words)
//   W     a_1 a_2 a_7 a_8 for u in [-384, 1056)      G     a_0 a_3 a_4 a_5 a_6, u in [0, 1056)
//   CT    copy-check table   SG SIGMA   IV   INFO three TileInfo   IC init cache
//   XS    canonical row-0 selectors per G quad   QSEL/A9 per u-quad row-0 selector word / a_9
//   CAR   fixed words and a_9 of the carried quads u 0..15 (their deferred gates)
//   GS    two G sets (this tile / next)   ACC counters
constexpr int F_W = 0;
constexpr int F_G = F_W + 4 * F_WS;
constexpr int F_CT = F_G + 5 * F_TS;
constexpr int F_SG = F_CT + 12 * G_CHECKS;
constexpr int F_IV = F_SG + 40;    // IV, 8 x u64
constexpr int F_INFO = F_IV + 16;  // three TileInfo (tiles i, i + 1, i + 2 of the sequence)
constexpr int F_IC = F_INFO + 72;
constexpr int F_XS = F_IC + 2 * INIT_ROWS;
constexpr int F_QSEL = F_XS + 16;
constexpr int F_A9 = F_QSEL + NQ;
constexpr int F_CAR = F_A9 + NQ;
constexpr int F_GS = F_CAR + 32;
constexpr int F_ACC = F_GS + 2 * FSET;
constexpr int F_WORDS = F_ACC + 22;
static_assert(F_INFO % 4 == 0 && F_IV % 2 == 0 && F_IC % 4 == 0 && (F_IC + INIT_ROWS) % 4 == 0 && F_G % 4 == 0 &&
              F_CAR % 4 == 0 && F_GS % 4 == 0 && F_ACC % 2 == 0 && F_WS % 4 == 0 && F_TS % 4 == 0,
              "aligned carve");
static_assert((F_WORDS + ROW_TABLE_WORDS) * 4 * 3 <= 160 * 1024, "three fused workgroups per CU");
static_assert(check_table_ok<F_W, F_WS>(), "72 copy checks per G, fields in range");
static_assert(F_GT_WORDS == GT_WORDS_ && F_MAX_G * LPG <= BLOCK, "G table layout / copy lanes");

__constant__ __attribute__((aligned(16))) CheckTable c_fchecks = make_check_table<F_W, F_WS>();
using FTile = TileT<F_W, F_WS, F_G, F_TS>;

// Rows read by each gate past its selector row, minus one (LAYOUT.md §4 identities):
// abcd 4, efgh 11, ijkl 7, a1 4, b1 12, c1 4, d1 8, a2 4, b2 8, c2 4, d2 8, digest 7, xor 8,
// xor3 8, const 1, fmask 4.
constexpr uint64_t gate_span() {
  const uint32_t rows[16] = {4, 11, 7, 4, 12, 4, 8, 4, 8, 4, 8, 7, 8, 8, 1, 4};
  uint64_t s = 0;
  for (int i = 0; i < 16; i++) s |= (uint64_t)(rows[i] - 1) << (4 * i);
  return s;
}
constexpr uint64_t kGateSpan = gate_span();

// Selector bits of row r (u coordinates) whose gate's last row lies in [lo, hi).
__device__ __forceinline__ uint32_t gates_ending_in(uint32_t sel, int r, int lo, int hi) {
  uint32_t keep = 0;
  for (uint32_t m = sel; m; m &= m - 1) {
    const int s = __builtin_ctz(m);
    const int last = r + (int)((kGateSpan >> (4 * s)) & 15u);
    if (last >= lo && last < hi) keep |= 1u << s;
  }
  return keep;
}

// Test-only fault injection (b2f_debug_inject): XOR `mask` into one cell as it is assigned,
// so the trace written and the trace checked are the corrupted one.
struct Inject {
  uint64_t quad;  // global quad index, ~0: none
  uint32_t j;     // row inside the quad
  uint32_t col;   // 0..9 advice a_col, 10 fixed
  uint32_t mask;
};

template <bool INJ>
__device__ __forceinline__ void build_quad(Quad& Q, const QuadOps& P, uint64_t gq,
                                           const uint32_t* rows, const uint64_t* IV,
                                           const Inject& inj) {
  zero(Q);
  if (P.rounds != ~0u) {
    const uint32_t rq = P.lq - INIT_QUADS;
    if (P.lq >= INIT_QUADS && rq < ROUND_QUADS * P.rounds) {
      const uint32_t p = (rq % ROUND_QUADS) % G_QUADS;
      quad_round(Q, P.w[0], P.w[1], P.w[2], P.w[3], P.w[4], P.w[5], p, rows);
    } else {
      quad_cells_ops(Q, P, IV);
    }
  }
  if (INJ && gq == inj.quad) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
#pragma unroll
      for (int c = 0; c < 10; c++)
        if (c == (int)inj.col && j == (int)inj.j) Q.c[c][j] ^= inj.mask;
      if (inj.col == 10 && j == (int)inj.j) Q.fx[j] ^= inj.mask;
    }
  }
}

constexpr GTCarve kFusedGT{FS_QM, FS_NG, FS_GT, F_IC, F_W, F_WS, (NQ + 3) / 4, NQ, SHIFT, F_MAX_G};

// Per-quad gates of a selector quad the G pass does not take (init/final blocks, any
// non-canonical selector row): the gates of rows r0..r0+3 whose last row is in [lo, hi).
__device__ __forceinline__ void quad_gates_f(const FTile& T, EvalAcc& A, const uint4& fx,
                                             const uint4& a9, int r0, int lo, int hi,
                                             int64_t base0) {
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint32_t k0 = comp(fx, j);
    const uint32_t sel = gates_ending_in(k0 & 0xffffu, r0 + j, lo, hi);
    if (!sel) continue;
    uint32_t failed;
    if (sel == (1u << S_CONST)) failed = T.at(A1, r0 + j) == (k0 >> 16) ? 0u : sel;
    else failed = row_gates(T, sel, (uint32_t)(r0 + j), comp(a9, j), k0);
    if (failed) A.fail_gates((uint64_t)(base0 + r0 + j), failed);
  }
}

// A quad's gates go to the G pass iff it is a round quad with exactly the canonical selectors.
__device__ __forceinline__ bool canonical_quad(const uint32_t* L, const uint32_t* S, int uq,
                                               const uint4& fx) {
  const uint32_t pq = reinterpret_cast<const uint8_t*>(S + FS_QM)[uq];
  const uint32_t rest = (fx.y | fx.z | fx.w) & 0xffffu;
  return pq != 0xffu && rest == 0 && (fx.x & 0xffffu) == L[F_XS + (pq & 15u)];
}

__device__ __forceinline__ uint4 lds4(const uint32_t* L, int w) {
  return *reinterpret_cast<const uint4*>(L + w);
}
__device__ __forceinline__ void sts4(uint32_t* L, int w, const uint4& v) {
  *reinterpret_cast<uint4*>(L + w) = v;
}

#ifndef B2F_FUSED_WAVES
#define B2F_FUSED_WAVES 3  // waves per SIMD (LDS allows 3 workgroups per CU)
#endif

// MODE: FZ_LOOKUP / FZ_GATES / FZ_COPIES which checks run, FZ_STORE write the trace to HBM,
// FZ_INJECT the test-only fault injection. Product launches: FZ_FULL (diagnostic
// variants via B2F_DIAG_FUSED).
enum { FZ_LOOKUP = 1, FZ_STORE = 2, FZ_INJECT = 4, FZ_GATES = 8, FZ_COPIES = 16, FZ_FULL = 27,
       FZ_NOSTAGE = 32, FZ_NOGT = 64,  // 32, 64: assignment-only diagnostics (no checks)
       FZ_CLOCK = 128 };  // per-phase s_memtime totals per wave (diagnostics, b2f_debug_clock)

template <int MODE>
__global__ void __launch_bounds__(BLOCK, B2F_FUSED_WAVES)
fused_kernel(const b2f_input* __restrict__ in, uint32_t n, const uint64_t* __restrict__ off,
             uint64_t total_rows, const uint64_t* __restrict__ rec, uint32_t* __restrict__ adv,
             uint32_t* __restrict__ fixed, const TileInfo* __restrict__ tinfo, uint64_t n_tiles,
             uint32_t band, b2f_eval_report* __restrict__ rep, const int* __restrict__ status,
             Inject inj, unsigned long long* __restrict__ clk) {
  __shared__ __attribute__((aligned(16))) uint32_t L[F_WORDS];
  uint64_t ck[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tp = 0;
  auto tick = [&](int k) {
    if (MODE & FZ_CLOCK) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      if (k >= 0) ck[k] += now - tp;
      tp = now;
    }
  };
  __shared__ uint32_t rows[ROW_TABLE_WORDS];
  const int tid = threadIdx.x;
  if (*status) return;  // the record kernel rejected the layout: write nothing
  for (int i = tid; i < 12 * G_CHECKS; i += BLOCK)
    L[F_CT + i] = reinterpret_cast<const uint32_t*>(&c_fchecks)[i];
  if (tid < 40) L[F_SG + tid] = reinterpret_cast<const uint32_t*>(c_sigma)[tid];
  if (tid < 16) L[F_IV + tid] = reinterpret_cast<const uint32_t*>(c_iv)[tid];
  if (tid < 16) L[F_XS + tid] = expected_sel((uint32_t)tid);
  if (tid < ROW_TABLE_WORDS) rows[tid] = (&c_rows.r[0][0])[tid];
  if (tid < 20) L[F_ACC + tid] = 0;
  if (tid == 20) *reinterpret_cast<uint64_t*>(L + F_ACC + 20) = ~0ull;
  if (tid < 32) L[F_CAR + tid] = 0;
  if (tid < 36) {  // zero halo rows u in [1040, 1056) of the 9 staged columns (never written)
    const int c = tid / 4, q = tid & 3;
    const int w = c < 4 ? F_W + c * F_WS + HIST + U_END + 4 * q : F_G + (c - 4) * F_TS + U_END + 4 * q;
    sts4(L, w, make_uint4(0, 0, 0, 0));
  }
  const FTile T{L};
  const uint8_t* Sg = reinterpret_cast<const uint8_t*>(L + F_SG);
  const uint64_t* IV = reinterpret_cast<const uint64_t*>(L + F_IV);
  EvalAcc A{L + F_ACC};

  const uint64_t total_quads = total_rows >> 2;
  const uint64_t used_rows = off[n];
  const uint64_t G = gridDim.x, B = band;
  auto seq = [&](uint64_t i) -> uint64_t { return (blockIdx.x + (i / B) * G) * B + (i % B); };
  auto info_of = [&](uint64_t i) -> const uint32_t* { return L + F_INFO + 24 * (uint32_t)(i % 3); };

  // Software pipeline, one tile deep: at the top of iteration i every global load for tile
  // i + 1 is issued (its quads' operand words, its first instance's init words) before tile
  // i's stores, and TileInfo runs two tiles ahead (three LDS slots).
  uint64_t t = seq(0);
  QuadOps P;              // operands of this tile's quad
  uint64_t icw = 0;       // init word `tid` of this tile's first instance (lanes < 41)
  uint4 ti = make_uint4(0, 0, 0, 0);  // TileInfo two tiles ahead (lanes 0..5)
  if (t < n_tiles && tid < 6) {
    sts4(L, F_INFO + tid * 4, reinterpret_cast<const uint4*>(tinfo + t)[tid]);
    const uint64_t t1 = seq(1), t2 = seq(2);
    if (t1 < n_tiles) sts4(L, F_INFO + 24 + tid * 4, reinterpret_cast<const uint4*>(tinfo + t1)[tid]);
    if (t2 < n_tiles) ti = reinterpret_cast<const uint4*>(tinfo + t2)[tid];
  }
  __syncthreads();
  if (t < n_tiles) {
    const uint32_t* info = info_of(0);
    const uint64_t* Off = reinterpret_cast<const uint64_t*>(info + 2);
    quad_ops(P, 4 * (t * BLOCK + tid), info[0], Off, n, used_rows, in, rec, Sg);
    if (tid < (int)INIT_QUADS && info[0] < n) icw = init_word(in + info[0], tid);
    if (tid < 64)
      build_g_table(L + F_GS, info, Sg, (int64_t)(t * TILE_ROWS) - SHIFT, n, total_rows, tid, kFusedGT);
  }
  bool ic_now = true;  // the first tile of a band always (re)builds the init cache
  for (uint64_t i = 0; t < n_tiles; i++, t = seq(i)) {
    const uint64_t tn = seq(i + 1);
    const bool has_next = tn < n_tiles;
    const bool band_start = (i % B) == 0;
    const bool last_tile = t + 1 == n_tiles;
    const uint32_t cur = (uint32_t)(i & 1), nxt = cur ^ 1u;
    const int64_t base0 = (int64_t)(t * TILE_ROWS) - SHIFT;
    const uint64_t gq = t * BLOCK + tid;
    const uint64_t row0 = 4 * gq;
    const int u0 = SHIFT + 4 * tid;  // this thread's rows in u coordinates
    const uint32_t* info = info_of(i);
    const uint32_t* ninfo = info_of(i + 1);
    const uint32_t first = info[0];

    tick(-1);
    // ---- A0. loads for tile i + 1
    QuadOps Pn;
    uint64_t icw_n = 0;
    bool ic_next = false;
    if (has_next) {
      const uint64_t* nOff = reinterpret_cast<const uint64_t*>(ninfo + 2);
      quad_ops(Pn, 4 * (tn * BLOCK + tid), ninfo[0], nOff, n, used_rows, in, rec, Sg);
      ic_next = ((i + 1) % B) == 0 || ninfo[0] != first;
      if (ic_next && tid < (int)INIT_QUADS && ninfo[0] < n) icw_n = init_word(in + ninfo[0], tid);
    }

    tick(0);
    // ---- A1. first tile of a band: recompute rows [tile0 - 400, tile0) (history window and
    // the carried quads) from the previous tile's instance context
    if (band_start && tid < HIST_QUADS) {
      QuadOps H;
      H.rounds = ~0u;
      H.lq = 0;
#pragma unroll
      for (int k = 0; k < 6; k++) H.w[k] = 0;
      const int64_t hrow = base0 - HIST + 4 * tid;
      if (hrow >= 0 && t > 0) {
        const TileInfo* tp = tinfo + (t - 1);
        quad_ops(H, (uint64_t)hrow, tp->first, tp->off, n, used_rows, in, rec, Sg);
      }
      Quad Qh;
      build_quad<(MODE & FZ_INJECT) != 0>(Qh, H, hrow >= 0 ? (uint64_t)hrow / 4 : ~0ull, rows, IV, inj);
      sts4(L, F_W + 0 * F_WS + 4 * tid, make_uint4(Qh.c[A1][0], Qh.c[A1][1], Qh.c[A1][2], Qh.c[A1][3]));
      sts4(L, F_W + 1 * F_WS + 4 * tid, make_uint4(Qh.c[A2][0], Qh.c[A2][1], Qh.c[A2][2], Qh.c[A2][3]));
      sts4(L, F_W + 2 * F_WS + 4 * tid, make_uint4(Qh.c[A7][0], Qh.c[A7][1], Qh.c[A7][2], Qh.c[A7][3]));
      sts4(L, F_W + 3 * F_WS + 4 * tid, make_uint4(Qh.c[A8][0], Qh.c[A8][1], Qh.c[A8][2], Qh.c[A8][3]));
      if (tid >= HIST / 4) {  // u in [0, 16): the carried quads
        const int uc = 4 * (tid - HIST / 4);
        sts4(L, F_G + 0 * F_TS + uc, make_uint4(Qh.c[A0][0], Qh.c[A0][1], Qh.c[A0][2], Qh.c[A0][3]));
        sts4(L, F_G + 1 * F_TS + uc, make_uint4(Qh.c[A3][0], Qh.c[A3][1], Qh.c[A3][2], Qh.c[A3][3]));
        sts4(L, F_G + 2 * F_TS + uc, make_uint4(Qh.c[A4][0], Qh.c[A4][1], Qh.c[A4][2], Qh.c[A4][3]));
        sts4(L, F_G + 3 * F_TS + uc, make_uint4(Qh.c[A5][0], Qh.c[A5][1], Qh.c[A5][2], Qh.c[A5][3]));
        sts4(L, F_G + 4 * F_TS + uc, make_uint4(Qh.c[A6][0], Qh.c[A6][1], Qh.c[A6][2], Qh.c[A6][3]));
        const uint32_t rest = (Qh.fx[1] | Qh.fx[2] | Qh.fx[3]) & 0xffffu;
        L[F_QSEL + tid - HIST / 4] = (Qh.fx[0] & 0xffffu) | (rest ? 1u << 16 : 0u);
        L[F_A9 + tid - HIST / 4] = Qh.c[A9][0];
        sts4(L, F_CAR + uc, make_uint4(Qh.fx[0], Qh.fx[1], Qh.fx[2], Qh.fx[3]));
        sts4(L, F_CAR + 16 + uc, make_uint4(Qh.c[A9][0], Qh.c[A9][1], Qh.c[A9][2], Qh.c[A9][3]));
      }
    }

    // ---- A2. init-region cache (a_1 | a_2 of rows 0..163) of the tile's first instance
    if (ic_now && first < n && tid < (int)INIT_QUADS) {
      const uint64_t o = reinterpret_cast<const uint64_t*>(info + 2)[0];
      QuadOps Pi;
      Pi.w[0] = icw;
#pragma unroll
      for (int k = 1; k < 6; k++) Pi.w[k] = 0;
      Pi.lq = (uint32_t)tid;
      Pi.rounds = 0;  // init quads decode the same for any rounds
      Quad Qi;
      zero(Qi);
      quad_cells_ops(Qi, Pi, IV);
      if ((MODE & FZ_INJECT) && o / 4 + tid == inj.quad) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          if (inj.col == A1 && j == (int)inj.j) Qi.c[A1][j] ^= inj.mask;
          if (inj.col == A2 && j == (int)inj.j) Qi.c[A2][j] ^= inj.mask;
        }
      }
      sts4(L, F_IC + 4 * tid, make_uint4(Qi.c[A1][0], Qi.c[A1][1], Qi.c[A1][2], Qi.c[A1][3]));
      sts4(L, F_IC + INIT_ROWS + 4 * tid, make_uint4(Qi.c[A2][0], Qi.c[A2][1], Qi.c[A2][2], Qi.c[A2][3]));
    }

    tick(1);
    // ---- A3. assign the quad, check its lookups, stage it, store it
    Quad Q;
    build_quad<(MODE & FZ_INJECT) != 0>(Q, P, gq, rows, IV, inj);
    const uint32_t own_lq = P.lq, own_rounds = P.rounds;
    const uint4 fx = make_uint4(Q.fx[0], Q.fx[1], Q.fx[2], Q.fx[3]);
    const uint4 a9 = make_uint4(Q.c[A9][0], Q.c[A9][1], Q.c[A9][2], Q.c[A9][3]);
    if (!(MODE & FZ_NOSTAGE)) {
    if (!band_start && tid >= (TILE_ROWS - HIST) / 4 - SHIFT / 4) {
      // the rows this thread is about to overwrite become the history window (u - 1024)
#pragma unroll
      for (int c = 0; c < 4; c++)
        sts4(L, F_W + c * F_WS + HIST + u0 - TILE_ROWS, lds4(L, F_W + c * F_WS + HIST + u0));
      if (tid >= BLOCK - SHIFT / 4) {  // ... and the last four quads are carried whole
#pragma unroll
        for (int c = 0; c < 5; c++)
          sts4(L, F_G + c * F_TS + u0 - TILE_ROWS, lds4(L, F_G + c * F_TS + u0));
        L[F_QSEL + tid - (BLOCK - SHIFT / 4)] = L[F_QSEL + SHIFT / 4 + tid];
        L[F_A9 + tid - (BLOCK - SHIFT / 4)] = L[F_A9 + SHIFT / 4 + tid];
      }
    }
    sts4(L, F_W + 0 * F_WS + HIST + u0, make_uint4(Q.c[A1][0], Q.c[A1][1], Q.c[A1][2], Q.c[A1][3]));
    sts4(L, F_W + 1 * F_WS + HIST + u0, make_uint4(Q.c[A2][0], Q.c[A2][1], Q.c[A2][2], Q.c[A2][3]));
    sts4(L, F_W + 2 * F_WS + HIST + u0, make_uint4(Q.c[A7][0], Q.c[A7][1], Q.c[A7][2], Q.c[A7][3]));
    sts4(L, F_W + 3 * F_WS + HIST + u0, make_uint4(Q.c[A8][0], Q.c[A8][1], Q.c[A8][2], Q.c[A8][3]));
    sts4(L, F_G + 0 * F_TS + u0, make_uint4(Q.c[A0][0], Q.c[A0][1], Q.c[A0][2], Q.c[A0][3]));
    sts4(L, F_G + 1 * F_TS + u0, make_uint4(Q.c[A3][0], Q.c[A3][1], Q.c[A3][2], Q.c[A3][3]));
    sts4(L, F_G + 2 * F_TS + u0, make_uint4(Q.c[A4][0], Q.c[A4][1], Q.c[A4][2], Q.c[A4][3]));
    sts4(L, F_G + 3 * F_TS + u0, make_uint4(Q.c[A5][0], Q.c[A5][1], Q.c[A5][2], Q.c[A5][3]));
    sts4(L, F_G + 4 * F_TS + u0, make_uint4(Q.c[A6][0], Q.c[A6][1], Q.c[A6][2], Q.c[A6][3]));
    L[F_QSEL + SHIFT / 4 + tid] = (fx.x & 0xffffu) | (((fx.y | fx.z | fx.w) & 0xffffu) ? 1u << 16 : 0u);
    L[F_A9 + SHIFT / 4 + tid] = a9.x;
    }
    tick(2);
    if ((MODE & FZ_STORE) && gq < total_quads) {
#pragma unroll
      for (int c = 0; c < 11; c++) {
        const u32x4 v = c < 10 ? u32x4{Q.c[c][0], Q.c[c][1], Q.c[c][2], Q.c[c][3]}
                               : u32x4{Q.fx[0], Q.fx[1], Q.fx[2], Q.fx[3]};
        u32x4* dst = reinterpret_cast<u32x4*>((c < 10 ? adv + (uint64_t)c * total_rows : fixed) + row0);
        __builtin_nontemporal_store(v, dst);
      }
    }

    tick(3);
    // ---- A4. TileInfo: stage the one of tile i + 2, load the one of tile i + 3
    if (tid < 6) {
      sts4(L, F_INFO + 24 * (uint32_t)((i + 2) % 3) + 4 * tid, ti);
      const uint64_t t3 = seq(i + 3);
      ti = t3 < n_tiles ? reinterpret_cast<const uint4*>(tinfo + t3)[tid] : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    tick(4);

    // ---- C. build the next tile's G table, check this tile
    if (!(MODE & FZ_NOGT) && has_next && (tid >> 6) == GT_WAVE)
      build_g_table(L + F_GS + nxt * FSET, ninfo, Sg, (int64_t)(tn * TILE_ROWS) - SHIFT, n,
                    total_rows, (uint32_t)tid & 63u, kFusedGT);
    const uint32_t* S = L + F_GS + cur * FSET;
    tick(5);
    if ((MODE & FZ_LOOKUP) && gq < total_quads) {
      // the staged cells of this thread's rows (LDS, as every other check reads them)
      const uint4 q0 = T.quad(A0, (uint32_t)u0), q1 = T.quad(A1, (uint32_t)u0), q2 = T.quad(A2, (uint32_t)u0);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t tg = comp(q0, j), de = comp(q1, j), sp = comp(q2, j);
        if (!(de < 65536u && tg == tag16(de) && sp == spread16(de & 0xffffu)))
          A.fail(row0 + j, B2F_CODE_LOOKUP);
      }
    }
    if ((MODE & FZ_GATES) && gq < total_quads) {
      // the fixed cells this thread assigned against the keygen structure of its quad
      uint4 xf = make_uint4(0, 0, 0, 0);
      if (own_rounds != ~0u) {
        const QuadInfo d = decode_quad(own_lq, own_rounds);
        xf = fixed_of_quad(d, d.kind == K_CONST ? IV[d.a & 7u] : 0ull);
      }
      if ((fx.x ^ xf.x) | (fx.y ^ xf.y) | (fx.z ^ xf.z) | (fx.w ^ xf.w)) {
#pragma unroll
        for (int j = 0; j < 4; j++)
          if (comp(fx, j) != comp(xf, j)) A.fail(row0 + j, B2F_CODE_FIXED);
      }
    }
    const GCarve C{F_QSEL, F_A9, F_CT, F_G, F_TS, SHIFT, U_END, true};
    const uint32_t ng = S[FS_NG];
    if (MODE & FZ_GATES) g_pass(T, A, L, S + FS_GT, ng, base0, (uint32_t)tid & 63u, (uint32_t)tid >> 6, C);
    if (MODE & FZ_COPIES) g_copies(A, L, S + FS_GT, ng, base0, (uint32_t)tid, C);
    tick(6);
    const int hi = last_tile ? U_END + F_HALO : U_END;
    if ((MODE & (FZ_GATES | FZ_COPIES)) && !canonical_quad(L, S, SHIFT / 4 + tid, fx)) {
      if (MODE & FZ_GATES) quad_gates_f(T, A, fx, a9, u0, SHIFT, hi, base0);
      const uint32_t pq = reinterpret_cast<const uint8_t*>(S + FS_QM)[SHIFT / 4 + tid];
      if ((MODE & FZ_COPIES) && pq == 0xffu && own_rounds != ~0u) {  // init/final-block copies
        const uint64_t o = row0 - 4ull * own_lq;
        const uint64_t ofirst = first < n ? reinterpret_cast<const uint64_t*>(info + 2)[0] : ~0ull;
        const Src<F_WS> src{L + F_W, L + F_IC, adv, total_rows, (uint64_t)(base0 - HIST), ofirst};
        copies_edge(A, T.quad(A3, (uint32_t)u0), T.quad(A4, (uint32_t)u0), T.quad(A5, (uint32_t)u0),
                    src, o, own_rounds, own_lq);
      }
    }
    if (tid >= BLOCK - SHIFT / 4) {
      // the carried quad u 0..15 this thread assigned last tile: its gates that end here
      const int qc = tid - (BLOCK - SHIFT / 4);
      const uint4 cfx = lds4(L, F_CAR + 4 * qc), ca9 = lds4(L, F_CAR + 16 + 4 * qc);
      if ((MODE & FZ_GATES) && !canonical_quad(L, S, qc, cfx))
        quad_gates_f(T, A, cfx, ca9, 4 * qc, SHIFT, hi, base0);
      sts4(L, F_CAR + 4 * qc, fx);
      sts4(L, F_CAR + 16 + 4 * qc, a9);
    }
    __syncthreads();
    tick(7);
    P = Pn;
    icw = icw_n;
    ic_now = ic_next;
  }
  if ((MODE & FZ_CLOCK) && (tid & 63) == 0) {
#pragma unroll
    for (int k = 0; k < 8; k++) atomicAdd(&clk[8 * (tid >> 6) + k], (unsigned long long)ck[k]);
  }
  // ---- flush the workgroup's counters: one global atomic per non-zero counter
  flush_report(A, rep, tid);
}

}  // namespace

namespace b2f {

// Launch the fused kernel (b2f_fill_eval_dev): `tinfo` holds the TileInfo of every tile for
// rows t * 1024 - 16 (tile_info_kernel with shift 16), `rec` the record kernel's states.
hipError_t launch_fill_eval(const b2f_input* d_in, uint32_t n, const uint64_t* d_off,
                            uint64_t total_rows, const uint64_t* rec, uint32_t* d_adv,
                            uint32_t* d_fixed, const void* tinfo, uint64_t n_tiles, uint32_t band,
                            b2f_eval_report* d_rep, const int* d_status, uint64_t inj_row,
                            uint32_t inj_col, uint32_t inj_mask, int mode, int cu_count,
                            unsigned long long* clk, hipStream_t s) {
  if (band == 0) band = 1;
  const uint64_t n_bands = (n_tiles + band - 1) / band;
  const uint64_t cap = (uint64_t)cu_count * 3;
  const uint32_t grid = (uint32_t)(n_bands < cap ? (n_bands ? n_bands : 1) : cap);
  Inject inj;
  inj.quad = inj_row == ~0ull ? ~0ull : inj_row / 4;
  inj.j = (uint32_t)(inj_row & 3);
  inj.col = inj_col;
  inj.mask = inj_mask;
#ifndef B2F_DIAG
  mode = FZ_FULL;  // the product library launches the full kernel only
#endif
  if (inj.quad != ~0ull) mode |= FZ_INJECT;
  switch (mode) {
#define B2F_FUSED(M)                                                                          \
  case M:                                                                                     \
    hipLaunchKernelGGL(fused_kernel<M>, dim3(grid), dim3(BLOCK), 0, s, d_in, n, d_off,        \
                       total_rows, rec, d_adv, d_fixed, reinterpret_cast<const TileInfo*>(tinfo), \
                       n_tiles, band, d_rep, d_status, inj, clk);                             \
    break;
#ifdef B2F_DIAG
    B2F_FUSED(0) B2F_FUSED(2) B2F_FUSED(3) B2F_FUSED(10) B2F_FUSED(18) B2F_FUSED(8) B2F_FUSED(16)
    B2F_FUSED(34) B2F_FUSED(66) B2F_FUSED(98) B2F_FUSED(FZ_FULL | FZ_CLOCK)
#endif
    B2F_FUSED(FZ_FULL | FZ_INJECT)
    default: B2F_FUSED(FZ_FULL)
#undef B2F_FUSED
  }
  return hipGetLastError();
}

}  // namespace b2f

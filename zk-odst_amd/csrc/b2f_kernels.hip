// b2f_kernels.hip -- gfx950 kernels of the BLAKE2f Table16 engine and the C ABI of
// include/b2f.h. Trace contract: docs/LAYOUT.md. Design notes: DESIGN.md.
//
// Kernels (one stream, in order):
//   record_kernel  a DPP quad per instance: the BLAKE2f compression itself (RFC 7693 / EIP-152,
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
#include <map>
#include <vector>

#include "../../include/b2f.h"
#include "b2f_common.h"

using namespace b2f;

namespace b2f {
size_t lookup_scratch_bytes(uint32_t group, uint64_t usable_rows);
hipError_t launch_lookup(const uint32_t* d_advice, uint64_t total_rows,
                         const uint64_t* d_row_begin, uint32_t n_circuits, uint64_t usable_rows,
                         const uint64_t* theta, const uint64_t* beta, const uint64_t* gamma,
                         uint32_t form, uint64_t* d_out, uint64_t out_rows, uint64_t* d_first_bad,
                         void* scratch, uint32_t group, int* sticky, hipStream_t s2,
                         hipEvent_t ev_fork, hipEvent_t ev_join, hipStream_t s3, hipEvent_t ev_tab,
                         hipEvent_t ev_sorted, hipStream_t s);
hipError_t launch_spread_table(uint64_t usable_rows, uint32_t form, uint64_t* d_out,
                               uint64_t out_rows, hipStream_t s);
size_t perm_scratch_bytes(uint32_t k, uint64_t usable_rows, size_t n_inst, uint32_t chunk_len);
size_t perm_sigma_scratch_bytes(uint32_t k);
hipError_t launch_permutation_sigma(const uint64_t* d_inst, size_t n_inst, const uint32_t* d_pool, uint32_t k,
                                    const uint64_t* omega, const uint64_t* delta, uint32_t form,
                                    uint64_t* d_sigma, uint64_t out_rows, void* scratch, hipStream_t s);
hipError_t launch_permutation(const uint32_t* d_advice, uint64_t total_rows, uint64_t row0,
                              const uint64_t* d_inst, size_t n_inst, const uint32_t* d_pool,
                              uint32_t k, uint64_t usable_rows, const uint64_t* omega,
                              const uint64_t* delta, const uint64_t* beta, const uint64_t* gamma,
                              uint32_t chunk_len, uint32_t form, uint64_t* d_sigma, uint64_t* d_z,
                              uint64_t out_rows, void* scratch, int* sticky, hipStream_t s2,
                              hipEvent_t ev_fork, hipEvent_t ev_join, hipStream_t s);
hipError_t launch_export_fp(const uint32_t* d_advice, uint64_t total_rows, uint64_t row_begin,
                            uint64_t nrows, uint32_t form, uint64_t* d_out, uint64_t out_rows,
                            int cu_count, unsigned* tctr, hipStream_t s);  // b2f_export.hip
size_t fused_scratch_bytes(uint64_t tiles);
uint64_t fused_instance_tiles(uint64_t total_rows, uint64_t n);
hipError_t launch_eval_fast(const uint32_t* d_adv, const uint32_t* d_fixed, const uint64_t* d_off, uint32_t n,
                            uint64_t total_rows, void* scratch, uint64_t tiles, const int* d_status,
                            int cu_count, hipStream_t s, const uint32_t** gate, int mode);  // b2f_fused.hip
hipError_t launch_fill_eval(const b2f_input* d_in, uint32_t n, const uint64_t* d_off,
                            uint64_t total_rows, const uint64_t* rec, uint32_t* d_adv,
                            uint32_t* d_fixed, void* scratch, uint64_t tiles,
                            b2f_eval_report* d_rep, const int* d_status, uint64_t inj_row,
                            uint32_t inj_col, uint32_t inj_mask, int mode, int cu_count,
                            unsigned long long* clk, const uint64_t* seg, uint64_t seg_cap,
                            hipStream_t s);  // b2f_fused.hip
}

namespace {


// ------------------------------------------------------------------------- record kernel

// Four lanes (a DPP quad) per instance: lane c holds column c of the state (v[c], v[c+4],
// v[c+8], v[c+12]) and runs the column step's G(c, c+4, c+8, c+12); for the diagonal step the
// b, c and d rows are rotated by 1, 2 and 3 lanes so that lane c runs G(c, 4+(c+1)%4,
// 8+(c+2)%4, 12+(c+3)%4), then rotated back. Every half-round state is dumped (128 B per
// quad) for the fill's quad builders.
template <int CTRL>
__device__ __forceinline__ uint64_t quad_dpp64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xF, 0xF, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, true);
  return ((uint64_t)hi << 32) | lo;
}
constexpr int QROT1 = 0x39, QROT2 = 0x4E, QROT3 = 0x93;  // lane j <- lane (j + k) % 4

// A device-side error: the per-call word (the call's later kernels exit early on it), the
// sticky word (only b2f_sync clears it, so a later call cannot erase an earlier error) and,
// for calls that produce a verdict, the report: a rejected batch never reads clean.
__device__ __forceinline__ void raise_error(int* status, int* sticky, b2f_eval_report* rep, int code) {
  atomicOr(status, 1 << code);
  atomicOr(sticky, 1 << code);
  if (rep) {
    rep->rows_checked = 0;
    const unsigned long long why = code == B2F_ERR_CHECK ? B2F_CODE_CHECK : B2F_CODE_LAYOUT;
    atomicMin((unsigned long long*)&rep->first_failure, why);
  }
}

__global__ void __launch_bounds__(BLOCK) record_kernel(const b2f_input* __restrict__ in,
                                                      uint32_t n,
                                                      const uint64_t* __restrict__ off,
                                                      uint64_t total_rows,
                                                      uint64_t states_cap,
                                                      uint64_t* __restrict__ rec,
                                                      uint64_t* __restrict__ h_out,
                                                      int* __restrict__ status,
                                                      int* __restrict__ sticky,
                                                      b2f_eval_report* __restrict__ rep,
                                                      bool lite, uint64_t* __restrict__ seg,
                                                      uint64_t seg_cap) {
  const uint32_t gt = blockIdx.x * BLOCK + threadIdx.x;
  const uint32_t i = gt >> 2, c = gt & 3u;  // the quad's four lanes share instance i
  if (i >= n) return;
  const b2f_input* x = in + i;
  uint32_t rounds = x->rounds;
  uint64_t o0 = off[i], o1 = off[i + 1];
  if (rounds > B2F_MAX_ROUNDS) {
    if (c == 0) raise_error(status, sticky, rep, B2F_ERR_ROUNDS);
    return;
  }
  uint64_t R = (uint64_t)FIXED_ROWS + (uint64_t)ROUND_ROWS * rounds;
  bool bad = (o1 - o0 != R) || o1 > total_rows || (i == 0 && o0 != 0) ||
             (o0 < (uint64_t)FIXED_ROWS * i) || ((o0 - (uint64_t)FIXED_ROWS * i) % ROUND_ROWS);
  uint64_t st = bad ? 0 : state_index(o0, i);
  if (!bad && st + 2ull * rounds + 1 > states_cap) bad = true;
  if (bad) {
    if (c == 0) raise_error(status, sticky, rep, B2F_ERR_LAYOUT);
    return;
  }

  const uint64_t h0 = x->h[c], h1 = x->h[c + 4];
  uint64_t va = h0, vb = h1, vc = c_iv[c], vd = c_iv[c + 4];
  if (c == 0) vd ^= x->t[0];
  if (c == 1) vd ^= x->t[1];
  if (c == 2 && x->f) vd = ~vd;

  // the instance's 16 message words in LDS (each lane of the quad loads four), so the rounds'
  // SIGMA-permuted reads are LDS reads instead of dependent global loads
  __shared__ uint64_t Msg[BLOCK / 4][16];
  uint64_t* mw = Msg[threadIdx.x >> 2];
#pragma unroll
  for (int k = 0; k < 4; k++) mw[4 * c + k] = x->m[4 * c + k];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

#ifndef B2F_REC_COLUMN  // diagnostics: B2F_REC_COLUMN = the column-wise 8-byte stores
  // each dump transposed inside the quad through LDS: lane c writes row c of the 4 x 4 work matrix
  // (words 4c .. 4c + 3, 32 contiguous bytes) instead of column c as four 8-byte stores
  __shared__ __attribute__((aligned(16))) uint64_t Tq[BLOCK / 4][16];
  uint64_t* tq = Tq[threadIdx.x >> 2];
  uint64_t* s = rec + st * 16 + 4 * c;
  // lite (the fused path, whose half-round launch carries the state from tile to tile): only the
  // last two states -- the edge launch's final state and its producers' last half-round -- of the
  // 2 rounds + 1
  uint32_t k = 0;
  const uint32_t keep = lite ? (rounds ? 2 * rounds - 1 : 0) : 0;
  const uint32_t hr_all = 2 * rounds;
  // lite: also the states before and at every later segment start m SEG_HR < 2 rounds (a
  // segment's first tile starts from the one and recomputes the previous tile's tail from the
  // other); the segments themselves go to the fused launch's list
  auto keep_state = [&](uint32_t q) {
    return q >= keep || (q % SEG_HR == 0 && q != 0 && q < hr_all) ||
           ((q + 1) % SEG_HR == 0 && q + 1 < hr_all);
  };
  if (lite && seg && c == 0 && hr_all > SEG_HR) {
    const uint64_t nseg = (hr_all - 1) / SEG_HR;  // segments m = 1 .. nseg
    const uint64_t at = atomicAdd(reinterpret_cast<unsigned long long*>(seg), (unsigned long long)nseg);
    for (uint64_t m = 1; m <= nseg; m++)
      if (at + m - 1 < seg_cap) seg[1 + at + m - 1] = ((uint64_t)i << 32) | m;
    // the list is sized from an upper bound on the states, so this never fires; if it did, the
    // fused launch drains only seg_cap entries and the call must not read clean
    if (at + nseg > seg_cap) raise_error(status, sticky, rep, B2F_ERR_CHECK);
  }
  auto dump = [&](void) {
    if (!keep_state(k++)) {
      s += 16;
      return;
    }
    tq[c] = va;
    tq[4 + c] = vb;
    tq[8 + c] = vc;
    tq[12 + c] = vd;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint4 r0 = *reinterpret_cast<const uint4*>(tq + 4 * c), r1 = *reinterpret_cast<const uint4*>(tq + 4 * c + 2);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    *reinterpret_cast<uint4*>(s) = r0;
    *reinterpret_cast<uint4*>(s + 2) = r1;
    s += 16;
  };
#else
  uint64_t* s = rec + st * 16 + c;
  auto dump = [&](void) {
    s[0] = va;
    s[4] = vb;
    s[8] = vc;
    s[12] = vd;
    s += 16;
  };
#endif
  auto G = [&](uint64_t mx, uint64_t my) {
    va = va + vb + mx; vd = rotr64(vd ^ va, 32);
    vc = vc + vd;      vb = rotr64(vb ^ vc, 24);
    va = va + vb + my; vd = rotr64(vd ^ va, 16);
    vc = vc + vd;      vb = rotr64(vb ^ vc, 63);
  };
  dump();
  for (uint32_t r = 0; r < rounds; r++) {
    const uint8_t* sg = c_sigma[r % 10];
    const uint64_t m0 = mw[sg[2 * c]], m1 = mw[sg[2 * c + 1]];
    const uint64_t m2 = mw[sg[8 + 2 * c]], m3 = mw[sg[9 + 2 * c]];
    G(m0, m1);  // column step
    dump();
    vb = quad_dpp64<QROT1>(vb);
    vc = quad_dpp64<QROT2>(vc);
    vd = quad_dpp64<QROT3>(vd);
    G(m2, m3);  // diagonal step
    vb = quad_dpp64<QROT3>(vb);
    vc = quad_dpp64<QROT2>(vc);
    vd = quad_dpp64<QROT1>(vd);
    dump();
  }
  if (h_out) {
    h_out[8 * (uint64_t)i + c] = h0 ^ va ^ vc;
    h_out[8 * (uint64_t)i + c + 4] = h1 ^ vb ^ vd;
  }
}


// Per-tile instance context: the instance holding the tile's first row and the offsets of the
// next 8 instances. One tiny prepass shared by the fill and eval launches of a call.
// `shift`: context of row t * 1024 - shift (the fused kernel's checks lag by 16 rows).
__global__ void tile_info_kernel(const uint64_t* __restrict__ off, uint32_t n, uint64_t n_tiles,
                                 uint32_t shift, TileInfo* __restrict__ ti) {
  uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_tiles) return;
  uint64_t row = t * TILE_ROWS >= shift ? t * TILE_ROWS - shift : 0;
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


// MODE (diagnostics; the product uses FILL_FULL): bit 0 = compute the cells (else zeros),
// bit 1 = non-temporal stores (else plain stores), bit 3 = per-phase s_memtime totals per wave
// slot into clk (b2f_debug_clock; phases: next tile's operand loads issued, cells formed -- the
// wait for this tile's loads included --, stores issued, loop, final vmcnt drain).
enum { FILL_COMPUTE = 1, FILL_NT = 2, FILL_FULL = 3, FILL_CLOCK = 8 };

// Tiles of 1024 rows are dealt round-robin over the (persistent) workgroups, so at any time
// the chip writes a narrow band of every column: one DRAM-friendly front per column instead
// of one per workgroup. Software-pipelined one tile deep: the tile's instance context is read
// with scalar loads and the operand words of tile t + grid (quad_ops) are loaded before tile
// t's stores are issued (vmcnt counts loads and stores in issue order, so a load issued after
// the stores would wait for them).
#ifndef B2F_FILL_WAVES
#define B2F_FILL_WAVES 1  // minimum waves per SIMD the fill is compiled for (register bound)
#endif
#ifndef B2F_FILL_DYN
// 1: tiles claimed from a counter in chunks of FILL_CHUNK. One tile per claim was 15.21 vs 10.13
// ms (2^18 x 12, profiles/r06k_ab_dyn_*.txt): 1.3 M claims in 10 ms on one address serialise.
// Per claim 4 / 8 / 16 tiles: 9.02 / 9.07 / 9.14 ms against 10.01 dealt round-robin; {1,4,12}:
// 4.68 / 4.71 / 4.77 against 5.16 (profiles/r06l_ab_fill_*.txt, r06m_ab_fill_*.txt); 2 against 4
// on another box: 9.25 vs 9.36, 4.45 vs 4.47 (profiles/r06n_ab_*.txt)
#define B2F_FILL_DYN 1
#endif
#ifndef B2F_FILL_CHUNK
#define B2F_FILL_CHUNK 2
#endif
constexpr uint32_t FILL_CHUNK = B2F_FILL_CHUNK;
template <int MODE>
__global__ void __launch_bounds__(BLOCK, B2F_FILL_WAVES) fill_kernel(const b2f_input* __restrict__ in,
                                                    uint32_t n,
                                                    const uint64_t* __restrict__ off,
                                                    uint64_t total_rows,
                                                    const uint64_t* __restrict__ rec,
                                                    uint32_t* __restrict__ adv,
                                                    uint32_t* __restrict__ fixed,
                                                    const int* __restrict__ status,
                                                    const TileInfo* __restrict__ tinfo,
                                                    uint64_t n_tiles,
                                                    unsigned long long* __restrict__ clk,
                                                    unsigned* __restrict__ tctr) {
  __shared__ uint32_t rows[ROW_TABLE_WORDS];
  __shared__ uint32_t s_tile[2];  // B2F_FILL_DYN: the workgroup's claimed tiles (double-buffered)
  uint64_t ck[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tp = 0;
  auto tick = [&](int k) {
    if (MODE & FILL_CLOCK) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      if (k >= 0) ck[k] += now - tp;
      tp = now;
    }
  };
  __shared__ __attribute__((aligned(16))) uint32_t sgiv[40 + 16];  // SIGMA bytes, IV
  const int tid = threadIdx.x;
  if (tid < ROW_TABLE_WORDS) rows[tid] = (&c_rows.r[0][0])[tid];
  if (tid < 40) sgiv[tid] = reinterpret_cast<const uint32_t*>(c_sigma)[tid];
  if (tid < 16) sgiv[40 + tid] = reinterpret_cast<const uint32_t*>(c_iv)[tid];
  __syncthreads();
  if (*status) return;  // the record kernel rejected the layout: write nothing
  const uint8_t* Sg = reinterpret_cast<const uint8_t*>(sgiv);
  const uint64_t* IV = reinterpret_cast<const uint64_t*>(sgiv + 40);
  const uint64_t total_quads = total_rows >> 2;
  const uint64_t used_rows = off[n];
  const uint64_t G = gridDim.x;
  auto ops = [&](QuadOps& R, uint64_t tt) {
    R.rounds = ~0u;
    R.lq = 0;
#pragma unroll
    for (int k = 0; k < 6; k++) R.w[k] = 0;
    if (MODE & FILL_COMPUTE) {
      const TileInfo ti = tinfo[tt];  // workgroup-uniform: scalar loads
      quad_ops_ti(R, 4 * (tt * BLOCK + tid), ti, n, used_rows, in, rec, Sg);
    }
  };
#if B2F_FILL_DYN
  // tiles claimed from the launch's counter in chunks of FILL_CHUNK consecutive tiles (a barrier
  // per chunk shares the claim), one tile ahead: the workgroups finish within a chunk of each other
  uint32_t slot = 0, cleft = 0;
  uint64_t cbase = 0;
  auto claim = [&]() -> uint64_t {
    if (cleft == 0) {  // workgroup-uniform
      if (tid == 0) s_tile[slot] = atomicAdd(tctr, (unsigned)FILL_CHUNK);
      __syncthreads();
      cbase = __builtin_amdgcn_readfirstlane(s_tile[slot]);
      slot ^= 1u;
      cleft = FILL_CHUNK;
    }
    cleft--;
    return cbase++;
  };
  (void)G;
  uint64_t t = claim();
#else
  (void)tctr;
  uint64_t t = blockIdx.x;
#endif
  QuadOps P;
  tick(-1);
  if (t < n_tiles) ops(P, t);
  tick(0);
  while (t < n_tiles) {
#if B2F_FILL_DYN
    const uint64_t tn = claim();
#else
    const uint64_t tn = t + G;
#endif
    QuadOps Pn;
    Pn.rounds = ~0u;
    if (tn < n_tiles) ops(Pn, tn);
    tick(0);
    const uint64_t gq = t * BLOCK + tid;
    if (gq < total_quads) {
      Quad Q;
      zero(Q);
      if ((MODE & FILL_COMPUTE) && P.rounds != ~0u) {
        const uint32_t rq = P.lq - INIT_QUADS;
        if (P.lq >= INIT_QUADS && rq < ROUND_QUADS * P.rounds)
          quad_round(Q, P.w[0], P.w[1], P.w[2], P.w[3], P.w[4], P.w[5], (rq % ROUND_QUADS) % G_QUADS, rows);
        else
          quad_cells_ops(Q, P, IV);  // init and final regions
      }
      if (MODE & FILL_CLOCK) {  // the cells must exist before the clock reads: a use of them
        uint32_t sink = 0;
#pragma unroll
        for (int c = 0; c < 10; c++) sink ^= Q.c[c][0];
        asm volatile("" ::"v"(sink));
      }
      tick(1);
      const uint64_t row = 4 * gq;
#pragma unroll
      for (int c = 0; c < 11; c++) {
        u32x4 v = c < 10 ? u32x4{Q.c[c][0], Q.c[c][1], Q.c[c][2], Q.c[c][3]}
                         : u32x4{Q.fx[0], Q.fx[1], Q.fx[2], Q.fx[3]};
        u32x4* dst = reinterpret_cast<u32x4*>((c < 10 ? adv + (uint64_t)c * total_rows : fixed) + row);
        if (MODE & FILL_NT) __builtin_nontemporal_store(v, dst);
        else *dst = v;
      }
    }
    tick(2);
    P = Pn;
    t = tn;
    tick(3);
  }
  if (MODE & FILL_CLOCK) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tick(4);
    if ((tid & 63) == 0) {
#pragma unroll
      for (int k = 0; k < 8; k++) atomicAdd(&clk[8 * (tid >> 6) + k], (unsigned long long)ck[k]);
    }
  }
}

// Diagnostics (B2F_DIAG_FILL=4 in the diagnostics library): a second store floor for the fill,
// a plain non-temporal 16-byte stream of zeros over the same 11 columns in address order (each
// column front to back, grid-stride, nothing else per chunk): what the box's write path does
// for these 60 GB with no tile structure at all.
#ifdef B2F_DIAG
__global__ void __launch_bounds__(BLOCK) store_stream_kernel(uint32_t* __restrict__ adv,
                                                            uint32_t* __restrict__ fixed,
                                                            uint64_t total_rows) {
  const uint64_t per_col = total_rows >> 2, chunks = 11 * per_col;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  const u32x4 z = u32x4{0u, 0u, 0u, 0u};
  for (uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; j < chunks; j += stride) {
    const uint64_t c = j / per_col, q = j - c * per_col;
    u32x4* dst = reinterpret_cast<u32x4*>((c < 10 ? adv + c * total_rows : fixed) + 4 * q);
    __builtin_nontemporal_store(z, dst);
  }
}
#endif

// Diagnostics (B2F_DIAG_EVAL=32 in the diagnostics library): the read counterpart of
// store_stream_kernel -- every 16-byte quad of the same 11 columns loaded once in address order
// (grid-stride, 4 loads in flight per thread), XOR-folded so no load is dead (the fold lands in
// the spare status word only if it equals a constant): the box's read rate for these bytes with
// no tile structure, the eval's load floor. (eval_kernel<1>, the floor before round 6, does not
// count as one: its FETCH_SIZE is 0.86x the trace's bytes, profiles/r06z3_eval_floor_fetch.json.)
#ifdef B2F_DIAG
__global__ void __launch_bounds__(BLOCK) load_stream_kernel(const uint32_t* __restrict__ adv,
                                                           const uint32_t* __restrict__ fixed,
                                                           uint64_t total_rows, int* __restrict__ sink) {
  const uint64_t per_col = total_rows >> 2, chunks = 11 * per_col;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  auto at = [&](uint64_t j) -> const u32x4* {
    const uint64_t c = j / per_col, q = j - c * per_col;
    return reinterpret_cast<const u32x4*>((c < 10 ? adv + c * total_rows : fixed) + 4 * q);
  };
  uint32_t acc = 0;
  for (uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; j < chunks; j += 4 * stride) {
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint64_t jk = j + k * stride;
      v[k] = jk < chunks ? *at(jk) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int k = 0; k < 4; k++) acc ^= v[k][0] ^ v[k][1] ^ v[k][2] ^ v[k][3];
  }
  if (acc == 0x9e3779b9u) sink[0] = 1;
}
#endif

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
constexpr int L_IV = L_ACC + 20 + 2;    // IV, 8 x u64 (CONST rows of the fixed-column check)
constexpr int LDS_WORDS = L_IV + 16;
static_assert(L_INFO % 4 == 0 && L_IC % 4 == 0 && L_G % 4 == 0 && L_CT % 4 == 0 && L_ACC % 2 == 0 &&
                  L_IV % 2 == 0,
              "aligned carve");
static_assert(LDS_WORDS * 4 * 3 <= 160 * 1024, "three eval workgroups per CU");
static_assert(GT_WORDS == GT_WORDS_ && L_GS % 4 == 0 && GSET % 4 == 0, "G table entries are two aligned uint4");
static_assert(MAX_TILE_G * LPG <= BLOCK, "copy lanes");


// Extra (non-own-quad) loads of a tile: 2 slots per thread.
constexpr int X_HIST = 4 * (HIST / 4);          // 384: 96 quads x 4 canonical columns
constexpr int X_HALO = X_HIST + 9 * (HALO_ROWS / 4);  // +36: 4 quads x 9 gate columns
constexpr int X_INIT = X_HALO + 2 * INIT_QUADS;  // +82: 41 quads x (a_1, a_2)
constexpr int X_INFO = X_INIT + 5;               // +5: TileInfo words 0..19 (first, off[9])
constexpr int X_INFO2 = X_INFO + 5;              // +5: the same for tile t + gridDim
static_assert(X_INFO2 <= 2 * BLOCK, "two extra slots per thread");


static_assert(check_table_ok<L_W, WSTRIDE>(), "72 copy checks per G, fields in range");
__constant__ __attribute__((aligned(16))) CheckTable c_checks = make_check_table<L_W, WSTRIDE>();
using Tile = TileT<L_W, WSTRIDE, L_G, TSTRIDE>;
constexpr int CHECK_WORDS = (int)(sizeof(CheckTable) / 4);  // 864


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


constexpr GTCarve kEvalGT{GS_QM, GS_NG, GS_GT, L_IC, L_W, WSTRIDE, BLOCK / 4, BLOCK, 0, MAX_TILE_G};

// MODE (diagnostics; the product uses EVAL_FULL): which checks run on a staged tile.
enum { EVAL_LOOKUP = 1, EVAL_GATES = 2, EVAL_COPIES = 4, EVAL_FULL = 7, EVAL_TOUCH = 8,
       EVAL_CLOCK = 16,    // EVAL_CLOCK: per-phase s_memtime totals per wave (diagnostics)
       EVAL_STREAM = 32 };  // (diagnostics) load_stream_kernel alone: the read floor

// Tiles per band: a workgroup checks EVAL_BAND consecutive tiles, then jumps a grid's worth of
// bands (XCD-aware over bands). Inside a band the history window of a tile is the previous
// tile's tail, moved in LDS instead of loaded again.
#ifndef B2F_EVAL_BAND
#define B2F_EVAL_BAND 8
#endif
constexpr uint64_t EVAL_BAND = B2F_EVAL_BAND;
__device__ __forceinline__ bool hist_in_lds(uint64_t t) { return EVAL_BAND > 1 && t % EVAL_BAND != 0; }

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
                                            uint64_t tnext, uint64_t n_tiles) {
  const uint64_t tile0 = t * TILE_ROWS;
  const uint64_t of = ((uint64_t)fo.w << 32) | fo.z;
  const uint32_t k = x.kind;
  const uint64_t w = k == XK_INIT ? of : k == XK_INFO ? 24 * t : k == XK_INFO2 ? 24 * tnext : tile0;
  const bool ok = k == XK_HIST    ? tile0 >= (uint64_t)HIST && !hist_in_lds(t)
                : k == XK_HALO    ? (t + 1) * BLOCK + x.q < total_quads
                : k == XK_INIT    ? fo.x < n && of + INIT_ROWS <= total_rows
                : k == XK_INFO    ? true
                : k == XK_INFO2   ? tnext < n_tiles
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
                                                    int* __restrict__ status,
                                                    int* __restrict__ sticky,
                                                    unsigned long long* __restrict__ clk,
                                                    const uint32_t* __restrict__ gate) {
  // gate: the fast clean-check pass (launch_eval_fast) found nothing to record -- the report
  // report_init_kernel wrote is already the verdict (an accepted layout only)
  if (gate && *gate == 0 && *status == 0) return;
  __shared__ __attribute__((aligned(16))) uint32_t L[LDS_WORDS];
  uint64_t ck[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tp = 0;
  auto tick = [&](int k) {
    if (MODE & EVAL_CLOCK) {
      const uint64_t now = __builtin_amdgcn_s_memtime();
      if (k >= 0) ck[k] += now - tp;
      tp = now;
    }
  };
  const int tid = threadIdx.x;
  for (int i = tid; i < CHECK_WORDS; i += BLOCK)
    L[L_CT + i] = reinterpret_cast<const uint32_t*>(&c_checks)[i];
  if (tid < 40) L[L_SG + tid] = reinterpret_cast<const uint32_t*>(c_sigma)[tid];
  if (tid < 16) L[L_XS + tid] = expected_sel((uint32_t)tid);
  if (tid < 16) L[L_IV + tid] = reinterpret_cast<const uint32_t*>(c_iv)[tid];
  const uint64_t* IV = reinterpret_cast<const uint64_t*>(L + L_IV);
  const Tile T{L};
  const uint8_t* Sg = reinterpret_cast<const uint8_t*>(L + L_SG);  // [10][16]

  EvalAcc A{L + L_ACC};
  Fails<true> Rec{A, false};  // failures recorded as they are found (a fast-flag pass measured slower here)
  if (tid < 20) L[L_ACC + tid] = 0;
  if (tid == 20) *reinterpret_cast<uint64_t*>(L + L_ACC + 20) = ~0ull;

  const uint64_t total_quads = total_rows >> 2;
  const uint64_t used_rows = off[n];
  const bool layout_ok = used_rows <= total_rows && off[0] == 0;  // never read past the trace
  if (!layout_ok && blockIdx.x == 0 && tid == 0) raise_error(status, sticky, rep, B2F_ERR_LAYOUT);
  const uint64_t G = gridDim.x;

  // XCD-aware deal: workgroups are dispatched to the 8 XCDs round-robin (b % 8), so give each
  // XCD a contiguous run of G / 8 tiles per band. A tile's history window and halo are then the
  // rows its same-XCD neighbours just loaded, served from that XCD's L2 rather than refetched
  // (placement is only a speed hint; any placement gives the same result).
  const uint64_t b0 = (G % 8 == 0) ? (blockIdx.x % 8) * (G / 8) + blockIdx.x / 8 : blockIdx.x;
  auto seq = [&](uint64_t k) { return (b0 + (k / EVAL_BAND) * G) * EVAL_BAND + k % EVAL_BAND; };
  uint64_t t = seq(0);
  // fo (first instance and its offset, per tile) is workgroup-uniform. Only the first tile's
  // is a scalar load; the next tiles' come from the staged TileInfo in LDS (INFO2): on CDNA
  // lgkmcnt counts scalar loads and LDS operations together, so a scalar load issued in the
  // tile loop would make the first LDS read of the checks wait for a memory round trip.
  uint4 q[NCOL_T], x0 = make_uint4(0, 0, 0, 0), x1 = x0, fo = x0;
  const Extra e0 = make_extra(tid, adv, total_rows, tinfo);
  const Extra e1 = make_extra(tid + BLOCK, adv, total_rows, tinfo);
  auto load_tile = [&](uint64_t tt, const uint4& f, uint64_t tt_next) {
    const uint64_t gq = tt * BLOCK + tid;
#pragma unroll
    for (int c = 0; c < NCOL_T; c++)
      q[c] = gq < total_quads
                 ? *reinterpret_cast<const uint4*>((c < 10 ? adv + (uint64_t)c * total_rows : fixed) + 4 * gq)
                 : make_uint4(0, 0, 0, 0);
    x0 = extra_load(e0, tt, f, n, total_rows, total_quads, tt_next, n_tiles);
    x1 = extra_load(e1, tt, f, n, total_rows, total_quads, tt_next, n_tiles);
  };
  if (layout_ok && t < n_tiles) {
    fo = *reinterpret_cast<const uint4*>(tinfo + t);
    load_tile(t, fo, seq(1));
  }
  for (uint32_t iter = 0; layout_ok && t < n_tiles; iter++, t = seq(iter)) {
    tick(-1);
    const bool hist_lds = hist_in_lds(t);
    if (hist_lds && tid >= (TILE_ROWS - HIST) / 4) {
      // the previous tile's tail (still staged) becomes this tile's history window
#pragma unroll
      for (int ci = 0; ci < 4; ci++) {
        const int w = L_W + ci * WSTRIDE + HIST + 4 * tid;
        *reinterpret_cast<uint4*>(&L[w - TILE_ROWS]) = *reinterpret_cast<const uint4*>(&L[w]);
      }
    }
    // ---- stage tile t: registers -> LDS
#pragma unroll
    for (int c = 0; c < 9; c++) *reinterpret_cast<uint4*>(&L[lds_cell(c, 4 * tid)]) = q[c];
    const uint4 cur9 = q[A9], curfx = q[10];
    if (MODE & (EVAL_GATES | EVAL_COPIES)) {
      L[L_QSEL + tid] = (curfx.x & 0xffffu) | (((curfx.y | curfx.z | curfx.w) & 0xffffu) ? 1u << 16 : 0u);
      L[L_A9 + tid] = cur9.x;
    }
    if (e0.kind != XK_NONE && !(hist_lds && e0.kind == XK_HIST)) *reinterpret_cast<uint4*>(&L[e0.lds]) = x0;
    if (e1.kind != XK_NONE && !(hist_lds && e1.kind == XK_HIST)) *reinterpret_cast<uint4*>(&L[e1.lds]) = x1;
    // ---- lookups on the quad's 4 rows, from the loaded cells, before the barrier
    if ((MODE & EVAL_LOOKUP) && t * BLOCK + tid < total_quads) {
      const uint64_t r0 = 4 * (t * BLOCK + tid);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t tg = comp(q[A0], j), de = comp(q[A1], j), sp = comp(q[A2], j);
        if (!(de < 65536u && tg == tag16(de) && sp == spread16(de & 0xffffu)))
          A.fail(r0 + j, B2F_CODE_LOOKUP);
      }
    }
    tick(0);
    __syncthreads();
    tick(1);
    // ---- prefetch this workgroup's next tile into registers while tile t is checked
    const uint64_t tn = seq(iter + 1);
    if (tn < n_tiles) {
      // TileInfo of tile tn, staged from the INFO2 slots this iteration
      const uint4 fo_next = make_uint4(L[L_INFO2], 0u, L[L_INFO2 + 2], L[L_INFO2 + 3]);
      load_tile(tn, fo_next, seq(iter + 2));
    }
    tick(2);
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
    if (MODE & (EVAL_GATES | EVAL_COPIES)) {
      // ---- G tables: the first wave builds the next tile's (from INFO2) while this tile is
      // checked with the one built during the previous iteration
      const uint32_t* S = L + L_GS + (iter & 1) * GSET;
      uint32_t* Sn = L + L_GS + ((iter + 1) & 1) * GSET;
      if (iter == 0) {  // nothing was built ahead for the first tile
        if (tid < 64)
          build_g_table(L + L_GS, L + L_INFO, Sg, (int64_t)tile0, n, total_rows, (uint32_t)tid, kEvalGT);
        __syncthreads();
      }
      if ((tid >> 6) == GT_WAVE)  // the wave with the lightest G pass (XOR) builds ahead
        build_g_table(Sn, L + L_INFO2, Sg, (int64_t)(tn * TILE_ROWS), tn < n_tiles ? n : 0,
                      total_rows, (uint32_t)tid & 63u, kEvalGT);
      tick(3);
      const GCarve C{L_QSEL, L_A9, L_CT, L_G, TSTRIDE, 0, TILE_ROWS, false};
      const uint32_t ng = S[GS_NG];
      if (MODE & EVAL_GATES)
        g_pass(T, Rec, L, S + GS_GT, ng, (int64_t)tile0, (uint32_t)tid & 63u, (uint32_t)tid >> 6, C);
      tick(4);
      if (MODE & EVAL_COPIES) g_copies(Rec, L, S + GS_GT, ng, (int64_t)tile0, (uint32_t)tid, C);
      tick(5);
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
        // the fixed column against the keygen structure: canonical selectors for round quads
        // (G table), the decoded init/final block otherwise, zero past the last instance
        uint4 xf = make_uint4(in_g ? L[L_XS + (pq & 15u)] : 0u, 0u, 0u, 0u);
        if (!in_g && row0 < used_rows && (MODE & (EVAL_GATES | EVAL_COPIES))) {
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
            const uint32_t lq = (uint32_t)((row0 - o) >> 2);
            if (MODE & EVAL_GATES) {
              const QuadInfo d = decode_quad(lq, rounds);
              xf = fixed_of_quad(d, d.kind == K_CONST ? IV[d.a & 7u] : 0ull);
            }
            if (MODE & EVAL_COPIES) {
              const uint64_t ofirst = first < n ? Off[0] : ~0ull;
              const Src<WSTRIDE> src{L + L_W, L + L_IC, adv, total_rows, tile0 - HIST, ofirst};
              const uint4 dq[3] = {T.quad(A3, lr0), T.quad(A4, lr0), T.quad(A5, lr0)};
              copies_edge(Rec, dq[0], dq[1], dq[2], src, o, rounds, lq);
            }
          }
        }
        if ((MODE & EVAL_GATES) && ((curfx.x ^ xf.x) | (curfx.y ^ xf.y) | (curfx.z ^ xf.z) | (curfx.w ^ xf.w))) {
#pragma unroll
          for (int j = 0; j < 4; j++)
            if (comp(curfx, j) != comp(xf, j)) A.fail(row0 + j, B2F_CODE_FIXED);
        }
      }
    }
    tick(6);
    __syncthreads();
    tick(7);
  }
  if ((MODE & EVAL_CLOCK) && (tid & 63) == 0) {
#pragma unroll
    for (int k = 0; k < 8; k++) atomicAdd(&clk[8 * (tid >> 6) + k], (unsigned long long)ck[k]);
  }
  // ---- flush the workgroup's counters: one global atomic per non-zero counter
  __syncthreads();
  flush_report(A, rep, tid);
}

// Device-side layout validation for b2f_eval_dev: every instance's rows must be R(rounds) for
// some rounds and lie inside the trace. The eval kernel relies on it (an invalid layout is an
// error whatever the counters say; it only has to stay in bounds).
__global__ void offsets_check_kernel(const uint64_t* __restrict__ off, uint32_t n,
                                     uint64_t total_rows, int* __restrict__ status,
                                     int* __restrict__ sticky, b2f_eval_report* __restrict__ rep) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t o = off[i], o1 = off[i + 1], R = o1 - o;
  const bool bad = o1 < o || o1 > total_rows || (i == 0 && o != 0) || R < FIXED_ROWS ||
                   R > MAX_INSTANCE_ROWS || ((uint32_t)R - FIXED_ROWS) % ROUND_ROWS != 0;
  if (bad) raise_error(status, sticky, rep, B2F_ERR_LAYOUT);
}

// Multi-block chaining (Blake2f::update/finalize, blake2f.rs:101-168): the inputs of one block
// step for messages 0 .. n-1 (the host orders messages by block count, so the messages still
// running at a step are a prefix): h from the previous step's outputs, the step's words.
__global__ void chain_inputs_kernel(const uint64_t* __restrict__ h_prev,
                                    const uint64_t* __restrict__ blocks,
                                    const uint64_t* __restrict__ t, const uint32_t* __restrict__ f,
                                    uint32_t rounds, uint32_t n, b2f_input* __restrict__ out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  b2f_input x;
#pragma unroll
  for (int k = 0; k < 8; k++) x.h[k] = h_prev[8ull * i + k];
#pragma unroll
  for (int k = 0; k < 16; k++) x.m[k] = blocks[16ull * i + k];
  x.t[0] = t[2ull * i];
  x.t[1] = t[2ull * i + 1];
  x.rounds = rounds;
  x.f = f[i] ? 1u : 0u;
  out[i] = x;
}

// Keygen structure of the fixed column (b2f_fill_fixed_dev): the selector masks and IV
// constants every row carries by its position in the row map alone (halo2 keygen with
// Value::unknown() witnesses). Thread per quad, one 1024-row tile per
// workgroup, the tile's instance context from TileInfo (scalar loads).
__global__ void __launch_bounds__(BLOCK) fixed_kernel(const uint64_t* __restrict__ off, uint32_t n,
                                                     uint64_t total_rows,
                                                     const TileInfo* __restrict__ tinfo,
                                                     uint32_t* __restrict__ fixed,
                                                     const int* __restrict__ status) {
  if (*status) return;  // offsets_check_kernel rejected the row map: write nothing
  const uint64_t t = blockIdx.x;
  const uint64_t gq = t * BLOCK + threadIdx.x;
  if (gq >= (total_rows >> 2)) return;
  const uint64_t row = 4 * gq;
  const TileInfo ti = tinfo[t];
  uint4 f = make_uint4(0, 0, 0, 0);
  if (row < off[n] && ti.first < n) {
    uint64_t o = ti.off[0], o1 = ti.off[1];
    uint32_t i = 0;
#pragma unroll
    for (int k = 1; k + 1 < NOFF; k++)
      if (ti.off[k] <= row) { o = ti.off[k]; o1 = ti.off[k + 1]; i = (uint32_t)k; }
    if (row >= o && row < o1 && ti.first + i < n) {
      const uint32_t rounds = ((uint32_t)(o1 - o) - FIXED_ROWS) / ROUND_ROWS;
      const QuadInfo d = decode_quad((uint32_t)((row - o) >> 2), rounds);
      f = fixed_of_quad(d, d.kind == K_CONST ? c_iv[d.a & 7u] : 0ull);
    }
  }
  __builtin_nontemporal_store(u32x4{f.x, f.y, f.z, f.w}, reinterpret_cast<u32x4*>(fixed + row));
}

__global__ void report_init_kernel(b2f_eval_report* rep, uint64_t total_rows) {
  for (int s = 0; s < B2F_NUM_GATES; s++) rep->gate_failures[s] = 0;
  rep->lookup_failures = 0;
  rep->copy_failures = 0;
  rep->first_failure = ~0ull;
  rep->rows_checked = total_rows;
  rep->fixed_failures = 0;
}

}  // namespace

// ============================================================================ host / C ABI

struct b2f_ctx {
  int device;
  char err[512];
  int* d_status;       // [0] fill call, [1] eval call, [2] sticky (cleared by b2f_sync only), [3] fill tile counter,
                       // [4] export tile counter
  uint64_t* d_rec;     // half-round states
  uint64_t rec_cap;    // in states (16 x u64 each)
  uint64_t* d_seg;     // the fused launch's segment list (count, entries: instance << 32 | m)
  uint64_t seg_cap;    // in u64 words
  TileInfo* d_tiles;   // per-tile instance context
  uint64_t tiles_cap;
  int timing;
  std::vector<hipEvent_t> pool;  // event pairs, reused after every b2f_kernel_times
  std::vector<int> kinds;        // kernel kind of pair i
  int cu_count;
  unsigned long long* d_clock;  // 32 u64: EVAL_CLOCK phase totals (diagnostics)
  const uint32_t* d_eval_gate;  // the last eval's fast-pass word (0: the fast pass found the trace clean)
  uint64_t inj_row;    // b2f_debug_inject (UINT64_MAX: off)
  uint32_t inj_col, inj_mask;
  void* d_lk;          // lookup-column scratch (b2f_lookup.hip carve)
  size_t lk_cap;
  void* d_fz;          // fused-path scratch: tile descriptors + deferred rows (b2f_fused.hip)
  size_t fz_cap;
  // permutation columns (b2f_perm.hip): keygen mapping patterns per rounds (host cache and
  // the device pool holding them), the per-call instance table, scratch
  std::map<uint32_t, std::vector<uint32_t>> pm_pat;
  std::map<uint32_t, uint64_t> pm_pool_off;  // rounds -> offset in d_pm_pool (u32 units)
  uint32_t* d_pm_pool;
  uint64_t* h_pm_inst;     // pinned staging of the per-call instance table
  size_t h_pm_inst_cap;
  hipEvent_t pm_inst_ev;   // recorded after the table's async upload (the staging is reusable
  bool pm_inst_ev_live;    // once it completes)
  uint64_t* d_pm_inst;
  size_t pm_inst_cap;
  void* d_pm;
  size_t pm_cap;
  // a second stream and two events: the grand products' inversions run beside their block
  // down-sweep (b2f_gprod.h), forked from and joined back to the caller's stream
  hipStream_t s2;
  hipEvent_t ev_fork, ev_join;
  hipStream_t s3;                // the lookup's table pass and sort (beside the count pass)
  hipEvent_t ev_tab, ev_sorted;
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

// Diagnostic kernel variants for ablation runs (B2F_DIAG_FILL / B2F_DIAG_EVAL /
// B2F_DIAG_FUSED / B2F_FILL_WGS / B2F_BAND) exist only in the diagnostics library
// (libb2f_diag.so, built with -DB2F_DIAG). The product library (libb2f.so) reads no environment
// and always launches the full kernels.
#ifdef B2F_DIAG
int diag_mode(const char* var, int full) {
  const char* v = getenv(var);
  return v ? atoi(v) : full;
}
// B2F_DIAG_FUSED: only the product variant (27) and the diagnostic ones that skip every check
// (0, 2, 3, 10, 18, 8, 16, 34, 66, 98) are accepted; anything else runs the product kernel.
int fused_mode() {
  const int m = diag_mode("B2F_DIAG_FUSED", 27);
  const bool safe = m == 27 || m == (27 | 128) || m == 130 || m == 128 ||
                    ((m & ~(1 | 2 | 8 | 16)) == 0);
  return safe ? m : 27;
}
#else
constexpr int diag_mode(const char*, int full) { return full; }
constexpr int fused_mode() { return 27; }
#endif

// the side stream and events of the grand products (created on first use)
int ensure_side(b2f_ctx* ctx) {
  if (!ctx->s2) HIPCHK(ctx, hipStreamCreateWithFlags(&ctx->s2, hipStreamNonBlocking));
  if (!ctx->ev_fork) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
  if (!ctx->ev_join) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
  if (!ctx->s3) HIPCHK(ctx, hipStreamCreateWithFlags(&ctx->s3, hipStreamNonBlocking));
  if (!ctx->ev_tab) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->ev_tab, hipEventDisableTiming));
  if (!ctx->ev_sorted) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->ev_sorted, hipEventDisableTiming));
  return B2F_OK;
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
                      hipStream_t s, uint32_t shift = 0) {
  if (n_tiles > ctx->tiles_cap) {
    HIPCHK(ctx, hipStreamSynchronize(s));
    if (ctx->d_tiles) HIPCHK(ctx, hipFree(ctx->d_tiles));
    ctx->d_tiles = nullptr;
    ctx->tiles_cap = 0;
    HIPCHK(ctx, hipMalloc(&ctx->d_tiles, n_tiles * sizeof(TileInfo)));
    ctx->tiles_cap = n_tiles;
  }
  hipLaunchKernelGGL(tile_info_kernel, dim3((uint32_t)((n_tiles + 255) / 256)), dim3(256), 0, s,
                     d_offsets, (uint32_t)n, n_tiles, shift, ctx->d_tiles);
  HIPCHK(ctx, hipGetLastError());
  return B2F_OK;
}

// The copy constraints of one instance (LAYOUT.md §4/§5), in synthesis order: the init XOR
// operands, then per round and G the operand cells of its eight blocks (the device check
// tables' DescTable, make_desc), then the final XOR3 operands. Each is (dst_row, dst_col,
// src_row, src_col), rows relative to the instance. Host code, no device work.
uint64_t copy_constraints(uint32_t rounds, uint32_t* out4, uint64_t cap) {
  uint64_t cnt = 0;
  auto put = [&](uint32_t dr, uint32_t dc, uint32_t sr, uint32_t sc) {
    if (out4 && cnt < cap) {
      uint32_t* q = out4 + 4 * cnt;
      q[0] = dr; q[1] = dc; q[2] = sr; q[3] = sc;
    }
    cnt++;
  };
  // v12 = IV4 ^ t0, v13 = IV5 ^ t1, v14 = IV6 ^ fmask (XOR blocks at 140 + 8a)
  for (uint32_t a = 0; a < 3; a++)
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t dr = 140 + 8 * a + 2 * k;
      put(dr, A3, 108 + 4 * (4 + a) + k, A2);
      put(dr, A4, (a < 2 ? 96 + 4 * a : 104) + k, A2);
    }
  constexpr DescTable D = make_desc();
  constexpr SigmaPairs SP = make_sigma_pairs();
  for (uint32_t r = 0; r < rounds; r++)
    for (uint32_t g = 0; g < 8; g++) {
      const uint32_t gb = INIT_ROWS + ROUND_ROWS * r + G_ROWS * g;
      const uint32_t hr = 2 * r + (g >= 4 ? 1u : 0u);
      for (uint32_t p = 0; p < G_QUADS; p++)
        for (uint32_t j = 0; j < 4; j++)
          for (uint32_t c = 0; c < 3; c++) {
            const uint32_t d = D.d[p][j][c], kind = d & 3u;
            if (!kind) continue;
            const uint32_t dr = gb + 4 * p + j, dc = A3 + c;
            if (kind == 1) {
              put(dr, dc, gb + ((d >> 2) & 63u), (d >> 8) & 15u);
            } else if (kind == 2) {
              uint32_t col = 0;
              const uint32_t w = kGidx[g][(d >> 2) & 3u];
              const uint32_t sr = state_src(w, (d >> 4) & 3u, (d >> 6) & 1u, hr, col);
              put(dr, dc, sr, col);
            } else {
              const uint32_t pair = SP.v[r % 10][g];
              const uint32_t mw = ((d >> 2) & 1u) ? pair >> 8 : pair & 0xffu;
              put(dr, dc, 32 + 4 * mw + ((d >> 4) & 3u), A1);
            }
          }
    }
  // h'_i = h_i ^ v_i ^ v_{i+8} (XOR3 blocks at 164 + 416 rounds + 8i)
  for (uint32_t i = 0; i < 8; i++)
    for (uint32_t k = 0; k < 4; k++) {
      const uint32_t dr = INIT_ROWS + ROUND_ROWS * rounds + 8 * i + 2 * k;
      uint32_t cv = 0, cu = 0;
      const uint32_t vs = state_src(i, k, 1, 2 * rounds, cv);
      const uint32_t us = state_src(i + 8, k, 1, 2 * rounds, cu);
      put(dr, A3, 4 * i + k, A2);
      put(dr, A4, vs, cv);
      put(dr, A5, us, cu);
    }
  return cnt;
}

// Keygen's permutation mapping of one instance (halo2_proofs 0.3.0 plonk/permutation/keygen.rs
// Assembly::copy): the instance's copy constraints replayed in synthesis order, each as
// copy(left = the copy's destination cell, right = its source) -- AssignedCell::copy_advice
// assigns the new cell, then constrain_equal(new, self). Cycles merge smaller-into-larger:
// every cell of the right cycle is re-pointed to the left cycle's representative and the two
// cells' mapping entries are swapped. Permutation column j is a_{j+1} (enable_equality order,
// table16.rs:312-314). Output: out[j * R + i] = (c' << 29) | r', the cell (c', r') that cell
// (j, i) maps to.
constexpr int PM_COLS = 8;
bool perm_mapping(uint32_t rounds, std::vector<uint32_t>& out) {
  const uint64_t R = layout_rows(rounds);
  if (!R) return false;
  const uint64_t ncp = copy_constraints(rounds, nullptr, 0);
  std::vector<uint32_t> cp(4 * ncp);
  copy_constraints(rounds, cp.data(), ncp);
  const uint64_t cells = PM_COLS * R;
  std::vector<uint32_t> mapping(cells), aux(cells), sizes(cells, 1);
  for (uint64_t x = 0; x < cells; x++) mapping[x] = aux[x] = (uint32_t)x;  // x = j * R + i
  for (uint64_t q = 0; q < ncp; q++) {
    const uint32_t dr = cp[4 * q], dc = cp[4 * q + 1], sr = cp[4 * q + 2], sc = cp[4 * q + 3];
    if (dc < 1 || dc > 8 || sc < 1 || sc > 8) return false;  // only a_1..a_8 take part
    const uint32_t left = (dc - 1) * (uint32_t)R + dr, right = (sc - 1) * (uint32_t)R + sr;
    uint32_t lc = aux[left], rc = aux[right];
    if (lc == rc) continue;
    if (sizes[lc] < sizes[rc]) std::swap(lc, rc);
    sizes[lc] += sizes[rc];
    uint32_t i = rc;
    do {
      aux[i] = lc;
      i = mapping[i];
    } while (i != rc);
    std::swap(mapping[left], mapping[right]);
  }
  out.resize(cells);
  for (uint64_t x = 0; x < cells; x++)
    out[x] = ((mapping[x] / (uint32_t)R) << 29) | (mapping[x] % (uint32_t)R);
  return true;
}

}  // namespace

extern "C" {

B2F_API int b2f_version(void) { return 2; }  // 2: fixed_failures, sticky errors, keygen calls

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
  ctx->inj_row = ~0ull;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) { delete ctx; return nullptr; }
  ctx->cu_count = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  if (hipMalloc(&ctx->d_status, 8 * sizeof(int)) != hipSuccess) { delete ctx; return nullptr; }
  // the sticky word must read 0 before the first call: a blocking memset on the null stream
  if (hipMemset(ctx->d_status, 0, 8 * sizeof(int)) != hipSuccess) { delete ctx; return nullptr; }
  return ctx;
}

B2F_API void b2f_destroy(b2f_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipFree(ctx->d_status);
  (void)hipFree(ctx->d_rec);
  (void)hipFree(ctx->d_seg);
  (void)hipFree(ctx->d_tiles);
  (void)hipFree(ctx->d_clock);
  (void)hipFree(ctx->d_lk);
  (void)hipFree(ctx->d_fz);
  (void)hipFree(ctx->d_pm_pool);
  (void)hipFree(ctx->d_pm_inst);
  (void)hipFree(ctx->d_pm);
  if (ctx->pm_inst_ev_live) (void)hipEventSynchronize(ctx->pm_inst_ev);
  if (ctx->pm_inst_ev) (void)hipEventDestroy(ctx->pm_inst_ev);
  if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
  if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
  if (ctx->s2) (void)hipStreamDestroy(ctx->s2);
  if (ctx->ev_tab) (void)hipEventDestroy(ctx->ev_tab);
  if (ctx->ev_sorted) (void)hipEventDestroy(ctx->ev_sorted);
  if (ctx->s3) (void)hipStreamDestroy(ctx->s3);
  (void)hipHostFree(ctx->h_pm_inst);
  for (hipEvent_t e : ctx->pool) (void)hipEventDestroy(e);
  delete ctx;
}

B2F_API const char* b2f_last_error(const b2f_ctx* ctx) { return ctx ? ctx->err : "null context"; }

B2F_API int b2f_num_kernels(void) { return B2F_NUM_KERNELS; }

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

}  // extern "C"

namespace {
// Entries of the fused launch's segment list. Diagnostics build only: B2F_DIAG_SEG_CAP caps it
// below what the batch needs, so a test sees the overflow raise B2F_ERR_CHECK.
uint64_t seg_entries(const b2f_ctx* ctx) {
  const uint64_t cap = ctx->seg_cap ? ctx->seg_cap - 1 : 0;
  const int lim = diag_mode("B2F_DIAG_SEG_CAP", -1);
  return lim >= 0 && (uint64_t)lim < cap ? (uint64_t)lim : cap;
}

// Argument checks, record scratch and the record kernel: the first part of b2f_fill_dev and
// b2f_fill_eval_dev.
int fill_prologue(b2f_ctx* ctx, const b2f_input* d_in, size_t n, const uint64_t* d_offsets,
                  uint64_t total_rows, uint32_t* d_advice, uint32_t* d_fixed, uint64_t* d_h_out,
                  b2f_eval_report* d_report, hipStream_t s, bool lite = false) {
  if (!d_in || !d_offsets || !d_advice || !d_fixed || n == 0)
    return set_err(ctx, B2F_ERR_ARG, "fill: null buffer or empty batch");
  if (n > 0xffffffffull) return set_err(ctx, B2F_ERR_ARG, "fill: more than 2^32 instances");
  if (total_rows % 4) return set_err(ctx, B2F_ERR_ARG, "fill: total_rows %% 4 != 0");
  if (((uintptr_t)d_advice | (uintptr_t)d_fixed | (uintptr_t)d_in) & 15)
    return set_err(ctx, B2F_ERR_ARG, "fill: buffers must be 16-byte aligned");
  if (total_rows < (uint64_t)FIXED_ROWS * n)
    return set_err(ctx, B2F_ERR_ROWS, "fill: %llu rows cannot hold %zu instances",
                   (unsigned long long)total_rows, n);
  HIPCHK(ctx, hipSetDevice(ctx->device));
  // states = 2*sum(rounds) + n  <=  2*(total_rows - 228 n)/416 + n
  uint64_t states = 2 * ((total_rows - (uint64_t)FIXED_ROWS * n) / ROUND_ROWS) + n;
  if (states >= (1ull << 32))
    return set_err(ctx, B2F_ERR_ROWS, "fill: %llu rows exceed the 2^32 half-round states of one call",
                   (unsigned long long)total_rows);
  if (states > ctx->rec_cap) {
    HIPCHK(ctx, hipStreamSynchronize(s));
    if (ctx->d_rec) HIPCHK(ctx, hipFree(ctx->d_rec));
    ctx->d_rec = nullptr;
    ctx->rec_cap = 0;
    HIPCHK(ctx, hipMalloc(&ctx->d_rec, states * 16 * sizeof(uint64_t)));
    ctx->rec_cap = states;
  }
  HIPCHK(ctx, hipMemsetAsync(ctx->d_status, 0, sizeof(int), s));
  if (d_report) {  // before the record kernel, which marks the report of a rejected batch
    hipLaunchKernelGGL(report_init_kernel, dim3(1), dim3(1), 0, s, d_report, total_rows);
    HIPCHK(ctx, hipGetLastError());
  }
  uint32_t nn = (uint32_t)n;
  int tk = timed_begin(ctx, B2F_KERNEL_RECORD, s);
  uint64_t* seg = nullptr;
  if (lite) {  // the fused launch's segment list: count, then at most states / SEG_HR entries
    const uint64_t cap = states / SEG_HR + 1;
    if (cap + 1 > ctx->seg_cap) {
      HIPCHK(ctx, hipStreamSynchronize(s));
      if (ctx->d_seg) HIPCHK(ctx, hipFree(ctx->d_seg));
      ctx->d_seg = nullptr;
      ctx->seg_cap = 0;
      HIPCHK(ctx, hipMalloc(&ctx->d_seg, (cap + 1) * sizeof(uint64_t)));
      ctx->seg_cap = cap + 1;
    }
    seg = ctx->d_seg;
    HIPCHK(ctx, hipMemsetAsync(seg, 0, sizeof(uint64_t), s));
  }
  hipLaunchKernelGGL(record_kernel, dim3((uint32_t)((4ull * nn + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, d_in, nn,
                     d_offsets, total_rows, ctx->rec_cap, ctx->d_rec, d_h_out, ctx->d_status,
                     ctx->d_status + 2, d_report, lite, seg, lite ? seg_entries(ctx) : 0);
  HIPCHK(ctx, hipGetLastError());
  timed_end(ctx, tk, s);
  return B2F_OK;
}
}  // namespace

extern "C" {

B2F_API int b2f_fill_dev(b2f_ctx* ctx, const b2f_input* d_in, size_t n, const uint64_t* d_offsets,
                         uint64_t total_rows, uint32_t* d_advice, uint32_t* d_fixed,
                         uint64_t* d_h_out, void* stream) {
  if (!ctx) return B2F_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  int rc = fill_prologue(ctx, d_in, n, d_offsets, total_rows, d_advice, d_fixed, d_h_out, nullptr, s);
  if (rc) return rc;
  const uint32_t nn = (uint32_t)n;
  uint64_t nt = n_tiles_of(total_rows);
  rc = launch_tile_index(ctx, d_offsets, n, nt, s);
  if (rc) return rc;
  uint32_t wgs = grid_for(ctx, nt, diag_mode("B2F_FILL_WGS", 8));
  int tk = timed_begin(ctx, B2F_KERNEL_FILL, s);
#ifdef B2F_DIAG
  if (diag_mode("B2F_DIAG_FILL", FILL_FULL) == 4) {
    hipLaunchKernelGGL(store_stream_kernel, dim3(ctx->cu_count * 8), dim3(BLOCK), 0, s, d_advice, d_fixed,
                       total_rows);
    HIPCHK(ctx, hipGetLastError());
    timed_end(ctx, tk, s);
    return B2F_OK;
  }
#endif
  const int fmode = diag_mode("B2F_DIAG_FILL", FILL_FULL);
  if ((fmode & FILL_CLOCK) && !ctx->d_clock) {
    HIPCHK(ctx, hipMalloc(&ctx->d_clock, 32 * sizeof(unsigned long long)));
    HIPCHK(ctx, hipMemset(ctx->d_clock, 0, 32 * sizeof(unsigned long long)));
  }
  // the tile counter of B2F_FILL_DYN: the fourth status word
  unsigned* tctr = reinterpret_cast<unsigned*>(ctx->d_status + 3);
  HIPCHK(ctx, hipMemsetAsync(tctr, 0, sizeof(unsigned), s));
  switch (fmode) {
#define B2F_FILL(M)                                                                            \
  case M:                                                                                      \
    hipLaunchKernelGGL(fill_kernel<M>, dim3(wgs), dim3(BLOCK), 0, s, d_in, nn, d_offsets,      \
                       total_rows, ctx->d_rec, d_advice, d_fixed, ctx->d_status, ctx->d_tiles, \
                       nt, ctx->d_clock, tctr);                                                \
    break;
#ifdef B2F_DIAG
    B2F_FILL(0) B2F_FILL(1) B2F_FILL(2) B2F_FILL(FILL_FULL | FILL_CLOCK)
#endif
    default: B2F_FILL(3)
#undef B2F_FILL
  }
  HIPCHK(ctx, hipGetLastError());
  timed_end(ctx, tk, s);
  return B2F_OK;
}

// The fused path's scratch (tile descriptors, deferred rows, redo list, the eval's dirty word),
// grown on demand.
static int ensure_fused_scratch(b2f_ctx* ctx, size_t need, hipStream_t s) {
  if (need > ctx->fz_cap) {
    HIPCHK(ctx, hipStreamSynchronize(s));
    if (ctx->d_fz) HIPCHK(ctx, hipFree(ctx->d_fz));
    ctx->d_fz = nullptr;
    ctx->fz_cap = 0;
    HIPCHK(ctx, hipMalloc(&ctx->d_fz, need));
    ctx->fz_cap = need;
  }
  return B2F_OK;
}

B2F_API int b2f_fill_eval_dev(b2f_ctx* ctx, const b2f_input* d_in, size_t n,
                              const uint64_t* d_offsets, uint64_t total_rows, uint32_t* d_advice,
                              uint32_t* d_fixed, uint64_t* d_h_out, b2f_eval_report* d_report,
                              void* stream) {
  if (!ctx) return B2F_ERR_ARG;
  if (!d_report) return set_err(ctx, B2F_ERR_ARG, "fill_eval: null report");
  hipStream_t s = (hipStream_t)stream;
  // lite record: the half-round launch carries the state from tile to tile; only the edge launch
  // reads recorded states (the last two of each instance)
  int rc = fill_prologue(ctx, d_in, n, d_offsets, total_rows, d_advice, d_fixed, d_h_out, d_report, s, true);
  if (rc) return rc;
  const uint64_t tiles = fused_instance_tiles(total_rows, n);
  rc = ensure_fused_scratch(ctx, fused_scratch_bytes(tiles), s);
  if (rc) return rc;
  const int fmode = fused_mode();
  if ((fmode & 128) && !ctx->d_clock) {
    HIPCHK(ctx, hipMalloc(&ctx->d_clock, 32 * sizeof(unsigned long long)));
    HIPCHK(ctx, hipMemset(ctx->d_clock, 0, 32 * sizeof(unsigned long long)));
  }
  const int tk = timed_begin(ctx, B2F_KERNEL_FILL_EVAL, s);
  HIPCHK(ctx, launch_fill_eval(d_in, (uint32_t)n, d_offsets, total_rows, ctx->d_rec, d_advice,
                               d_fixed, ctx->d_fz, tiles, d_report, ctx->d_status,
                               ctx->inj_row, ctx->inj_col, ctx->inj_mask, fmode,
                               ctx->cu_count, ctx->d_clock, ctx->d_seg, seg_entries(ctx), s));
  timed_end(ctx, tk, s);
  return B2F_OK;
}

B2F_API int b2f_debug_clock(b2f_ctx* ctx, uint64_t* out) {
  if (!ctx || !out) return B2F_ERR_ARG;
  for (int i = 0; i < 32; i++) out[i] = 0;
  if (!ctx->d_clock) return B2F_OK;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipDeviceSynchronize());
  HIPCHK(ctx, hipMemcpy(out, ctx->d_clock, 32 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  HIPCHK(ctx, hipMemset(ctx->d_clock, 0, 32 * sizeof(uint64_t)));
  return B2F_OK;
}

B2F_API int b2f_debug_eval_path(b2f_ctx* ctx, uint32_t* out) {
  if (!ctx || !out) return B2F_ERR_ARG;
  *out = 2;
  if (!ctx->d_eval_gate) return B2F_OK;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipDeviceSynchronize());
  uint32_t w = 0;
  HIPCHK(ctx, hipMemcpy(&w, ctx->d_eval_gate, sizeof w, hipMemcpyDeviceToHost));
  *out = w ? 1u : 0u;
  return B2F_OK;
}

B2F_API int b2f_debug_inject(b2f_ctx* ctx, uint64_t row, uint32_t col, uint32_t mask) {
  if (!ctx) return B2F_ERR_ARG;
  if (row != UINT64_MAX && col > B2F_NUM_ADVICE)
    return set_err(ctx, B2F_ERR_ARG, "inject: column %u (0..9 advice, 10 fixed)", col);
  ctx->inj_row = row;
  ctx->inj_col = col;
  ctx->inj_mask = mask;
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
                     d_offsets, (uint32_t)n, total_rows, ctx->d_status + 1, ctx->d_status + 2,
                     d_report);
  HIPCHK(ctx, hipGetLastError());
  uint64_t nt = n_tiles_of(total_rows);
  int rc = launch_tile_index(ctx, d_offsets, n, nt, s);
  if (rc) return rc;
  uint32_t wgs = grid_for(ctx, (nt + EVAL_BAND - 1) / EVAL_BAND, 3);
  const int emode = diag_mode("B2F_DIAG_EVAL", EVAL_FULL);
  if ((emode & EVAL_CLOCK) && !ctx->d_clock) {
    HIPCHK(ctx, hipMalloc(&ctx->d_clock, 32 * sizeof(unsigned long long)));
    HIPCHK(ctx, hipMemset(ctx->d_clock, 0, 32 * sizeof(unsigned long long)));
  }
  // the product path: the fast clean-check pass first; the exact eval kernel runs only if it
  // flagged something (device-side gate). Diagnostic modes run the exact kernel alone.
  const uint32_t* gate = nullptr;
  // (diagnostics: B2F_DIAG_EVALFAST = the fast pass's check mode, the exact kernel then skipped)
  const int fmode = diag_mode("B2F_DIAG_EVALFAST", 27);
  const bool fast = (emode == EVAL_FULL || fmode != 27) && total_rows >= (uint64_t)FIXED_ROWS * n;
  if (fast) {
    rc = ensure_fused_scratch(ctx, fused_scratch_bytes(fused_instance_tiles(total_rows, n)), s);
    if (rc) return rc;
  }
  int tk = timed_begin(ctx, B2F_KERNEL_EVAL, s);
#ifdef B2F_DIAG
  if (emode == EVAL_STREAM) {  // the read floor alone (the spare eighth status word as its sink)
    hipLaunchKernelGGL(load_stream_kernel, dim3(ctx->cu_count * 8), dim3(BLOCK), 0, s, d_advice, d_fixed,
                       total_rows, ctx->d_status + 7);
    HIPCHK(ctx, hipGetLastError());
    timed_end(ctx, tk, s);
    return B2F_OK;
  }
#endif
  if (fast)
    HIPCHK(ctx, launch_eval_fast(d_advice, d_fixed, d_offsets, (uint32_t)n, total_rows, ctx->d_fz,
                                 fused_instance_tiles(total_rows, n), ctx->d_status + 1, ctx->cu_count, s, &gate,
                                 fmode));
  ctx->d_eval_gate = gate;
  if (fmode != 27) {  // diagnostics: the fast pass alone
    timed_end(ctx, tk, s);
    return B2F_OK;
  }
  switch (emode) {
#define B2F_EVAL(M)                                                                             \
  case M:                                                                                       \
    hipLaunchKernelGGL(eval_kernel<M>, dim3(wgs), dim3(BLOCK), 0, s, d_advice, d_fixed,         \
                       d_offsets, (uint32_t)n, total_rows, ctx->d_tiles, nt, d_report,          \
                       ctx->d_status + 1, ctx->d_status + 2, ctx->d_clock, gate);               \
    break;
#ifdef B2F_DIAG
    B2F_EVAL(1) B2F_EVAL(2) B2F_EVAL(3) B2F_EVAL(4) B2F_EVAL(5) B2F_EVAL(6) B2F_EVAL(8)
    B2F_EVAL(EVAL_FULL | EVAL_CLOCK)
#endif
    default: B2F_EVAL(7)
#undef B2F_EVAL
  }
  HIPCHK(ctx, hipGetLastError());
  timed_end(ctx, tk, s);
  return B2F_OK;
}

B2F_API int b2f_chain_inputs_dev(b2f_ctx* ctx, const uint64_t* d_h_prev, const uint64_t* d_blocks,
                                 const uint64_t* d_t, const uint32_t* d_f, uint32_t rounds,
                                 size_t n, b2f_input* d_out, void* stream) {
  if (!ctx) return B2F_ERR_ARG;
  if (!d_h_prev || !d_blocks || !d_t || !d_f || !d_out)
    return set_err(ctx, B2F_ERR_ARG, "chain: null buffer");
  if (rounds > B2F_MAX_ROUNDS) return set_err(ctx, B2F_ERR_ROUNDS, "chain: rounds > %u", B2F_MAX_ROUNDS);
  if (n > 0xffffffffull) return set_err(ctx, B2F_ERR_ARG, "chain: more than 2^32 messages");
  if (n == 0) return B2F_OK;
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  hipLaunchKernelGGL(chain_inputs_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, d_h_prev,
                     d_blocks, d_t, d_f, rounds, (uint32_t)n, d_out);
  HIPCHK(ctx, hipGetLastError());
  return B2F_OK;
}

B2F_API int b2f_export_fp_dev(b2f_ctx* ctx, const uint32_t* d_advice, uint64_t total_rows,
                              uint64_t row_begin, uint64_t nrows, uint32_t form,
                              uint64_t* d_out, uint64_t out_rows, void* stream) {
  if (!ctx) return B2F_ERR_ARG;
  if (!d_advice || !d_out) return set_err(ctx, B2F_ERR_ARG, "export: null buffer");
  if (form > B2F_FP_BN254_MONTGOMERY) return set_err(ctx, B2F_ERR_ARG, "export: unknown form %u", form);
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
                               ctx->cu_count, reinterpret_cast<unsigned*>(ctx->d_status + 4), s));
  timed_end(ctx, tk, s);
  return B2F_OK;
}

B2F_API int b2f_lookup_columns_dev(b2f_ctx* ctx, const uint32_t* d_advice, uint64_t total_rows,
                                   const uint64_t* d_row_begin, uint32_t n_circuits,
                                   uint64_t usable_rows, const uint64_t theta[4],
                                   const uint64_t beta[4], const uint64_t gamma[4], uint32_t form,
                                   uint64_t* d_out, uint64_t out_rows, uint64_t* d_first_bad,
                                   void* stream) {
  if (!ctx) return B2F_ERR_ARG;
  if (!d_advice || !d_row_begin || !theta || !beta || !gamma || !d_out || !d_first_bad)
    return set_err(ctx, B2F_ERR_ARG, "lookup: null buffer");
  if (form > B2F_FP_BN254_MONTGOMERY) return set_err(ctx, B2F_ERR_ARG, "lookup: unknown form %u", form);
  if ((uintptr_t)d_out & 15) return set_err(ctx, B2F_ERR_ARG, "lookup: d_out must be 16-byte aligned");
  if (usable_rows < (1ull << 16) || usable_rows > (1ull << 31))
    return set_err(ctx, B2F_ERR_ROWS, "lookup: usable_rows %llu not in [2^16, 2^31]",
                   (unsigned long long)usable_rows);
  if (out_rows < usable_rows + 1)
    return set_err(ctx, B2F_ERR_ROWS, "lookup: out_rows < usable_rows + 1");
  auto canon = [form](const uint64_t* v) {  // < the field's modulus
    static const uint64_t moduli[2][4] = {
        {0x992d30ed00000001ull, 0x224698fc094cf91bull, 0, 0x4000000000000000ull},  // pasta Fp
        {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull,
         0x30644e72e131a029ull}};  // BN254 Fr
    const uint64_t* p = moduli[form >> 1];
    for (int i = 3; i >= 0; i--)
      if (v[i] != p[i]) return v[i] < p[i];
    return false;
  };
  if (!canon(theta) || !canon(beta) || !canon(gamma))
    return set_err(ctx, B2F_ERR_ARG, "lookup: challenge not a canonical field element");
  if (n_circuits == 0) return B2F_OK;
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  // circuits per pass: at most 2^24 rows (128 circuits of 2^17), enough workgroups to fill
  // the chip several times over; per-circuit scratch is 1.1 MiB (count, pos, D, LP, samples) +
  // 224 B per 1,024-row block (num products, prefixes, look-back state)
  uint32_t group = (uint32_t)((1ull << 24) / usable_rows);
  if (group < 1) group = 1;
  if (group > n_circuits) group = n_circuits;
  const size_t need = lookup_scratch_bytes(group, usable_rows);
  if (need > ctx->lk_cap) {
    HIPCHK(ctx, hipStreamSynchronize(s));
    if (ctx->d_lk) HIPCHK(ctx, hipFree(ctx->d_lk));
    ctx->d_lk = nullptr;
    ctx->lk_cap = 0;
    HIPCHK(ctx, hipMalloc(&ctx->d_lk, need));
    ctx->lk_cap = need;
  }
  if (int rc = ensure_side(ctx)) return rc;
  int tk = timed_begin(ctx, B2F_KERNEL_LOOKUP, s);
  HIPCHK(ctx, launch_lookup(d_advice, total_rows, d_row_begin, n_circuits, usable_rows, theta, beta,
                            gamma, form, d_out, out_rows, d_first_bad, ctx->d_lk, group,
                            ctx->d_status + 2, ctx->s2, ctx->ev_fork, ctx->ev_join, ctx->s3,
                            ctx->ev_tab, ctx->ev_sorted, s));
  timed_end(ctx, tk, s);
  return B2F_OK;
}

B2F_API int b2f_spread_table_dev(b2f_ctx* ctx, uint64_t usable_rows, uint32_t form, uint64_t* d_out,
                                 uint64_t out_rows, void* stream) {
  if (!ctx) return B2F_ERR_ARG;
  if (!d_out || ((uintptr_t)d_out & 15)) return set_err(ctx, B2F_ERR_ARG, "spread table: d_out null or unaligned");
  if (form > B2F_FP_BN254_MONTGOMERY) return set_err(ctx, B2F_ERR_ARG, "spread table: unknown form %u", form);
  if (usable_rows < (1ull << 16) || usable_rows >= (1ull << 32) || out_rows < usable_rows)
    return set_err(ctx, B2F_ERR_ROWS, "spread table: need 2^16 <= usable_rows < 2^32, out_rows >= usable_rows");
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  int tk = timed_begin(ctx, B2F_KERNEL_EXPORT, s);
  HIPCHK(ctx, launch_spread_table(usable_rows, form, d_out, out_rows, s));
  timed_end(ctx, tk, s);
  return B2F_OK;
}

B2F_API uint64_t b2f_permutation_mapping(uint32_t rounds, uint32_t* out, uint64_t cap) {
  std::vector<uint32_t> m;
  if (!perm_mapping(rounds, m)) return 0;
  if (out) memcpy(out, m.data(), 4 * (m.size() < cap ? m.size() : cap));
  return m.size();
}

}  // extern "C"

namespace {
// The host part shared by the permutation calls: field checks, the instance row map, the mapping
// patterns (built once per rounds, pooled on the device), the instance table (pinned staging,
// async upload) and the scratch (need_scr bytes). *row0 / *used: the circuit's first trace row
// and its rows. Whatever the caller launches next is stream-ordered after the table upload.
int perm_setup(b2f_ctx* ctx, const char* what, const uint64_t* h_offsets, size_t n, uint32_t k,
               uint32_t form, const uint64_t* const* elems, int n_elems, size_t need_scr,
               hipStream_t s, uint64_t* row0, uint64_t* used) {
  if (form > B2F_FP_BN254_MONTGOMERY) return set_err(ctx, B2F_ERR_ARG, "%s: unknown form %u", what, form);
  if (k < 10 || k > 30) return set_err(ctx, B2F_ERR_ARG, "%s: k %u not in [10, 30]", what, k);
  static const uint64_t moduli[2][4] = {
      {0x992d30ed00000001ull, 0x224698fc094cf91bull, 0, 0x4000000000000000ull},
      {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull, 0x30644e72e131a029ull}};
  auto canon = [&](const uint64_t* v) {
    const uint64_t* p = moduli[form >> 1];
    for (int i = 3; i >= 0; i--)
      if (v[i] != p[i]) return v[i] < p[i];
    return false;
  };
  for (int i = 0; i < n_elems; i++)
    if (!canon(elems[i])) return set_err(ctx, B2F_ERR_ARG, "%s: omega/delta/beta/gamma not canonical field elements", what);
  *row0 = h_offsets[0];
  std::vector<uint32_t> need;
  for (size_t i = 0; i < n; i++) {
    const uint64_t R = h_offsets[i + 1] - h_offsets[i];
    if (h_offsets[i + 1] < h_offsets[i] || R < FIXED_ROWS || (R - FIXED_ROWS) % ROUND_ROWS ||
        (R - FIXED_ROWS) / ROUND_ROWS > B2F_MAX_ROUNDS)
      return set_err(ctx, B2F_ERR_LAYOUT, "%s: offsets[%zu..%zu] is not an instance", what, i, i + 1);
    need.push_back((uint32_t)((R - FIXED_ROWS) / ROUND_ROWS));
  }
  *used = h_offsets[n] - *row0;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  // mapping patterns: build the missing ones, rebuild the device pool if it lacks any
  bool rebuild = false;
  for (uint32_t r : need) {
    if (!ctx->pm_pat.count(r)) {
      std::vector<uint32_t> m;
      if (!perm_mapping(r, m)) return set_err(ctx, B2F_ERR_ROUNDS, "%s: rounds %u", what, r);
      ctx->pm_pat[r] = std::move(m);
    }
    if (!ctx->pm_pool_off.count(r)) rebuild = true;
  }
  if (rebuild) {
    std::vector<uint32_t> pool;
    ctx->pm_pool_off.clear();
    for (auto& kv : ctx->pm_pat) {
      ctx->pm_pool_off[kv.first] = pool.size();
      pool.insert(pool.end(), kv.second.begin(), kv.second.end());
    }
    HIPCHK(ctx, hipStreamSynchronize(s));
    if (ctx->d_pm_pool) HIPCHK(ctx, hipFree(ctx->d_pm_pool));
    ctx->d_pm_pool = nullptr;
    HIPCHK(ctx, hipMalloc(&ctx->d_pm_pool, 4 * pool.size()));
    HIPCHK(ctx, hipMemcpy(ctx->d_pm_pool, pool.data(), 4 * pool.size(), hipMemcpyHostToDevice));
  }
  // instance table: n + 1 circuit start rows, then n pool offsets, staged in pinned host
  // memory and uploaded asynchronously; the host waits only for the previous call's upload
  // (so the staging can be rewritten), or for the whole stream when a device buffer grows
  const size_t m = 2 * n + 1;
  if (ctx->pm_inst_ev_live) {
    HIPCHK(ctx, hipEventSynchronize(ctx->pm_inst_ev));
    ctx->pm_inst_ev_live = false;
  }
  if (m > ctx->h_pm_inst_cap) {
    if (ctx->h_pm_inst) HIPCHK(ctx, hipHostFree(ctx->h_pm_inst));
    ctx->h_pm_inst = nullptr;
    ctx->h_pm_inst_cap = 0;
    HIPCHK(ctx, hipHostMalloc((void**)&ctx->h_pm_inst, 8 * m, hipHostMallocDefault));
    ctx->h_pm_inst_cap = m;
  }
  if (!ctx->pm_inst_ev) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->pm_inst_ev, hipEventDisableTiming));
  uint64_t* it = ctx->h_pm_inst;
  for (size_t i = 0; i <= n; i++) it[i] = h_offsets[i] - *row0;
  for (size_t i = 0; i < n; i++) it[n + 1 + i] = ctx->pm_pool_off[need[i]];
  if (m > ctx->pm_inst_cap || need_scr > ctx->pm_cap) {
    HIPCHK(ctx, hipStreamSynchronize(s));
    if (m > ctx->pm_inst_cap) {
      if (ctx->d_pm_inst) HIPCHK(ctx, hipFree(ctx->d_pm_inst));
      ctx->d_pm_inst = nullptr;
      ctx->pm_inst_cap = 0;
      HIPCHK(ctx, hipMalloc(&ctx->d_pm_inst, 8 * m));
      ctx->pm_inst_cap = m;
    }
    if (need_scr > ctx->pm_cap) {
      if (ctx->d_pm) HIPCHK(ctx, hipFree(ctx->d_pm));
      ctx->d_pm = nullptr;
      ctx->pm_cap = 0;
      HIPCHK(ctx, hipMalloc(&ctx->d_pm, need_scr));
      ctx->pm_cap = need_scr;
    }
  }
  // stream-ordered after the previous call's kernels, which read the same device table
  HIPCHK(ctx, hipMemcpyAsync(ctx->d_pm_inst, it, 8 * m, hipMemcpyHostToDevice, s));
  HIPCHK(ctx, hipEventRecord(ctx->pm_inst_ev, s));
  ctx->pm_inst_ev_live = true;
  return B2F_OK;
}
}  // namespace

extern "C" {

B2F_API int b2f_permutation_columns_dev(b2f_ctx* ctx, const uint32_t* d_advice, uint64_t total_rows,
                                        const uint64_t* h_offsets, size_t n, uint32_t k,
                                        uint64_t usable_rows, const uint64_t omega[4],
                                        const uint64_t delta[4], const uint64_t beta[4],
                                        const uint64_t gamma[4], uint32_t chunk_len, uint32_t form,
                                        uint64_t* d_sigma, uint64_t* d_z, uint64_t out_rows,
                                        void* stream) {
  if (!ctx) return B2F_ERR_ARG;
  if (!d_advice || !h_offsets || !omega || !delta || !beta || !gamma || !d_z || n == 0)
    return set_err(ctx, B2F_ERR_ARG, "permutation: null buffer or no instances");
  if (chunk_len < 1 || chunk_len > PM_COLS)
    return set_err(ctx, B2F_ERR_ARG, "permutation: chunk_len %u not in [1, 8]", chunk_len);
  if (k < 10 || k > 30) return set_err(ctx, B2F_ERR_ARG, "permutation: k %u not in [10, 30]", k);
  if (((uintptr_t)d_z & 15) || ((uintptr_t)d_sigma & 15))
    return set_err(ctx, B2F_ERR_ARG, "permutation: outputs must be 16-byte aligned");
  const uint64_t n_rows = 1ull << k;
  if (h_offsets[n] > total_rows) return set_err(ctx, B2F_ERR_ROWS, "permutation: instances past total_rows");
  if (h_offsets[n] - h_offsets[0] > usable_rows || usable_rows >= n_rows)
    return set_err(ctx, B2F_ERR_ROWS, "permutation: need used rows %llu <= usable_rows %llu < 2^k",
                   (unsigned long long)(h_offsets[n] - h_offsets[0]), (unsigned long long)usable_rows);
  if (out_rows < usable_rows + 1 || (d_sigma && out_rows < n_rows))
    return set_err(ctx, B2F_ERR_ROWS, "permutation: out_rows too small");
  hipStream_t s = (hipStream_t)stream;
  const uint64_t* elems[4] = {omega, delta, beta, gamma};
  uint64_t row0 = 0, used = 0;
  if (int rc = perm_setup(ctx, "permutation", h_offsets, n, k, form, elems, 4,
                          perm_scratch_bytes(k, usable_rows, n, chunk_len), s, &row0, &used))
    return rc;
  if (int rc = ensure_side(ctx)) return rc;
  int tk = timed_begin(ctx, B2F_KERNEL_PERM, s);
  HIPCHK(ctx, launch_permutation(d_advice, total_rows, row0, ctx->d_pm_inst, n, ctx->d_pm_pool, k,
                                 usable_rows, omega, delta, beta, gamma, chunk_len, form, d_sigma,
                                 d_z, out_rows, ctx->d_pm, ctx->d_status + 2, ctx->s2, ctx->ev_fork,
                                 ctx->ev_join, s));
  timed_end(ctx, tk, s);
  return B2F_OK;
}

B2F_API int b2f_permutation_sigma_dev(b2f_ctx* ctx, const uint64_t* h_offsets, size_t n, uint32_t k,
                                      const uint64_t omega[4], const uint64_t delta[4], uint32_t form,
                                      uint64_t* d_sigma, uint64_t out_rows, void* stream) {
  if (!ctx) return B2F_ERR_ARG;
  if (!h_offsets || !omega || !delta || !d_sigma || n == 0)
    return set_err(ctx, B2F_ERR_ARG, "permutation sigma: null buffer or no instances");
  if ((uintptr_t)d_sigma & 15) return set_err(ctx, B2F_ERR_ARG, "permutation sigma: d_sigma must be 16-byte aligned");
  if (k < 10 || k > 30) return set_err(ctx, B2F_ERR_ARG, "permutation sigma: k %u not in [10, 30]", k);
  const uint64_t n_rows = 1ull << k;
  if (h_offsets[n] - h_offsets[0] >= n_rows)
    return set_err(ctx, B2F_ERR_ROWS, "permutation sigma: the instances need %llu rows >= 2^k",
                   (unsigned long long)(h_offsets[n] - h_offsets[0]));
  if (out_rows < n_rows) return set_err(ctx, B2F_ERR_ROWS, "permutation sigma: out_rows < 2^k");
  hipStream_t s = (hipStream_t)stream;
  const uint64_t* elems[2] = {omega, delta};
  uint64_t row0 = 0, used = 0;
  if (int rc = perm_setup(ctx, "permutation sigma", h_offsets, n, k, form, elems, 2, perm_sigma_scratch_bytes(k),
                          s, &row0, &used))
    return rc;
  int tk = timed_begin(ctx, B2F_KERNEL_PERM_SIGMA, s);
  HIPCHK(ctx, launch_permutation_sigma(ctx->d_pm_inst, n, ctx->d_pm_pool, k, omega, delta, form, d_sigma,
                                       out_rows, ctx->d_pm, s));
  timed_end(ctx, tk, s);
  return B2F_OK;
}

B2F_API int b2f_fill_fixed_dev(b2f_ctx* ctx, const uint64_t* d_offsets, size_t n,
                               uint64_t total_rows, uint32_t* d_fixed, void* stream) {
  if (!ctx) return B2F_ERR_ARG;
  if (!d_offsets || !d_fixed || n == 0) return set_err(ctx, B2F_ERR_ARG, "fill_fixed: null buffer or empty batch");
  if (n > 0xffffffffull) return set_err(ctx, B2F_ERR_ARG, "fill_fixed: more than 2^32 instances");
  if (total_rows % 4) return set_err(ctx, B2F_ERR_ARG, "fill_fixed: total_rows %% 4 != 0");
  if ((uintptr_t)d_fixed & 15) return set_err(ctx, B2F_ERR_ARG, "fill_fixed: d_fixed must be 16-byte aligned");
  if (total_rows < (uint64_t)FIXED_ROWS * n)
    return set_err(ctx, B2F_ERR_ROWS, "fill_fixed: %llu rows cannot hold %zu instances",
                   (unsigned long long)total_rows, n);
  hipStream_t s = (hipStream_t)stream;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipMemsetAsync(ctx->d_status, 0, sizeof(int), s));
  hipLaunchKernelGGL(offsets_check_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s,
                     d_offsets, (uint32_t)n, total_rows, ctx->d_status, ctx->d_status + 2,
                     (b2f_eval_report*)nullptr);
  HIPCHK(ctx, hipGetLastError());
  const uint64_t nt = n_tiles_of(total_rows);
  int rc = launch_tile_index(ctx, d_offsets, n, nt, s);
  if (rc) return rc;
  hipLaunchKernelGGL(fixed_kernel, dim3((uint32_t)nt), dim3(BLOCK), 0, s, d_offsets, (uint32_t)n,
                     total_rows, ctx->d_tiles, d_fixed, ctx->d_status);
  HIPCHK(ctx, hipGetLastError());
  return B2F_OK;
}

B2F_API uint64_t b2f_copy_constraints(uint32_t rounds, uint32_t* out4, uint64_t cap) {
  if (rounds > B2F_MAX_ROUNDS) return 0;
  return copy_constraints(rounds, out4, cap);
}

B2F_API int b2f_sync(b2f_ctx* ctx, void* stream) {
  if (!ctx) return B2F_ERR_ARG;
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipStreamSynchronize((hipStream_t)stream));
  int bits = 0;  // the sticky word: every error raised since the previous b2f_sync
  HIPCHK(ctx, hipMemcpy(&bits, ctx->d_status + 2, sizeof bits, hipMemcpyDeviceToHost));
  HIPCHK(ctx, hipMemset(ctx->d_status + 2, 0, sizeof bits));
  if (bits & (1 << B2F_ERR_ROUNDS)) return set_err(ctx, B2F_ERR_ROUNDS, "rounds > %u", B2F_MAX_ROUNDS);
  if (bits & (1 << B2F_ERR_LAYOUT))
    return set_err(ctx, B2F_ERR_LAYOUT, "row offsets are not the LAYOUT v1 prefix sums");
  if (bits & (1 << B2F_ERR_FIELD))
    return set_err(ctx, B2F_ERR_FIELD, "a grand product's denominator is zero (challenge collision)");
  if (bits & (1 << B2F_ERR_CHECK))
    return set_err(ctx, B2F_ERR_CHECK, "internal cross-check failed (lookup den product vs input side, or "
                                       "the fused pass's segment list overflowed)");
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


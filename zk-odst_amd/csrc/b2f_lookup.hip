// b2f_lookup.hip -- lookup-argument prover columns of the spread lookup (SURVEY.md §8(f)
// row 4): for circuits cut from the trace (usable rows each), halo2_proofs 0.3.0's
// compressed input A, compressed table S, permuted input A', permuted table S' and the
// grand product z (lookup/prover.rs: commit_permuted, permute_expression_pair,
// commit_product; restated in oracle/lookup.py), over pasta Fp or BN254 Fr (b2f_field.h).
//
// halo2 sorts the compressed inputs and walks a BTreeMap of table values. Here every input
// is a table row, so the sort is a counting sort over the 2^16 table rows in the order of
// their compressed values:
//   table pass (once per theta): T[x] = theta^2 tag(x) + theta x + spread(x) for x < 2^16,
//     sorted by canonical value (one radix sort by the top 64-bit limb, ties -- about 2^-33
//     likely -- ordered by the lower limbs), giving the rank order x_of_rank[r];
//   count:   histogram of the dense cell (a_1) over the circuit's rows (LDS-privatised, four
//            workgroups per circuit, a quarter of the bins each), with the row check (tag,
//            dense, spread) in table (first failing row reported);
//   scan:    in rank order, run starts pos[r] (exclusive prefix of counts), D[r] (runs up to
//            and including r) and the ranks with leftover table multiplicity, compacted
//            (lrank = their table index, lstart = their first leftover index), 16
//            workgroups per circuit (part totals, then each part's scan);
//   windows: per 1,024-row look-back block, the pos ranks its rows fall in and the compacted
//            leftover ranks its repeated rows take (lk_block_kernel: LDS-sampled searches,
//            one thread per block);
//   z pass:  row p of A' is T[x_of_rank[r]] for the run r holding p; a run start gets the
//            same S'[p]; the j-th repeated row gets leftover item L - 1 - j (halo2 hands
//            leftovers out in ascending order, each to the last open repeated row). The
//            workgroup scatters its block's windows into LDS tables by row and by leftover
//            index (table indices, so every gather reads T alone), so every row reads
//            its ranks; the same pass forms each row's factors num = (A + beta)(S + gamma) and
//            den = (A' + beta)(S' + gamma) in registers and writes the grand product z in one
//            go: the num side's block prefix and D^-1 come from a side-stream pre-pass over the
//            trace (D = prod num = prod den), the den side's suffix over blocks from a decoupled
//            look-back (lk_zpass_kernel below).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "../../include/b2f.h"
#include "b2f_field.h"
#include "b2f_gprod.h"

namespace b2f {

size_t lookup_scratch_bytes(uint32_t group, uint64_t usable_rows);
hipError_t launch_lookup(const uint32_t* d_advice, uint64_t total_rows,
                         const uint64_t* d_row_begin, uint32_t n_circuits, uint64_t usable_rows,
                         const uint64_t* theta, const uint64_t* beta, const uint64_t* gamma,
                         uint32_t form, uint64_t* d_out, uint64_t out_rows, uint64_t* d_first_bad,
                         void* scratch, uint32_t group, int* sticky, hipStream_t s2,
                         hipEvent_t ev_fork, hipEvent_t ev_join, hipStream_t s3, hipEvent_t ev_tab,
                         hipEvent_t ev_sorted, hipStream_t s);

namespace {

using field::Fe;
using field::load;
using field::store;
constexpr int TROWS = 1 << 16;

struct Chal {
  uint64_t theta[4], beta[4], gamma[4];
};

using gp::out_form;

__device__ __forceinline__ uint32_t spread16(uint32_t x) {
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x = (x | (x << 2)) & 0x33333333u;
  x = (x | (x << 1)) & 0x55555555u;
  return x;
}
__device__ __forceinline__ uint32_t tag16(uint32_t x) { return x < 256u ? 0u : (x < 32768u ? 1u : 2u); }

// ------------------------------------------------------------------ table pass (per theta)
template <class F>
__global__ __launch_bounds__(256) void lk_table_kernel(Chal ch, Fe* __restrict__ Tx,
                                                       uint64_t* __restrict__ key,
                                                       uint32_t* __restrict__ perm, Fe* __restrict__ bg) {
  const uint32_t x = blockIdx.x * 256 + threadIdx.x;
  if (x < 2) bg[x] = field::to_mont<F>(field::load_words(x ? ch.gamma : ch.beta));  // for the z pass
  const Fe th = field::to_mont<F>(field::load_words(ch.theta));
  const Fe th2 = field::mul<F>(th, th);
  const Fe t = field::add<F>(field::add<F>(field::mul<F>(th2, field::from_u32<F>(tag16(x))),
                                           field::mul<F>(th, field::from_u32<F>(x))),
                             field::from_u32<F>(spread16(x)));
  Tx[x] = t;
  const Fe c = field::to_canonical<F>(t);
#pragma unroll
  for (int k = 0; k < 4; k++)
    key[(uint64_t)k * TROWS + x] = (uint64_t)c.w[2 * k] | ((uint64_t)c.w[2 * k + 1] << 32);
  perm[x] = x;
}

// After one radix sort by the top 64-bit limb of the canonical value, equal top limbs are put in
// order by the three lower limbs: each thread of a run of equal top limbs (found by two binary
// searches in the sorted limbs) counts the run's members below it -- by the lower limbs, then
// by position -- and writes its table index at that rank into the output order; a thread not in
// a run copies its index. The rank order is then the order of the full 256-bit values, as four
// LSD passes over the limbs would give. For a uniform challenge runs are pairs at most (2^-33
// likely), but a structured one (theta = 3: every value below 2^192, one run of 2^16; theta = -3:
// a long run just below p, out of order) makes long runs, which cost O(L) per thread here, with
// L threads at once, instead of one thread's insertion sort (round 6; O(L^2) on one thread).
__global__ __launch_bounds__(256) void lk_tie_fix_kernel(const uint64_t* __restrict__ key,
                                                         const uint64_t* __restrict__ top,
                                                         const uint32_t* __restrict__ pin,
                                                         uint32_t* __restrict__ pout) {
  const uint32_t r = blockIdx.x * 256 + threadIdx.x;
  const uint64_t k = top[r];
  const uint32_t x = pin[r];
  const bool tl = r > 0 && top[r - 1] == k, tr = r + 1 < (uint32_t)TROWS && top[r + 1] == k;
  if (!tl && !tr) {
    pout[r] = x;
    return;
  }
  uint32_t lo = 0, hi = r;  // the run's first index: the first with top == k
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    if (top[m] < k) lo = m + 1;
    else hi = m;
  }
  const uint32_t s = lo;
  lo = r + 1;
  hi = TROWS;  // one past its last: the first with top > k
  while (lo < hi) {
    const uint32_t m = (lo + hi) >> 1;
    if (top[m] <= k) lo = m + 1;
    else hi = m;
  }
  const uint32_t e = lo;
  const uint64_t a2 = key[2ull * TROWS + x], a1 = key[(uint64_t)TROWS + x], a0 = key[x];
  uint32_t rank = 0;
#pragma unroll 8
  for (uint32_t q = s; q < e; q++) {  // (unrolled: eight members' loads in flight at once)
    const uint32_t y = pin[q];
    const uint64_t b2 = key[2ull * TROWS + y], b1 = key[(uint64_t)TROWS + y], b0 = key[y];
    rank += (b2 != a2 ? b2 < a2 : b1 != a1 ? b1 < a1 : b0 != a0 ? b0 < a0 : q < r) ? 1u : 0u;
  }
  pout[s + rank] = x;
}

// ------------------------------------------------------------------ per-circuit passes
struct Circ {
  uint64_t first;  // first trace row of the circuit
  uint64_t n_in;   // rows inside the trace (the rest read as zero rows)
};
__device__ __forceinline__ Circ circ(const uint64_t* row_begin, uint64_t total_rows,
                                     uint64_t usable, uint32_t c) {
  Circ k;
  k.first = row_begin[c];
  k.n_in = k.first >= total_rows ? 0 : (total_rows - k.first < usable ? total_rows - k.first : usable);
  return k;
}

// Histogram of the dense cell over a circuit's rows, privatised in LDS: workgroup (b, c) owns
// bins [b * 2^14, (b + 1) * 2^14) of circuit c (64 KiB of LDS counters), reads every row's
// dense cell (the later passes hit L2), counts the rows that fall in its range with LDS
// atomics and writes its bins with plain stores -- no global atomics and no memset. The
// table-membership check runs on each row once (rows dealt to the 4 workgroups by 1,024-row
// block); a circuit with a bad row reports it and its columns are meaningless, so rows are
// binned by their low 16 bits regardless.
constexpr int CNT_SPLIT = 4, CNT_BINS = TROWS / CNT_SPLIT, CNT_THREADS = 1024, CNT_UNROLL = 8;
static_assert(CNT_UNROLL % CNT_SPLIT == 0, "every workgroup checks one block per CNT_SPLIT blocks");
__global__ __launch_bounds__(CNT_THREADS) void lk_count_kernel(
    const uint32_t* __restrict__ adv, uint64_t total_rows, const uint64_t* __restrict__ row_begin,
    uint32_t c0, uint64_t usable, uint32_t* __restrict__ count, uint64_t* __restrict__ first_bad) {
  __shared__ uint32_t bins[CNT_BINS];
  const uint32_t b = blockIdx.x, c = blockIdx.y, t = threadIdx.x;
  const Circ k = circ(row_begin, total_rows, usable, c0 + c);
  for (uint32_t i = t; i < (uint32_t)CNT_BINS; i += CNT_THREADS) bins[i] = 0;
  __syncthreads();
  if (b == 0 && t == 0 && usable > k.n_in) atomicAdd(&bins[0], (uint32_t)(usable - k.n_in));  // zero rows
  uint64_t bad = ~0ull;
  // CNT_UNROLL blocks of rows per iteration: their loads are issued together, so the loop pays
  // one memory latency per CNT_UNROLL blocks (one per block: 110 us per call at 2^17 rows)
  for (uint64_t base = 0; base < k.n_in; base += (uint64_t)CNT_UNROLL * CNT_THREADS) {
    uint32_t a1[CNT_UNROLL];
#pragma unroll
    for (int u = 0; u < CNT_UNROLL; u++) {
      const uint64_t p = base + (uint64_t)u * CNT_THREADS + t;
      a1[u] = p < k.n_in ? adv[total_rows + k.first + p] : 0u;
    }
#pragma unroll
    for (int u = 0; u < CNT_UNROLL; u++) {
      const uint64_t p = base + (uint64_t)u * CNT_THREADS + t;
      if (p >= k.n_in) break;
      const uint64_t row = k.first + p;
      if (((p / CNT_THREADS) % CNT_SPLIT) == b) {  // this workgroup checks this block of rows
        const uint32_t a0 = adv[row], a2 = adv[2 * total_rows + row];
        const bool ok = a1[u] < (uint32_t)TROWS && a0 == tag16(a1[u]) && a2 == spread16(a1[u]);
        if (!ok && bad == ~0ull) bad = p;
      }
      const uint32_t x = a1[u] & 0xffffu;
      if ((x >> 14) == b) atomicAdd(&bins[x & (CNT_BINS - 1)], 1u);
    }
  }
  if (bad != ~0ull) atomicMin((unsigned long long*)first_bad + c0 + c, (unsigned long long)bad);
  __syncthreads();
  uint32_t* cnt = count + (uint64_t)c * TROWS + (uint64_t)b * CNT_BINS;
  for (uint32_t i = t; i < (uint32_t)CNT_BINS; i += CNT_THREADS) cnt[i] = bins[i];
}

// The rank-order scan of a circuit's counts, split over SC_PARTS workgroups per circuit of
// SC_THREADS threads x SC_PER consecutive ranks (the counts gathered into registers once per
// pass): lk_scan_sums writes each part's totals, lk_scan_write adds the totals of the parts
// before it and scans its own ranks. Four running sums: rows (pos = a run's first row), runs
// (dcnt, inclusive), leftover items (a rank's table multiplicity not taken by a run start) and
// leftover ranks -- the ranks with leftover items are written compacted (lrank, lstart = their
// first leftover index), so a block of rows' leftover items span at most one entry per item. (One 1,024-thread workgroup per circuit holding 64 ranks per
// thread kept the gathered counts in scratch and used 64 of the 256 CUs.)
#ifndef B2F_LK_SAMP
#define B2F_LK_SAMP 32  // pos / lstart sample stride of lk_block_kernel's LDS search tables
#endif
constexpr int SAMP = B2F_LK_SAMP;
static_assert(SAMP == 16 || SAMP == 32, "sample stride: a multiple of the scan's 16 ranks per thread");
constexpr int SAMPLE = TROWS / SAMP;  // every SAMP-th pos / lstart entry, for lk_block_kernel
constexpr int SC_PARTS = 16, SC_THREADS = 256, SC_PER = TROWS / (SC_PARTS * SC_THREADS);
static_assert(SC_PER == 16, "one search sample per thread");

// the counts of this thread's SC_PER ranks (rank order read as 16-byte vectors), the index of the
// rank holding table row 0 (-1: none), and the four sums: rows, runs, leftover table
// multiplicity, ranks with leftovers
struct RankRun {
  uint32_t nv[SC_PER];
  uint32_t xv[SC_PER];  // the table index of each rank
  int iz;
  uint32_t sc, sd, sl, sr;
};
__device__ __forceinline__ RankRun rank_run(const uint32_t* __restrict__ perm, const uint32_t* __restrict__ cnt,
                                            uint32_t r0, uint32_t mult0) {
  RankRun R;
  R.iz = -1;
  const uint4* pv = reinterpret_cast<const uint4*>(perm + r0);
#pragma unroll
  for (int i = 0; i < SC_PER / 4; i++) {
    const uint4 x = pv[i];
    R.nv[4 * i] = cnt[x.x];
    R.nv[4 * i + 1] = cnt[x.y];
    R.nv[4 * i + 2] = cnt[x.z];
    R.nv[4 * i + 3] = cnt[x.w];
    R.xv[4 * i] = x.x;
    R.xv[4 * i + 1] = x.y;
    R.xv[4 * i + 2] = x.z;
    R.xv[4 * i + 3] = x.w;
    R.iz = x.x == 0 ? 4 * i : x.y == 0 ? 4 * i + 1 : x.z == 0 ? 4 * i + 2 : x.w == 0 ? 4 * i + 3 : R.iz;
  }
  R.sc = R.sd = R.sl = R.sr = 0;
#pragma unroll
  for (int i = 0; i < SC_PER; i++) {
    const uint32_t n = R.nv[i];
    const uint32_t m = (i == R.iz ? mult0 : 1u) - (n ? 1u : 0u);
    R.sc += n;
    R.sd += n ? 1u : 0u;
    R.sl += m;
    R.sr += m ? 1u : 0u;
  }
  return R;
}

__global__ __launch_bounds__(SC_THREADS) void lk_scan_sums(const uint32_t* __restrict__ perm,
                                                           const uint32_t* __restrict__ count,
                                                           uint64_t usable, uint32_t* __restrict__ part) {
  const uint32_t pt = blockIdx.x, c = blockIdx.y, t = threadIdx.x;
  const uint32_t mult0 = (uint32_t)(usable - TROWS + 1);  // table row 0 fills the rest
  const RankRun R = rank_run(perm, count + (uint64_t)c * TROWS, (pt * SC_THREADS + t) * SC_PER, mult0);
  __shared__ uint32_t s[4][SC_THREADS];
  s[0][t] = R.sc;
  s[1][t] = R.sd;
  s[2][t] = R.sl;
  s[3][t] = R.sr;
  __syncthreads();
  for (uint32_t w = SC_THREADS / 2; w > 0; w >>= 1) {
    if (t < w) {
#pragma unroll
      for (int q = 0; q < 4; q++) s[q][t] += s[q][t + w];
    }
    __syncthreads();
  }
  if (t < 4) part[((uint64_t)c * SC_PARTS + pt) * 4 + t] = s[t][0];
}

__global__ __launch_bounds__(SC_THREADS) void lk_scan_write(const uint32_t* __restrict__ perm,
                                                            const uint32_t* __restrict__ count,
                                                            uint64_t usable, const uint32_t* __restrict__ part,
                                                            uint32_t* __restrict__ pos, uint32_t* __restrict__ dcnt,
                                                            uint32_t* __restrict__ lrank, uint32_t* __restrict__ lstart,
                                                            uint32_t* __restrict__ samp, uint32_t* __restrict__ nlr) {
  const uint32_t pt = blockIdx.x, c = blockIdx.y, t = threadIdx.x;
  const uint32_t mult0 = (uint32_t)(usable - TROWS + 1);
  const uint32_t r0 = (pt * SC_THREADS + t) * SC_PER;
  const RankRun R = rank_run(perm, count + (uint64_t)c * TROWS, r0, mult0);
  uint32_t bsum[4] = {0, 0, 0, 0};  // totals of the parts before this one
  for (uint32_t q = 0; q < pt; q++) {
    const uint32_t* pq = part + ((uint64_t)c * SC_PARTS + q) * 4;
#pragma unroll
    for (int i = 0; i < 4; i++) bsum[i] += pq[i];
  }
  __shared__ uint32_t s[4][SC_THREADS];
  const uint32_t own[4] = {R.sc, R.sd, R.sl, R.sr};
  uint32_t inc[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    s[i][t] = own[i];
    inc[i] = own[i];
  }
  __syncthreads();
  for (uint32_t off = 1; off < SC_THREADS; off <<= 1) {  // inclusive Hillis-Steele
    uint32_t a[4] = {0, 0, 0, 0};
    if (t >= off) {
#pragma unroll
      for (int i = 0; i < 4; i++) a[i] = s[i][t - off];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; i++) {
      inc[i] += a[i];
      s[i][t] = inc[i];
    }
    __syncthreads();
  }
  // exclusive: rows, runs, leftover items, leftover ranks
  uint32_t ec = bsum[0] + inc[0] - own[0], ed = bsum[1] + inc[1] - own[1], el = bsum[2] + inc[2] - own[2],
           er = bsum[3] + inc[3] - own[3];
  uint4* P4 = reinterpret_cast<uint4*>(pos + (uint64_t)c * TROWS + r0);
  uint4* D4 = reinterpret_cast<uint4*>(dcnt + (uint64_t)c * TROWS + r0);
  uint32_t* LR = lrank + (uint64_t)c * TROWS;
  uint32_t* LS = lstart + (uint64_t)c * TROWS;
  uint32_t* SP = samp + (uint64_t)c * 2 * SAMPLE;
  if (r0 % SAMP == 0) SP[r0 / SAMP] = ec;  // a pos sample
#pragma unroll
  for (int i = 0; i < SC_PER / 4; i++) {
    uint32_t pq[4], dq[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t n = R.nv[4 * i + j];
      const uint32_t m = (4 * i + j == R.iz ? mult0 : 1u) - (n ? 1u : 0u);  // leftovers
      pq[j] = ec;
      ed += n ? 1u : 0u;
      dq[j] = ed;
      if (m) {
        LR[er] = R.xv[4 * i + j];  // its table index: the z pass gathers Tx only
        LS[er] = el;
        if (er % SAMP == 0) SP[SAMPLE + er / SAMP] = el;  // an lstart sample
        er++;
      }
      ec += n;
      el += m;
    }
    P4[i] = make_uint4(pq[0], pq[1], pq[2], pq[3]);
    D4[i] = make_uint4(dq[0], dq[1], dq[2], dq[3]);
  }
  if (pt == SC_PARTS - 1 && t == SC_THREADS - 1) nlr[c] = er;  // ranks with leftovers
}

// ------------------------------------------------------------------ the grand product, one pass
// z[p + 1] = N_p / D_p with N_p = prod_{i <= p} num_i, D_p = prod_{i <= p} den_i,
// num_i = (A_i + beta)(S_i + gamma), den_i = (A'_i + beta)(S'_i + gamma). The rows are cut into
// look-back blocks of LB rows (one lk_zpass workgroup each, ZR consecutive rows per lane), and
//   z[p + 1] = (Nbefore_b D^-1) (Dafter_b) (N-prefix of the lanes before, in the block)
//              (D-suffix of the lanes after, in the block) (Nloc_p Dsuf_p, inside the lane)
// where Nbefore_b = the num product of the blocks before b and Dafter_b = the den product of
// the blocks after b. Both directions are available in ONE pass because the num side never
// depends on the permutation: A and S are known from the trace and the table alone, so
// lk_npart / lk_nscan form every block's num product, their prefix, the total D = prod num_i
// and D^-1 on the side stream, beside the count and scan passes (A' is a permutation of A and
// S' one of S -- the leftover items are exactly the table rows no run start took, row 0 with
// its usable - 2^16 + 1 multiplicity -- so prod den_i = prod num_i = D). The den side comes from
// the permuted columns the pass itself forms; its suffix over blocks is a decoupled look-back
// in descending block order (workgroups take tickets, so a block only ever waits for blocks
// whose workgroups already run). The pass writes the five columns once and nothing else: no
// factor, prefix or chunk slot makes a round trip through HBM (round 4's permute pass +
// gp_chunk + gp_write moved 384 B per row; this pass 164).
// Check: block 0's inclusive den product is D_den = prod den_i from the permuted
// columns, which must equal the num-side D; a difference (wrong A' or S') sets B2F_ERR_CHECK.
// LKMUL: the z pass's field products; a diagnostics build (-DB2F_LK_NOPROD, wrong results)
// replaces them by additions to time the pass without its products
#ifdef B2F_LK_NOPROD
#define LKMUL(x, y) field::add<F>(x, y)
#else
#define LKMUL(x, y) field::mul<F>(x, y)
#endif
// Rows per lane and waves per SIMD: ZR = 4 (7.25 products per row in the lanes against 8.25 at
// ZR = 2) at 4 waves: 128 VGPRs with 8 spilled (beta and gamma are uniform loads, the asm product
// of b2f_mont_asm.h keeps its accumulator in 4 fixed VGPRs). Measured per 64 x 131,065-row call:
// ZR = 2 at 4 waves 1.25-1.29 ms, ZR = 4 at 3 waves 1.12-1.15 (r05m), and with the block windows
// of lk_block_kernel 3 waves 1.04-1.05 against 4 waves 1.01-1.03 (r05q, same process)
#ifndef B2F_ZP_WAVES
#define B2F_ZP_WAVES 4
#endif
#ifndef B2F_ZR
#define B2F_ZR 4
#endif
constexpr int ZR = B2F_ZR;       // rows per lane
static_assert(ZR == 2 || ZR == 4, "rows per lane");
#ifndef B2F_ZT
#define B2F_ZT 256
#endif
constexpr int ZT = B2F_ZT;       // lanes per look-back block (lk_zpass workgroup)
constexpr int ZW = ZT / 64;      // its waves; a scanning lane takes ZW of the ZT lane totals
static_assert(ZT == 128 || ZT == 256, "2 or 4 waves per look-back block");
constexpr int LB = ZT * ZR;      // rows per look-back block
__host__ __device__ inline uint64_t n_lb(uint64_t usable) { return (usable + LB - 1) / LB; }

// Diagnostics (variant builds with -DB2F_LK_CLOCK only): per-phase s_memtime totals of
// lk_zpass_kernel summed over waves, read by b2f_debug_lk_clock (tools/lk_clock.py).
#ifdef B2F_LK_CLOCK
// [11] resident workgroups now, [12] their maximum, [13] / [14] first start / last end tick
__device__ unsigned long long g_lk_clock[24];
#define LKCLK_DECL                                                           \
  uint64_t lk_t = __builtin_amdgcn_s_memtime();                             \
  if (threadIdx.x == 0) {                                                   \
    atomicMin(&g_lk_clock[13], (unsigned long long)lk_t);                   \
    atomicMax(&g_lk_clock[12], atomicAdd(&g_lk_clock[11], 1ull) + 1);        \
  }
#define LKCLK_END                                                           \
  if (threadIdx.x == 0) {                                                   \
    atomicMax(&g_lk_clock[14], (unsigned long long)__builtin_amdgcn_s_memtime()); \
    atomicAdd(&g_lk_clock[11], ~0ull);                                      \
  }
#define LKCLK(i)                                                                 \
  do {                                                                           \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();                          \
    if (lane == 0) atomicAdd(&g_lk_clock[i], (unsigned long long)(now_ - lk_t)); \
    lk_t = now_;                                                                 \
  } while (0)
#else
#define LKCLK_DECL
#define LKCLK_END
#define LKCLK(i) \
  do {           \
  } while (0)
#endif

#ifdef B2F_DIAG
// Diagnostics build only (libb2f_diag.so, B2F_DIAG_LK_CORRUPT=1 at the call): row 0's A' of every
// circuit is read from the next table row, i.e. one wrong permuted cell, so the den-product
// cross-check must raise B2F_ERR_CHECK (a test that sees it fire).
__device__ uint32_t g_lk_corrupt;
#endif

__device__ __forceinline__ Fe shfl_fe(const Fe& v, int src) {
  Fe r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.w[i] = (uint32_t)__shfl((int)v.w[i], src, 64);
  return r;
}
__device__ __forceinline__ Fe shfl_xor_fe(const Fe& v, int m) {
  Fe r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.w[i] = (uint32_t)__shfl_xor((int)v.w[i], m, 64);
  return r;
}
// the product of the 64 lanes' values, in every lane
template <class F>
__device__ __forceinline__ Fe wave_prod(Fe v) {
#pragma unroll 1
  for (int m = 32; m > 0; m >>= 1) v = field::mul<F>(v, shfl_xor_fe(v, m));
  return v;
}

// Block num products, the A part: NP_LPB lanes per look-back block, each lane NP_RPL rows
// NP_LPB apart (the product is order-free, so a load instruction reads NP_LPB consecutive cells
// of each of the wave's blocks), two product chains per lane, then log2(NP_LPB) butterfly levels
// inside the lane group (a whole-wave product per block cost 6 levels on 8 rows per lane).
// Row y == g of the grid: the S part (S_i + gamma), the same for every circuit and every group,
// so only the first group's launch has that row.
constexpr int NP_RPL = 32;                 // rows per lane
constexpr int NP_LPB = LB / NP_RPL;        // lanes per block
constexpr int NP_BPW = 64 / NP_LPB;        // blocks per wave
static_assert(NP_LPB >= 2 && NP_LPB <= 64 && (NP_LPB & (NP_LPB - 1)) == 0, "lane groups");
template <class F>
__global__ __launch_bounds__(256) void lk_npart_kernel(const uint32_t* __restrict__ adv, uint64_t total_rows,
                                                       const uint64_t* __restrict__ row_begin, uint32_t c0,
                                                       uint32_t g, uint64_t usable, uint64_t nb,
                                                       const Fe* __restrict__ Tx, Chal ch,
                                                       Fe* __restrict__ partA, Fe* __restrict__ partS) {
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, y = blockIdx.y;
  const uint64_t b = ((uint64_t)blockIdx.x * 4 + wv) * NP_BPW + lane / NP_LPB;
  const bool s_part = y == g;
  const Fe add = field::to_mont<F>(field::load_words(s_part ? ch.gamma : ch.beta));
  const Circ k = s_part ? Circ{0, 0} : circ(row_begin, total_rows, usable, c0 + y);
  const uint64_t base = b * LB + lane % NP_LPB;
  Fe acc0 = field::one<F>(), acc1 = field::one<F>();
#pragma unroll 1
  for (int i0 = 0; i0 < NP_RPL; i0 += 4) {
    uint32_t x[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint64_t q = base + (uint64_t)NP_LPB * (i0 + u);
      x[u] = s_part ? (q < (uint64_t)TROWS ? (uint32_t)q : 0u)
                    : (q < k.n_in ? (adv[total_rows + k.first + q] & 0xffffu) : 0u);
    }
    Fe v[4];
#pragma unroll
    for (int u = 0; u < 4; u++)
      v[u] = base + (uint64_t)NP_LPB * (i0 + u) < usable ? field::add<F>(Tx[x[u]], add) : field::one<F>();
    acc0 = field::mul<F>(acc0, field::mul<F>(v[0], v[1]));
    acc1 = field::mul<F>(acc1, field::mul<F>(v[2], v[3]));
  }
  Fe acc = field::mul<F>(acc0, acc1);
#pragma unroll 1
  for (int m = 1; m < NP_LPB; m <<= 1) acc = field::mul<F>(acc, shfl_xor_fe(acc, m));
  if (lane % NP_LPB == 0 && b < nb) (s_part ? partS[b] : partA[(uint64_t)y * nb + b]) = acc;
}

// Per circuit: N_b = A part x S part, the exclusive prefix over blocks (runs per thread, a
// Hillis-Steele scan of the run products in LDS), D = the total, D^-1 (one lane's inversion at
// top issue priority; D = 0 -- a zero factor -- raises B2F_ERR_FIELD), then NK_b = Nbefore_b D^-1.
constexpr int NS_T = 256;
template <class F>
__global__ __launch_bounds__(NS_T) void lk_nscan_kernel(uint64_t nb, const Fe* __restrict__ partA,
                                                        const Fe* __restrict__ partS, Fe* __restrict__ NK,
                                                        Fe* __restrict__ Dnum, int* __restrict__ sticky) {
  __shared__ Fe sn[NS_T];
  __shared__ Fe sdinv;
  const uint32_t c = blockIdx.x, t = threadIdx.x;
  const uint64_t per = (nb + NS_T - 1) / NS_T;
  const uint64_t b0 = t * per < nb ? t * per : nb, e = b0 + per < nb ? b0 + per : nb;
  const Fe* pa = partA + (uint64_t)c * nb;
  Fe run = field::one<F>();
  for (uint64_t b = b0; b < e; b++) run = field::mul<F>(run, field::mul<F>(pa[b], partS[b]));
  Fe inc = run;
  sn[t] = inc;
  __syncthreads();
  for (int off = 1; off < NS_T; off <<= 1) {
    Fe x = inc;
    if (t >= (uint32_t)off) x = field::mul<F>(sn[t - off], inc);
    __syncthreads();
    sn[t] = inc = x;
    __syncthreads();
  }
  if (t == 0) {
    const Fe D = sn[NS_T - 1];
    Dnum[c] = D;
    __builtin_amdgcn_s_setprio(3);
    if (sticky && field::is_zero(D)) atomicOr(sticky, 1 << B2F_ERR_FIELD);
    bool ok;
    sdinv = field::inv_safegcd<F>(D, ok);
    if (sticky && !ok) atomicOr(sticky, 1 << B2F_ERR_CHECK);
    __builtin_amdgcn_s_setprio(0);
  }
  __syncthreads();
  Fe rn = field::mul<F>(t ? sn[t - 1] : field::one<F>(), sdinv);
  Fe* nk = NK + (uint64_t)c * nb;
  for (uint64_t b = b0; b < e; b++) {
    nk[b] = rn;
    rn = field::mul<F>(rn, field::mul<F>(pa[b], partS[b]));
  }
}

// Look-back state of a block: words 0..5 its den product (aggregate), 8..13 the den product of
// it and every block after it (inclusive), word 15 its status (1 aggregate, 2 inclusive). An
// element goes out as six 48-bit pieces, each in a u64 tagged in its top 16 bits and stored with
// a relaxed agent-scope atomic: a reader that sees all six tags has the whole value, so no
// release fence (and no L2 write-back) is needed; the status word (written after the pieces) is
// what pollers read -- one word per block -- and a reader that finds a piece untagged polls
// again. The state is zeroed before each launch.
constexpr int LBS_WORDS = 16;
constexpr uint64_t LB_M48 = (1ull << 48) - 1;
constexpr uint64_t LB_TAG_AGG = 0xB2F1ull << 48, LB_TAG_INC = 0xB2F2ull << 48;
__device__ __forceinline__ uint64_t lb_piece(const Fe& v, uint32_t k) {
  const uint64_t L0 = v.w[0] | (uint64_t)v.w[1] << 32, L1 = v.w[2] | (uint64_t)v.w[3] << 32;
  const uint64_t L2 = v.w[4] | (uint64_t)v.w[5] << 32, L3 = v.w[6] | (uint64_t)v.w[7] << 32;
  const uint64_t w[6] = {L0 & LB_M48, (L0 >> 48 | L1 << 16) & LB_M48, (L1 >> 32 | L2 << 32) & LB_M48,
                         (L2 >> 16) & LB_M48, L3 & LB_M48, L3 >> 48};
  uint64_t r = w[0];
#pragma unroll
  for (uint32_t i = 1; i < 6; i++) r = k == i ? w[i] : r;
  return r;
}
__device__ __forceinline__ Fe lb_join(const uint64_t (&w)[6]) {
  const uint64_t L0 = (w[0] & LB_M48) | (w[1] << 48);
  const uint64_t L1 = ((w[1] & LB_M48) >> 16) | (w[2] << 32);
  const uint64_t L2 = ((w[2] & LB_M48) >> 32) | ((w[3] & LB_M48) << 16);
  const uint64_t L3 = (w[4] & LB_M48) | (w[5] << 48);
  Fe v;
  v.w[0] = (uint32_t)L0; v.w[1] = (uint32_t)(L0 >> 32);
  v.w[2] = (uint32_t)L1; v.w[3] = (uint32_t)(L1 >> 32);
  v.w[4] = (uint32_t)L2; v.w[5] = (uint32_t)(L2 >> 32);
  v.w[6] = (uint32_t)L3; v.w[7] = (uint32_t)(L3 >> 32);
  return v;
}
// (exchange stores, memory-side fetch-add loads and an acquire fence per poll were measured
// neutral or slower, r05i-k: DESIGN.md §5)
__device__ __forceinline__ uint64_t lb_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// lanes 0..5 of the calling wave publish v (the same in every lane) as the aggregate (kind 1) or
// the inclusive value (kind 2) of block state st, then lane 0 its status
__device__ __forceinline__ void lb_publish(uint64_t* st, uint32_t lane, const Fe& v, uint32_t kind) {
  if (lane < 6) lb_store(st + (kind == 2 ? 8 : 0) + lane, lb_piece(v, lane) | (kind == 2 ? LB_TAG_INC : LB_TAG_AGG));
  if (lane == 0) lb_store(st + 15, kind);
}
// the value of kind `kind` of block state st; false while a piece is not yet visible
__device__ __forceinline__ bool lb_read(const uint64_t* st, uint32_t kind, Fe& v) {
  uint64_t w[6];
  const uint64_t tag = kind == 2 ? LB_TAG_INC : LB_TAG_AGG;
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 6; i++) {
    w[i] = lb_load(st + (kind == 2 ? 8 : 0) + i);
    ok &= (w[i] & ~LB_M48) == tag;
  }
  v = lb_join(w);
  return ok;
}

// One column's values of a wave's 64 ZR rows r0 .. (lane l holds rows r0 + ZR l + j in v[j]) to
// dst rows below lim as 1 KiB runs: 128 / ZR lanes at a time stage their 128 rows in the wave's
// LDS (a (2 ZR + 1) x 16-byte lane stride: conflict-free 16-byte writes) and the wave stores them
// with four 1 KiB instructions.
constexpr int ZLPS = 128 / ZR;          // lanes per staging round
constexpr int ZLST = 2 * ZR + 1;        // uint4 per staged lane (padded)
constexpr int ZSTAGE = ZLPS * ZLST;     // uint4 of staging per wave
template <bool NT>
__device__ __forceinline__ void wave_store_zr(uint64_t* dst, uint4* st, uint32_t lane, const Fe (&v)[ZR],
                                              uint32_t r0, uint32_t lim) {
  // the wave's rows are 128 ZR consecutive 16-byte chunks from a uniform base: chunk 256 h + 64 q
  // + lane is staged at q (32 / ZR) ZLST + ZLST (lane / 2 ZR) + lane % 2 ZR of round h
  uint4* d = reinterpret_cast<uint4*>(dst + 4ull * r0);
  const uint32_t rem2 = lim > r0 ? (lim - r0 < 64u * ZR ? 2 * (lim - r0) : 128u * ZR) : 0u;  // chunks below lim
  const uint32_t rd = ZLST * (lane / (2 * ZR)) + lane % (2 * ZR);
#pragma unroll
  for (uint32_t h = 0; h < ZR / 2; h++) {
    if (lane / ZLPS == h) {
      const uint32_t li = lane % ZLPS;
#pragma unroll
      for (int j = 0; j < ZR; j++) {
        st[li * ZLST + 2 * j] = make_uint4(v[j].w[0], v[j].w[1], v[j].w[2], v[j].w[3]);
        st[li * ZLST + 2 * j + 1] = make_uint4(v[j].w[4], v[j].w[5], v[j].w[6], v[j].w[7]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    uint4 x[4];
#pragma unroll
    for (int q = 0; q < 4; q++) x[q] = st[(32 / ZR) * ZLST * q + rd];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t ch = 256u * h + 64u * q + lane;
      if (ch < rem2) gp::put16<NT>(d + ch, x[q]);
    }
  }
}

// lk_block_kernel's searches: the last index r < lim with a[r] <= v (a nondecreasing, a[0] <= v).
// The top levels run over the workgroup's LDS sample s[k] = a[SAMP k] (ns valid samples) as a
// fixed-step branchless binary search, then the SAMP entries of that block (64 or 128
// contiguous bytes) are counted in registers; eq tells whether one of them equals v.
static_assert((SAMPLE & (SAMPLE - 1)) == 0, "fixed-step search");
__device__ __forceinline__ uint32_t le_sample(const uint32_t* s, uint32_t v, uint32_t ns) {
  uint32_t lo = 0;
#pragma unroll
  for (uint32_t step = SAMPLE / 2; step > 0; step >>= 1) lo = lo + step < ns && s[lo + step] <= v ? lo + step : lo;
  return lo;
}
__device__ __forceinline__ uint32_t le_block(const uint32_t* __restrict__ a, uint32_t kb, uint32_t v, uint32_t lim,
                                             bool& eq) {
  const uint4* blk = reinterpret_cast<const uint4*>(a + SAMP * kb);
  uint4 q[SAMP / 4];
#pragma unroll
  for (int i = 0; i < SAMP / 4; i++) q[i] = blk[i];
  const uint32_t i0 = SAMP * kb;
  uint32_t n = 0, e = 0;
#pragma unroll
  for (int i = 0; i < SAMP / 4; i++) {
    const uint32_t w[4] = {q[i].x, q[i].y, q[i].z, q[i].w};
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const bool in = i0 + 4 * i + u < lim;
      n += in && w[u] <= v ? 1u : 0u;
      e |= in && w[u] == v ? 1u : 0u;
    }
  }
  eq = e != 0;
  return i0 + n - 1;  // the block's first entry s[kb] <= v
}

// Per look-back block (rows [base, end), end = min(base + LB, usable)) of every circuit: the pos
// ranks of its first and last rows (every row of the block lies in a run of that rank window),
// J0 / J1 = the repeated rows (those that are not a run's first row) before base / before end,
// and the window of compacted leftover ranks holding leftover indices [n_left - J1,
// n_left - 1 - J0], which the block's repeated rows take (the j-th repeated row takes
// n_left - 1 - j). J(p) = p - dcnt[ra(p)] + [p starts its run]. One thread per block; the z pass
// then finds every row's runs from these windows without searching.
constexpr int BLK_WORDS = 8;
constexpr int BK_T = 128;
__global__ __launch_bounds__(BK_T) void lk_block_kernel(uint64_t usable, uint64_t nb, const uint32_t* __restrict__ pos,
                                                        const uint32_t* __restrict__ dcnt,
                                                        const uint32_t* __restrict__ lstart,
                                                        const uint32_t* __restrict__ samp,
                                                        const uint32_t* __restrict__ nlr, uint32_t* __restrict__ blk) {
  __shared__ uint4 ss[2 * SAMPLE / 4];
  const uint32_t c = blockIdx.y, t = threadIdx.x;
  {
    const uint4* sa = reinterpret_cast<const uint4*>(samp + (uint64_t)c * 2 * SAMPLE);
    for (uint32_t i = t; i < (uint32_t)SAMPLE / 2; i += BK_T) ss[i] = sa[i];
  }
  __syncthreads();
  const uint32_t* sP = reinterpret_cast<const uint32_t*>(ss);
  const uint32_t* sL = sP + SAMPLE;
  const uint32_t us = (uint32_t)usable;
  const uint32_t* P = pos + (uint64_t)c * TROWS;
  const uint32_t* D = dcnt + (uint64_t)c * TROWS;
  const uint32_t* LS = lstart + (uint64_t)c * TROWS;
  const uint32_t n_left = us - D[TROWS - 1], nr = nlr[c], nsl = (nr + SAMP - 1) / SAMP;
  for (uint64_t b = (uint64_t)blockIdx.x * BK_T + t; b < nb; b += (uint64_t)gridDim.x * BK_T) {
    const uint32_t base = (uint32_t)b * LB, end = us - base < (uint32_t)LB ? us : base + LB;
    bool st;
    const uint32_t r0 = le_block(P, le_sample(sP, base, SAMPLE), base, TROWS, st);
    const uint32_t J0 = base - D[r0] + (st ? 1u : 0u);
    const uint32_t r1 = le_block(P, le_sample(sP, end - 1, SAMPLE), end - 1, TROWS, st);
    uint32_t J1 = n_left;
    if (end < us) {
      const uint32_t re = le_block(P, le_sample(sP, end, SAMPLE), end, TROWS, st);
      J1 = end - D[re] + (st ? 1u : 0u);
    }
    uint32_t k0 = 1, k1 = 0;  // empty
    if (J1 > J0) {
      k0 = le_block(LS, le_sample(sL, n_left - J1, nsl), n_left - J1, nr, st);
      k1 = le_block(LS, le_sample(sL, n_left - 1 - J0, nsl), n_left - 1 - J0, nr, st);
    }
    uint4* o = reinterpret_cast<uint4*>(blk + ((uint64_t)c * nb + b) * BLK_WORDS);
    o[0] = make_uint4(r0, r1, J0, J1);
    o[1] = make_uint4(k0, k1, 0u, 0u);
  }
}

// The five columns of one look-back block (LB = ZT ZR rows). Lane t of the workgroup owns rows
// base + ZR t + j:
//  1. the runs: A' = T[x_of_rank[r]] for the run r holding p, S' = A' at a run start, else leftover item
//     n_left - 1 - j for the j-th repeated row (halo2 hands leftovers out in ascending order,
//     each to the last open repeated row). The workgroup scatters the runs of its pos window and
//     the leftover ranks of its lstart window (lk_block_kernel) into LDS tables indexed by row
//     and by leftover index, so each row reads its ranks instead of searching;
//  2. the den side: A', S' staged and stored as 1 KiB runs, den_j = (A' + beta)(S' + gamma), the
//     in-lane den suffix and the lane's den total; one wave scans the 256 den totals (suffix)
//     and publishes the block's den product as its look-back aggregate at once;
//  3. the num side: A = Tx[x] (x the dense cell), S = Tx[p] (row 0's value past the table),
//     num_j, the in-lane num prefix, Q_j = Nloc_j Dsuf_(j+1); another wave scans the 256 num
//     totals (prefix) while the den wave looks back over the blocks after this one (64 per step)
//     for the den product after the block -- its predecessors have had the whole num side to
//     publish -- and publishes its inclusive product;
//  4. z[p + 1] = (num prefix before the lane) (den suffix after the lane, times NK_b Dafter_b) Q_j.
// The scans run on waves chosen by the ticket, so the SIMDs share them; the LDS tables of step 1
// are reused for the lane totals once every wave has read its rows.
template <class F, bool MONT>
__global__ __launch_bounds__(ZT) __attribute__((amdgpu_waves_per_eu(B2F_ZP_WAVES))) void lk_zpass_kernel(
    const uint32_t* __restrict__ adv, uint64_t total_rows, const uint64_t* __restrict__ row_begin,
    uint32_t c0, uint32_t g, uint64_t usable, uint64_t nb, const Fe* __restrict__ Tx,
    const uint32_t* __restrict__ xrank, uint64_t* __restrict__ out, uint64_t out_rows, Chal ch,
    const uint32_t* __restrict__ pos, const uint32_t* __restrict__ dcnt, const uint32_t* __restrict__ lrank,
    const uint32_t* __restrict__ lstart, const uint32_t* __restrict__ blk, const uint32_t* __restrict__ nlr,
    const Fe* __restrict__ NK, const Fe* __restrict__ Dnum, const Fe* __restrict__ bg,
    uint64_t* __restrict__ lbs, uint32_t* __restrict__ ticket, int* __restrict__ sticky) {
  // the row and leftover tables, then (after every wave has read its rows) the lane totals
  constexpr int SMEM = 2 * LB * 4 > 2 * ZT * 32 ? 2 * LB * 4 : 2 * ZT * 32;
  __shared__ uint4 smem[SMEM / 16];
  uint32_t* ent = reinterpret_cast<uint32_t*>(smem);  // per row: rank | start << 16 | (j - J0) << 17
  uint32_t* yl = ent + LB;                             // per leftover index - ylo: its rank
  Fe* sN = reinterpret_cast<Fe*>(smem);
  Fe* sD = sN + ZT;
  __shared__ uint4 stage[ZW][ZSTAGE];  // per wave: the column staging
  __shared__ Fe sX[64], sDb;          // the den wave's exclusive values and block product, parked
  __shared__ uint32_t s_tk;
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  LKCLK_DECL
  if (t == 0) s_tk = atomicAdd(ticket, 1u);
  __syncthreads();
  const uint32_t tk = s_tk;
  // descending block order: every circuit's last block first
  const uint32_t c = tk % g;
  const uint64_t b = nb - 1 - tk / g;
  const Fe beta = bg[0], gamma = bg[1];  // Montgomery forms (lk_table_kernel): uniform loads
  const Circ k = circ(row_begin, total_rows, usable, c0 + c);
  // 32-bit row arithmetic (usable <= 2^31, b2f_lookup_columns_dev)
  const uint32_t us = (uint32_t)usable, n_in = (uint32_t)k.n_in;
  const uint32_t* a1 = adv + total_rows + k.first;  // the circuit's dense cells
  const uint32_t* P = pos + (uint64_t)c * TROWS;
  const uint32_t* D = dcnt + (uint64_t)c * TROWS;
  const uint32_t* LR = lrank + (uint64_t)c * TROWS;
  const uint32_t* LS = lstart + (uint64_t)c * TROWS;
  const uint32_t n_left = us - D[TROWS - 1];  // repeated rows = leftover items
  uint64_t* o = out + (uint64_t)(c0 + c) * 5 * out_rows * 4;
  const uint32_t base = (uint32_t)b * LB, p0 = base + ZR * t, r0 = base + 64u * ZR * wv;
  uint4* st = stage[wv];
  // lane totals sit transposed (entry i at (i % ZW) 64 + i / ZW): a scanning lane's ZW entries are
  // 64 elements apart and its neighbours' adjacent (4-entry rows put lanes 128 B apart on the
  // same banks)
  auto pz = [](uint32_t i) { return (i % ZW) * 64u + i / ZW; };
  const uint32_t wn = tk % ZW, wd = (tk + 1) % ZW;  // the num-scan and den-scan waves
  const uint32_t e0 = ZW * lane;                    // a scanning lane's first entry
  __syncthreads();
  LKCLK(0);
  uint32_t x[ZR], ra[ZR], rs[ZR];
  // 1. the runs of the block's rows: every rank of the pos window writes its rows' entries (its
  // table index x_of_rank, so the gathers below read Tx alone: one 2 MiB table in L2, not two),
  // every compacted leftover rank of the lstart window its leftover indices' table index
  {
    const uint4* bt = reinterpret_cast<const uint4*>(blk + ((uint64_t)c * nb + b) * BLK_WORDS);
    const uint4 w0 = bt[0], w1 = bt[1];
    const uint32_t J0 = w0.z, end = us - base < (uint32_t)LB ? us : base + LB, ylo = n_left - w0.w,
                   yhi = n_left - J0, nr = nlr[c];
    // the first SC_U ranks of each window per thread (windows are ~LB / 2 wide): every load in
    // flight before the first write; wider windows finish in the loops after
    constexpr int SC_U = 4;
    uint32_t ps0[SC_U], ps1[SC_U], pd[SC_U], px[SC_U], ly0[SC_U], ly1[SC_U], lr[SC_U];
#pragma unroll
    for (int u = 0; u < SC_U; u++) {
      const uint32_t r = w0.x + t + ZT * u, kk = w1.x + t + ZT * u;
      ps0[u] = ps1[u] = pd[u] = px[u] = 0;
      ly0[u] = ly1[u] = lr[u] = 0;
      if (r <= w0.y) {
        ps0[u] = P[r];
        ps1[u] = r + 1 < (uint32_t)TROWS ? P[r + 1] : us;
        pd[u] = D[r];
        px[u] = xrank[r];
      }
      if (kk <= w1.y) {
        ly0[u] = LS[kk];
        ly1[u] = kk + 1 < nr ? LS[kk + 1] : n_left;
        lr[u] = LR[kk];
      }
    }
    auto put_run = [&](uint32_t xr, uint32_t s0, uint32_t s1, uint32_t dr) {
      const uint32_t lo = s0 > base ? s0 : base, hi = s1 < end ? s1 : end;
      for (uint32_t q = lo; q < hi; q++) ent[q - base] = q == s0 ? (xr | 0x10000u) : (xr | ((q - dr - J0) << 17));
    };
    auto put_left = [&](uint32_t r, uint32_t y0, uint32_t y1) {
      const uint32_t lo = y0 > ylo ? y0 : ylo, hi = y1 < yhi ? y1 : yhi;
      for (uint32_t y = lo; y < hi; y++) yl[y - ylo] = r;
    };
#pragma unroll
    for (int u = 0; u < SC_U; u++) {
      put_run(px[u], ps0[u], ps1[u], pd[u]);  // empty (s0 = s1 = 0) past the window
      put_left(lr[u], ly0[u], ly1[u]);
    }
    for (uint32_t r = w0.x + t + ZT * SC_U; r <= w0.y; r += ZT)
      put_run(xrank[r], P[r], r + 1 < (uint32_t)TROWS ? P[r + 1] : us, D[r]);
    for (uint32_t kk = w1.x + t + ZT * SC_U; kk <= w1.y; kk += ZT)
      put_left(LR[kk], LS[kk], kk + 1 < nr ? LS[kk + 1] : n_left);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ZR; j++) {
      const uint32_t p = p0 + j;
      x[j] = p < n_in ? (a1[p] & 0xffffu) : 0u;
      ra[j] = rs[j] = 0;
      if (p < us) {
        const uint32_t e = ent[p - base];
        ra[j] = e & 0xffffu;
        rs[j] = (e & 0x10000u) ? ra[j] : yl[yhi - 1u - (e >> 17) - ylo];
      }
    }
  }
  LKCLK(1);
#ifdef B2F_DIAG
  if (g_lk_corrupt && b == 0 && t == 0) ra[0] = (ra[0] + 1u) & 0xffffu;
#endif
  // 2. the den side: A', S' -> d[j] = den_j, the in-lane suffix sf[j] = prod_{i > j} d_i, dl
  Fe a[ZR], d[ZR], v[ZR];
#pragma unroll
  for (int j = 0; j < ZR; j++) v[j] = Tx[ra[j]];  // ra, rs: table indices (step 1)
#pragma unroll
  for (int j = 0; j < ZR; j++) {
    d[j] = field::add<F>(v[j], beta);
    v[j] = gp::out_form<F>(v[j], MONT);
  }
  wave_store_zr<true>(o + 2 * out_rows * 4, st, lane, v, r0, us);
#pragma unroll
  for (int j = 0; j < ZR; j++) v[j] = Tx[rs[j]];
#pragma unroll
  for (int j = 0; j < ZR; j++) {
    d[j] = p0 + j < us ? LKMUL(d[j], field::add<F>(v[j], gamma)) : field::one<F>();
    v[j] = gp::out_form<F>(v[j], MONT);
  }
  wave_store_zr<true>(o + 3 * out_rows * 4, st, lane, v, r0, us);
  Fe sf[ZR];
  sf[ZR - 2] = d[ZR - 1];
#pragma unroll
  for (int j = ZR - 3; j >= 0; j--) sf[j] = LKMUL(d[j + 1], sf[j + 1]);
  const Fe dl = LKMUL(d[0], sf[0]);
  __syncthreads();  // every wave has read its rows: the tables' memory takes the lane totals
  sD[pz(t)] = dl;
  __syncthreads();
  LKCLK(2);
  // the den wave: its in-lane scan (suffix order: entry i of the scan is lane total 255 - i) and
  // the 6-level scan across its lanes; the block's product goes out as the aggregate at once
  uint64_t* my = lbs + ((uint64_t)c * nb + b) * LBS_WORDS;
  auto atd = [&](uint32_t i) { return pz((uint32_t)ZT - 1u - i); };
  if (wv == wd) {
    Fe Pd = sD[atd(e0)];
    sD[atd(e0)] = field::one<F>();
#ifdef B2F_LK_NOSCAN  // diagnostics (wrong z): the block scans' products left out, to bound what they cost
    if (false)
#endif
#pragma unroll 1
    for (uint32_t k2 = 1; k2 < (uint32_t)ZW; k2++) {
      const Fe e = sD[atd(e0 + k2)];
      sD[atd(e0 + k2)] = Pd;
      Pd = LKMUL(Pd, e);
    }
#ifdef B2F_LK_NOSCAN
    if (false)
#endif
#pragma unroll 1
    for (int off = 1; off < 64; off <<= 1) {
      const Fe y = shfl_fe(Pd, (int)lane - off);
      const Fe m = LKMUL(y, Pd);
      if (lane >= (uint32_t)off) Pd = m;
    }
    Fe X = shfl_fe(Pd, (int)lane - 1);
    if (lane == 0) X = field::one<F>();
    const Fe Db = shfl_fe(Pd, 63);
    if (b + 1 < nb) lb_publish(my, lane, Db, 1);
    sX[lane] = X;  // parked in LDS across the num side (registers are the limit there)
    if (lane == 0) sDb = Db;
  }
  LKCLK(3);
  // 3. the num side: A, S -> a[j] = num_j -> Nloc_j; Q_j = Nloc_j Dsuf_(j+1) (kept in v)
#pragma unroll
  for (int j = 0; j < ZR; j++) v[j] = Tx[x[j]];
#pragma unroll
  for (int j = 0; j < ZR; j++) {
    a[j] = field::add<F>(v[j], beta);
    v[j] = gp::out_form<F>(v[j], MONT);
  }
  wave_store_zr<true>(o, st, lane, v, r0, us);
#pragma unroll
  for (int j = 0; j < ZR; j++) v[j] = Tx[p0 + j < (uint32_t)TROWS ? p0 + j : 0u];
#pragma unroll
  for (int j = 0; j < ZR; j++) {
    a[j] = p0 + j < us ? LKMUL(a[j], field::add<F>(v[j], gamma)) : field::one<F>();
    v[j] = gp::out_form<F>(v[j], MONT);
  }
  wave_store_zr<true>(o + out_rows * 4, st, lane, v, r0, us);
#pragma unroll
  for (int j = 1; j < ZR; j++) a[j] = LKMUL(a[j - 1], a[j]);
#pragma unroll
  for (int j = 0; j < ZR - 1; j++) v[j] = LKMUL(a[j], sf[j]);
  v[ZR - 1] = a[ZR - 1];
  sN[pz(t)] = a[ZR - 1];
  __syncthreads();
  LKCLK(4);
  if (wv == wn) {
    // the num wave: the exclusive prefix of the 256 num totals, in place
    Fe Pn = sN[pz(e0)];
    sN[pz(e0)] = field::one<F>();
#ifdef B2F_LK_NOSCAN
    if (false)
#endif
#pragma unroll 1
    for (uint32_t k2 = 1; k2 < (uint32_t)ZW; k2++) {
      const Fe e = sN[pz(e0 + k2)];
      sN[pz(e0 + k2)] = Pn;
      Pn = LKMUL(Pn, e);
    }
#ifdef B2F_LK_NOSCAN
    if (false)
#endif
#pragma unroll 1
    for (int off = 1; off < 64; off <<= 1) {
      const Fe y = shfl_fe(Pn, (int)lane - off);
      const Fe m = LKMUL(y, Pn);
      if (lane >= (uint32_t)off) Pn = m;
    }
    Fe Xn = shfl_fe(Pn, (int)lane - 1);
    if (lane == 0) Xn = field::one<F>();
    sN[pz(e0)] = Xn;
#ifdef B2F_LK_NOSCAN
    if (false)
#endif
#pragma unroll 1
    for (uint32_t k2 = 1; k2 < (uint32_t)ZW; k2++) sN[pz(e0 + k2)] = LKMUL(Xn, sN[pz(e0 + k2)]);
  } else if (wv == wd) {
    // the den wave: the look-back over the blocks after b. Lane i watches block q0 + i's status
    // word; the blocks up to the first inclusive one (fi) must all have published, then their
    // values are read and multiplied.
    Fe after = field::one<F>();
#ifdef B2F_LK_NOWAIT  // diagnostics (wrong z): no look-back, to time what waiting for it costs
    if (false) {
#else
    if (b + 1 < nb) {
#endif
      uint64_t q0 = b + 1;
      while (true) {
        const uint64_t qb = q0 + lane;
        const uint32_t s = qb < nb ? (uint32_t)lb_load(lbs + ((uint64_t)c * nb + qb) * LBS_WORDS + 15) : 2u;
        const uint64_t inc = __ballot(s == 2), none = __ballot(s == 0);
        const uint32_t fi = inc ? (uint32_t)__builtin_ctzll(inc) : 64u;
        const uint64_t need = fi >= 63 ? ~0ull : ((2ull << fi) - 1);
        LKCLK(10);
#ifdef B2F_LK_CLOCK
        {
          const uint32_t s0 = __shfl((int)s, 0, 64);
          if (lane == 0) {
            atomicAdd(&g_lk_clock[15], 1ull);                         // polls
            if (s0 == 0) atomicAdd(&g_lk_clock[16], 1ull);            // ... with block b + 1 unpublished
            else if (none & need) atomicAdd(&g_lk_clock[17], 1ull);  // ... with a farther block unpublished
          }
        }
#endif
        if (none & need) {
          __builtin_amdgcn_s_sleep(8);
          continue;
        }
        Fe val = field::one<F>();
        bool ok = true;
        if (lane <= fi && qb < nb) ok = lb_read(lbs + ((uint64_t)c * nb + qb) * LBS_WORDS, s, val);
        if (__ballot(!ok)) {
#ifdef B2F_LK_CLOCK
          if (lane == 0) atomicAdd(&g_lk_clock[18], 1ull);  // status seen before its pieces
#endif
          __builtin_amdgcn_s_sleep(2);
          continue;
        }
        // the product of lanes 0 .. min(fi, 63) (the others hold 1) into lane 0
#pragma unroll 1
        for (uint32_t m = 1; m <= fi && m < 64; m <<= 1) val = LKMUL(val, shfl_xor_fe(val, (int)m));
        after = LKMUL(after, shfl_fe(val, 0));
#ifdef B2F_LK_CLOCK
        if (lane == 0) atomicAdd(&g_lk_clock[7], (unsigned long long)fi + 1);  // blocks looked at
#endif
        if (fi < 64) break;
        q0 += 64;
      }
    }
    LKCLK(9);
    const Fe incl = LKMUL(sDb, after);
    lb_publish(my, lane, incl, 2);
    if (lane == 0 && b == 0) {
      // the den product of the permuted columns against the num side's D
      const Fe dn = Dnum[c];
      uint32_t diff = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) diff |= dn.w[i] ^ incl.w[i];
      if (diff && sticky) atomicOr(sticky, 1 << B2F_ERR_CHECK);
      field::store(o + 4 * out_rows * 4, gp::out_form<F>(field::one<F>(), MONT));  // z[0] = 1
    }
    // the block's factor NK_b Dafter_b (Nbefore_b D^-1 Dafter_b) rides on the den side's
    // exclusive values, so a lane's K is one product: (num prefix) (den suffix)
    const Fe X = LKMUL(sX[lane], LKMUL(NK[(uint64_t)c * nb + b], after));
    sD[atd(e0)] = X;
#ifdef B2F_LK_NOSCAN
    if (false)
#endif
#pragma unroll 1
    for (uint32_t k2 = 1; k2 < (uint32_t)ZW; k2++) sD[atd(e0 + k2)] = LKMUL(X, sD[atd(e0 + k2)]);
  }
  __syncthreads();
  LKCLK(5);
  // 4. z
  const Fe K = LKMUL(sN[pz(t)], sD[pz(t)]);
#pragma unroll
  for (int j = 0; j < ZR; j++) v[j] = gp::out_form<F>(LKMUL(K, v[j]), MONT);
  wave_store_zr<true>(o + 4 * out_rows * 4 + 4, st, lane, v, r0, us);
  LKCLK(6);
  LKCLK_END
}

struct Carve {
  Fe* Tx;
  uint64_t* key;   // 4 x TROWS canonical limbs
  uint64_t* kout;  // TROWS
  uint32_t* perm;   // TROWS: the sort's input (x), then the rank order (lk_tie_fix_kernel)
  uint32_t* perm2;  // TROWS: the sort's output (by top limb)
  uint32_t* count;  // group x TROWS
  uint32_t* pos;
  uint32_t* dcnt;
  uint32_t* lrank;   // group x TROWS: the table indices of the ranks with leftover items, compacted
  uint32_t* lstart;  // group x TROWS: their first leftover index
  uint32_t* samp;    // group x 2 x SAMPLE: pos and lstart samples
  uint32_t* nlr;     // group: ranks with leftovers
  uint32_t* blk;     // group x nb x BLK_WORDS: lk_block_kernel's windows
  uint32_t* part;  // group x SC_PARTS x 3 (rank-scan part totals)
  Fe* partA;  // group x nb: block num products, the A part
  Fe* partS;  // nb: the S part (every circuit's)
  Fe* NK;     // group x nb: Nbefore_b D^-1
  Fe* Dnum;   // group: D from the num side
  Fe* bg;     // beta, gamma in Montgomery form
  uint64_t* lbs;     // group x nb x LBS_WORDS look-back state, then the ticket counter
  void* sort_tmp;
  size_t sort_bytes;
  size_t lbs_bytes;
  size_t total;
};

size_t sort_temp_bytes() {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs((void*)nullptr, bytes, (uint64_t*)nullptr, (uint64_t*)nullptr,
                                  (uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)TROWS, 0, 64);
  return bytes;
}

Carve carve(void* base, uint32_t group, uint64_t usable) {
  Carve k;
  char* p = (char*)base;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    void* r = p ? p + off : nullptr;
    off += (bytes + 255) & ~(size_t)255;
    return r;
  };
  const uint64_t nb = n_lb(usable);
  k.Tx = (Fe*)take(sizeof(Fe) * TROWS);
  k.key = (uint64_t*)take(8ull * 4 * TROWS);
  k.kout = (uint64_t*)take(8ull * TROWS);
  k.perm = (uint32_t*)take(4ull * TROWS);
  k.perm2 = (uint32_t*)take(4ull * TROWS);
  k.count = (uint32_t*)take(4ull * TROWS * group);
  k.pos = (uint32_t*)take(4ull * TROWS * group);
  k.dcnt = (uint32_t*)take(4ull * TROWS * group);
  k.lrank = (uint32_t*)take(4ull * TROWS * group);
  k.lstart = (uint32_t*)take(4ull * TROWS * group);
  k.samp = (uint32_t*)take(8ull * SAMPLE * group);
  k.nlr = (uint32_t*)take(4ull * group);
  k.blk = (uint32_t*)take(4ull * BLK_WORDS * nb * group);
  k.part = (uint32_t*)take(16ull * SC_PARTS * group);
  k.partA = (Fe*)take(sizeof(Fe) * nb * group);
  k.partS = (Fe*)take(sizeof(Fe) * nb);
  k.NK = (Fe*)take(sizeof(Fe) * nb * group);
  k.Dnum = (Fe*)take(sizeof(Fe) * group);
  k.bg = (Fe*)take(sizeof(Fe) * 2);
  k.lbs_bytes = 8ull * LBS_WORDS * nb * group + 64;  // + the ticket counter
  k.lbs = (uint64_t*)take(k.lbs_bytes);
  k.sort_bytes = sort_temp_bytes();
  k.sort_tmp = take(k.sort_bytes);
  k.total = off;
  return k;
}

#ifndef B2F_LK_SORT_SIDE
#define B2F_LK_SORT_SIDE 1  // 0 (variant): table pass + sort on the main stream before the count pass
#endif
// A third stream for the table pass and its sort (run_lookup)
struct SortSide {
  hipStream_t s3;
  hipEvent_t tab, sorted;
};

template <class F>
hipError_t run_lookup(const uint32_t* d_advice, uint64_t total_rows, const uint64_t* d_row_begin,
                      uint32_t n_circuits, uint64_t usable_rows, const Chal& ch, bool mont,
                      uint64_t* d_out, uint64_t out_rows, uint64_t* d_first_bad, void* scratch,
                      uint32_t group, int* sticky, const gp::Side& side, const SortSide& ss, hipStream_t s) {
  Carve k = carve(scratch, group, usable_rows);
  const uint64_t nb = n_lb(usable_rows);
#ifdef B2F_DIAG
  {
    const uint32_t corrupt = getenv("B2F_DIAG_LK_CORRUPT") ? 1u : 0u;
    hipError_t e0 = hipMemcpyToSymbol(HIP_SYMBOL(g_lk_corrupt), &corrupt, sizeof(corrupt));
    if (e0 != hipSuccess) return e0;
  }
#endif
  const dim3 tb(TROWS / 256);
  hipError_t e;
  // The table values, their rank order (a radix sort by the top limb, then ties ordered by the
  // lower limbs) and the per-circuit count pass are independent: the table pass and the sort run
  // on a third stream beside the count pass (the sort is six small rocprim launches, ~60 us of
  // latency on the main stream before round 6), and the num side's block products start as soon
  // as the table values exist, beside both (profiles/r06d_lookup_timeline.txt).
  hipStream_t st = B2F_LK_SORT_SIDE ? ss.s3 : s;
  if (B2F_LK_SORT_SIDE) {
    if ((e = hipEventRecord(side.fork, s)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(st, side.fork, 0)) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(lk_table_kernel<F>, tb, dim3(256), 0, st, ch, k.Tx, k.key, k.perm, k.bg);
  if ((e = hipEventRecord(ss.tab, st)) != hipSuccess) return e;
  {
    size_t bytes = k.sort_bytes;
    e = rocprim::radix_sort_pairs(k.sort_tmp, bytes, k.key + 3ull * TROWS, k.kout, k.perm, k.perm2,
                                  (size_t)TROWS, 0, 63, st);
    if (e != hipSuccess) return e;
  }
  // the tie fix reads the sort's order (perm2) and writes the final one over the sort's input
  hipLaunchKernelGGL(lk_tie_fix_kernel, tb, dim3(256), 0, st, k.key, k.kout, k.perm2, k.perm);
  uint32_t* pa = k.perm;
  if ((e = hipEventRecord(ss.sorted, st)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(d_first_bad, 0xff, 8ull * n_circuits, s)) != hipSuccess) return e;
  // Per group: the num side (block products, their prefix, D and D^-1) on the side stream,
  // forked at the group's start (after the previous group's z pass, which read the same NK
  // slots; the first group's after the table pass), beside the count and rank-scan passes; then
  // the z pass over all the group's circuits (a workgroup count that fills the chip).
  for (uint32_t c0 = 0; c0 < n_circuits; c0 += group) {
    const uint32_t g = n_circuits - c0 < group ? n_circuits - c0 : group;
    if (c0 == 0) {
      if (!B2F_LK_SORT_SIDE && (e = hipEventRecord(side.fork, s)) != hipSuccess) return e;
      if ((e = hipStreamWaitEvent(side.s2, side.fork, 0)) != hipSuccess) return e;
      if ((e = hipStreamWaitEvent(side.s2, ss.tab, 0)) != hipSuccess) return e;
    } else {
      if ((e = hipEventRecord(side.fork, s)) != hipSuccess) return e;
      if ((e = hipStreamWaitEvent(side.s2, side.fork, 0)) != hipSuccess) return e;
    }
    hipLaunchKernelGGL(lk_npart_kernel<F>, dim3((uint32_t)((nb + 4 * NP_BPW - 1) / (4 * NP_BPW)), g + (c0 == 0 ? 1 : 0)), dim3(256), 0,
                       side.s2, d_advice, total_rows, d_row_begin, c0, g, usable_rows, nb, k.Tx, ch, k.partA,
                       k.partS);
    hipLaunchKernelGGL(lk_nscan_kernel<F>, dim3(g), dim3(NS_T), 0, side.s2, nb, k.partA, k.partS, k.NK, k.Dnum,
                       sticky);
    if ((e = hipEventRecord(side.join, side.s2)) != hipSuccess) return e;
    hipLaunchKernelGGL(lk_count_kernel, dim3(CNT_SPLIT, g), dim3(CNT_THREADS), 0, s, d_advice,
                       total_rows, d_row_begin, c0, usable_rows, k.count, d_first_bad);
    if (c0 == 0 && B2F_LK_SORT_SIDE && (e = hipStreamWaitEvent(s, ss.sorted, 0)) != hipSuccess) return e;
    hipLaunchKernelGGL(lk_scan_sums, dim3(SC_PARTS, g), dim3(SC_THREADS), 0, s, pa, k.count, usable_rows, k.part);
    hipLaunchKernelGGL(lk_scan_write, dim3(SC_PARTS, g), dim3(SC_THREADS), 0, s, pa, k.count, usable_rows,
                       k.part, k.pos, k.dcnt, k.lrank, k.lstart, k.samp, k.nlr);
    hipLaunchKernelGGL(lk_block_kernel, dim3((uint32_t)((nb + BK_T - 1) / BK_T), g), dim3(BK_T), 0, s, usable_rows,
                       nb, k.pos, k.dcnt, k.lstart, k.samp, k.nlr, k.blk);
    if ((e = hipMemsetAsync(k.lbs, 0, 8ull * LBS_WORDS * nb * g + 64, s)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(s, side.join, 0)) != hipSuccess) return e;
    uint32_t* ticket = reinterpret_cast<uint32_t*>(k.lbs + LBS_WORDS * nb * g);
    hipLaunchKernelGGL((mont ? lk_zpass_kernel<F, true> : lk_zpass_kernel<F, false>), dim3((uint32_t)(nb * g)),
                       dim3(ZT), 0, s, d_advice, total_rows, d_row_begin, c0, g, usable_rows, nb, k.Tx, pa,
                       d_out, out_rows, ch, k.pos, k.dcnt, k.lrank, k.lstart, k.blk, k.nlr, k.NK, k.Dnum, k.bg, k.lbs, ticket, sticky);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

#ifdef B2F_LK_CLOCK
extern "C" __attribute__((visibility("default"))) int b2f_debug_lk_clock(uint64_t* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lk_clock), sizeof(g_lk_clock)) != hipSuccess) return B2F_ERR_HIP;
  unsigned long long zero[24] = {};
  zero[13] = ~0ull;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_lk_clock), zero, sizeof(zero)) == hipSuccess ? B2F_OK : B2F_ERR_HIP;
}
#endif

size_t lookup_scratch_bytes(uint32_t group, uint64_t usable_rows) {
  return carve(nullptr, group, usable_rows).total;
}

hipError_t launch_lookup(const uint32_t* d_advice, uint64_t total_rows,
                         const uint64_t* d_row_begin, uint32_t n_circuits, uint64_t usable_rows,
                         const uint64_t* theta, const uint64_t* beta, const uint64_t* gamma,
                         uint32_t form, uint64_t* d_out, uint64_t out_rows, uint64_t* d_first_bad,
                         void* scratch, uint32_t group, int* sticky, hipStream_t s2,
                         hipEvent_t ev_fork, hipEvent_t ev_join, hipStream_t s3, hipEvent_t ev_tab,
                         hipEvent_t ev_sorted, hipStream_t s) {
  const gp::Side side{s2, ev_fork, ev_join};
  const SortSide ss{s3, ev_tab, ev_sorted};
  Chal ch;
  for (int i = 0; i < 4; i++) {
    ch.theta[i] = theta[i];
    ch.beta[i] = beta[i];
    ch.gamma[i] = gamma[i];
  }
  const bool mont = (form & 1u) != 0;
  if (form >> 1)
    return run_lookup<field::Bn254>(d_advice, total_rows, d_row_begin, n_circuits, usable_rows, ch,
                                    mont, d_out, out_rows, d_first_bad, scratch, group, sticky, side, ss, s);
  return run_lookup<field::Pallas>(d_advice, total_rows, d_row_begin, n_circuits, usable_rows, ch,
                                   mont, d_out, out_rows, d_first_bad, scratch, group, sticky, side, ss, s);
}

}  // namespace b2f

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
//     likely -- ordered by the lower limbs), giving the rank order x_of_rank[r] and
//     Ts[r] = T[x_of_rank[r]];
//   count:   histogram of the dense cell (a_1) over the circuit's rows (LDS-privatised, four
//            workgroups per circuit, a quarter of the bins each), with the row check (tag,
//            dense, spread) in table (first failing row reported);
//   scan:    in rank order, run starts pos[r] (exclusive prefix of counts), D[r] (runs up to
//            and including r) and LP[r] (exclusive prefix of leftover table multiplicities), 16
//            workgroups per circuit (part totals, then each part's scan);
//   permute: row p of A' is Ts[r] for the run r holding p (binary search of pos); a run
//            start gets S'[p] = Ts[r]; the j-th repeated row gets leftover item L - 1 - j
//            (halo2 hands leftovers out in ascending order, each to the last open repeated
//            row), found by binary search of LP;
//   z:       the permute pass also writes each row's factors num = (A + beta)(S + gamma) and
//            den = (A' + beta)(S' + gamma); the grand product over them (b2f_gprod.h: one
//            inversion per circuit, 4 products per row) writes the z column.
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
                         hipEvent_t ev_fork, hipEvent_t ev_join, hipStream_t s);

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
                                                       uint32_t* __restrict__ perm) {
  const uint32_t x = blockIdx.x * 256 + threadIdx.x;
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

// After one radix sort by the top 64-bit limb of the canonical value: a run of equal top limbs
// (about 2^-33 likely for 2^16 uniform values, but possible) is put in order by the three lower
// limbs, in place, by the thread at the run's start (insertion sort). The rank order is then the
// order of the full 256-bit values, as four LSD passes over the limbs would give.
__global__ __launch_bounds__(256) void lk_tie_fix_kernel(const uint64_t* __restrict__ key,
                                                         const uint64_t* __restrict__ top,
                                                         uint32_t* __restrict__ perm) {
  const uint32_t r = blockIdx.x * 256 + threadIdx.x;
  const uint64_t k = top[r];
  if ((r > 0 && top[r - 1] == k) || r + 1 >= TROWS || top[r + 1] != k) return;
  uint32_t e = r + 1;
  while (e < TROWS && top[e] == k) e++;
  auto less = [&](uint32_t a, uint32_t b) {
    for (int l = 2; l >= 0; l--) {
      const uint64_t x = key[(uint64_t)l * TROWS + a], y = key[(uint64_t)l * TROWS + b];
      if (x != y) return x < y;
    }
    return false;
  };
  for (uint32_t i = r + 1; i < e; i++) {
    const uint32_t v = perm[i];
    uint32_t j = i;
    while (j > r && less(v, perm[j - 1])) {
      perm[j] = perm[j - 1];
      j--;
    }
    perm[j] = v;
  }
}

__global__ __launch_bounds__(256) void lk_rank_kernel(const Fe* __restrict__ Tx,
                                                      const uint32_t* __restrict__ perm,
                                                      Fe* __restrict__ Ts) {
  const uint32_t r = blockIdx.x * 256 + threadIdx.x;
  Ts[r] = Tx[perm[r]];
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
// before it and scans its own ranks. (One 1,024-thread workgroup per circuit holding 64 ranks per
// thread kept the gathered counts in scratch and used 64 of the 256 CUs.)
constexpr int SAMPLE = TROWS / 16;  // every 16th pos / lp entry, for the permute searches
constexpr int SC_PARTS = 16, SC_THREADS = 256, SC_PER = TROWS / (SC_PARTS * SC_THREADS);
static_assert(SC_PER == 16, "one search sample per thread");

// the counts of this thread's SC_PER ranks (rank order read as 16-byte vectors), the index of the
// rank holding table row 0 (-1: none), and the three sums: rows, runs, leftover table multiplicity
struct RankRun {
  uint32_t nv[SC_PER];
  int iz;
  uint32_t sc, sd, sl;
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
    R.iz = x.x == 0 ? 4 * i : x.y == 0 ? 4 * i + 1 : x.z == 0 ? 4 * i + 2 : x.w == 0 ? 4 * i + 3 : R.iz;
  }
  R.sc = R.sd = R.sl = 0;
#pragma unroll
  for (int i = 0; i < SC_PER; i++) {
    const uint32_t n = R.nv[i];
    R.sc += n;
    R.sd += n ? 1u : 0u;
    R.sl += (i == R.iz ? mult0 : 1u) - (n ? 1u : 0u);
  }
  return R;
}

__global__ __launch_bounds__(SC_THREADS) void lk_scan_sums(const uint32_t* __restrict__ perm,
                                                           const uint32_t* __restrict__ count,
                                                           uint64_t usable, uint32_t* __restrict__ part) {
  const uint32_t pt = blockIdx.x, c = blockIdx.y, t = threadIdx.x;
  const uint32_t mult0 = (uint32_t)(usable - TROWS + 1);  // table row 0 fills the rest
  const RankRun R = rank_run(perm, count + (uint64_t)c * TROWS, (pt * SC_THREADS + t) * SC_PER, mult0);
  __shared__ uint32_t s[3][SC_THREADS];
  s[0][t] = R.sc;
  s[1][t] = R.sd;
  s[2][t] = R.sl;
  __syncthreads();
  for (uint32_t w = SC_THREADS / 2; w > 0; w >>= 1) {
    if (t < w) {
      s[0][t] += s[0][t + w];
      s[1][t] += s[1][t + w];
      s[2][t] += s[2][t + w];
    }
    __syncthreads();
  }
  if (t < 3) part[((uint64_t)c * SC_PARTS + pt) * 3 + t] = s[t][0];
}

__global__ __launch_bounds__(SC_THREADS) void lk_scan_write(const uint32_t* __restrict__ perm,
                                                            const uint32_t* __restrict__ count,
                                                            uint64_t usable, const uint32_t* __restrict__ part,
                                                            uint32_t* __restrict__ pos, uint32_t* __restrict__ dcnt,
                                                            uint32_t* __restrict__ lp, uint32_t* __restrict__ samp) {
  const uint32_t pt = blockIdx.x, c = blockIdx.y, t = threadIdx.x;
  const uint32_t mult0 = (uint32_t)(usable - TROWS + 1);
  const uint32_t r0 = (pt * SC_THREADS + t) * SC_PER;
  const RankRun R = rank_run(perm, count + (uint64_t)c * TROWS, r0, mult0);
  uint32_t bc = 0, bd = 0, bl = 0;  // totals of the parts before this one
  for (uint32_t q = 0; q < pt; q++) {
    const uint32_t* pq = part + ((uint64_t)c * SC_PARTS + q) * 3;
    bc += pq[0];
    bd += pq[1];
    bl += pq[2];
  }
  __shared__ uint32_t s[3][SC_THREADS];
  s[0][t] = R.sc;
  s[1][t] = R.sd;
  s[2][t] = R.sl;
  __syncthreads();
  uint32_t ic = R.sc, id = R.sd, il = R.sl;
  for (uint32_t off = 1; off < SC_THREADS; off <<= 1) {  // inclusive Hillis-Steele
    uint32_t a = 0, b = 0, d = 0;
    if (t >= off) {
      a = s[0][t - off];
      b = s[1][t - off];
      d = s[2][t - off];
    }
    __syncthreads();
    ic += a;
    id += b;
    il += d;
    s[0][t] = ic;
    s[1][t] = id;
    s[2][t] = il;
    __syncthreads();
  }
  uint32_t ec = bc + ic - R.sc, ed = bd + id - R.sd, el = bl + il - R.sl;  // exclusive
  uint4* P4 = reinterpret_cast<uint4*>(pos + (uint64_t)c * TROWS + r0);
  uint4* D4 = reinterpret_cast<uint4*>(dcnt + (uint64_t)c * TROWS + r0);
  uint4* L4 = reinterpret_cast<uint4*>(lp + (uint64_t)c * TROWS + r0);
  samp[(uint64_t)c * 2 * SAMPLE + (r0 >> 4)] = ec;  // r0 is a multiple of 16: a search sample
  samp[(uint64_t)c * 2 * SAMPLE + SAMPLE + (r0 >> 4)] = el;
#pragma unroll
  for (int i = 0; i < SC_PER / 4; i++) {
    uint32_t pq[4], dq[4], lq[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t n = R.nv[4 * i + j];
      const uint32_t m = (4 * i + j == R.iz ? mult0 : 1u) - (n ? 1u : 0u);  // leftovers
      pq[j] = ec;
      ed += n ? 1u : 0u;
      dq[j] = ed;
      lq[j] = el;
      ec += n;
      el += m;
    }
    P4[i] = make_uint4(pq[0], pq[1], pq[2], pq[3]);
    D4[i] = make_uint4(dq[0], dq[1], dq[2], dq[3]);
    L4[i] = make_uint4(lq[0], lq[1], lq[2], lq[3]);
  }
}

// The grand product's den total D before the permute pass: A' is a permutation of A and S' one
// of S (the leftover items are exactly the table rows no run start took, row 0 with its
// usable - 2^16 + 1 multiplicity), so D = prod_p den_p = prod_p num_p = prod_p (A_p + beta) *
// prod_p (S_p + gamma). lk_dtot_kernel forms both from the rows -- A_p = Tx[dense cell] and
// S_p = Tx[p] (row 0's value past the table) -- one product per row: workgroups (pt, c < g) the
// A part of circuit c, workgroups (pt, g) the S part (the same for every circuit); lk_dinv
// multiplies the partial products and inverts D. All on the side stream, beside the count, scan
// and permute passes, so no inversion waits in front of gp_write. (A power per histogram bin,
// (Tx[x] + beta)^count[x], ran lanes of one wave through different exponents: 362 us beside
// the permute pass, r04n.) Rows bin by their low 16 bits in every pass, so the identity holds
// whether or not every row is in the table, and D = 0 still flags a zero factor.
constexpr int DP_PARTS = 16, DP_THREADS = 256;
template <class F>
__global__ __launch_bounds__(DP_THREADS) void lk_dtot_kernel(const uint32_t* __restrict__ adv, uint64_t total_rows,
                                                             const uint64_t* __restrict__ row_begin, uint32_t c0,
                                                             uint32_t g, uint64_t usable, const Fe* __restrict__ Tx,
                                                             Chal ch, Fe* __restrict__ part) {
  const uint32_t pt = blockIdx.x, c = blockIdx.y, t = threadIdx.x;
  const bool s_part = c == g;
  const Fe add = field::to_mont<F>(field::load_words(s_part ? ch.gamma : ch.beta));
  const Circ k = s_part ? Circ{0, 0} : circ(row_begin, total_rows, usable, c0 + c);
  const uint64_t per = (usable + DP_PARTS - 1) / DP_PARTS;
  const uint64_t b = (uint64_t)pt * per, e = b + per < usable ? b + per : usable;
  Fe acc = field::one<F>();
  // four rows per step: their cell and table loads issued together, then two independent products
  for (uint64_t p = b + t; p < e; p += 4 * DP_THREADS) {
    uint32_t x[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint64_t q = p + (uint64_t)u * DP_THREADS;
      x[u] = s_part ? (q < (uint64_t)TROWS ? (uint32_t)q : 0u)
                    : (q < k.n_in ? (adv[total_rows + k.first + q] & 0xffffu) : 0u);
    }
    Fe v[4];
#pragma unroll
    for (int u = 0; u < 4; u++)
      v[u] = p + (uint64_t)u * DP_THREADS < e ? field::add<F>(Tx[x[u]], add) : field::one<F>();
    acc = field::mul<F>(acc, field::mul<F>(field::mul<F>(v[0], v[1]), field::mul<F>(v[2], v[3])));
  }
  __shared__ Fe sp[DP_THREADS];
  for (uint32_t w = DP_THREADS / 2; w > 0; w >>= 1) {
    if (t >= w && t < 2 * w) sp[t] = acc;
    __syncthreads();
    if (t < w) acc = field::mul<F>(acc, sp[t + w]);
    __syncthreads();
  }
  if (t == 0) part[(uint64_t)c * DP_PARTS + pt] = acc;
}
// D_c = prod_i (A part i of c) (S part i), a tree over the DP_PARTS pairs, then D^-1 in place (one
// lane: gp::gp_inv's zero check and issue priority)
template <class F>
__global__ __launch_bounds__(DP_PARTS) void lk_dinv_kernel(const Fe* __restrict__ part, uint32_t g,
                                                           Fe* __restrict__ dt, int* __restrict__ sticky) {
  const uint32_t c = blockIdx.x, t = threadIdx.x;
  __shared__ Fe sp[DP_PARTS];
  Fe d = field::mul<F>(part[(uint64_t)c * DP_PARTS + t], part[(uint64_t)g * DP_PARTS + t]);
  for (uint32_t w = DP_PARTS / 2; w > 0; w >>= 1) {
    if (t >= w && t < 2 * w) sp[t] = d;
    __syncthreads();
    if (t < w) d = field::mul<F>(d, sp[t + w]);
    __syncthreads();
  }
  if (t != 0) return;
  __builtin_amdgcn_s_setprio(3);
  if (sticky && field::is_zero(d)) atomicOr(sticky, 1 << B2F_ERR_FIELD);
  dt[c] = field::inv_kaliski<F>(d);
}

// last index r with a[r] <= v (a nondecreasing over TROWS entries, a[0] <= v): the top 12
// levels of the search over the workgroup's LDS sample s[k] = a[16 k], then the 16 entries
// of that block (one 64-byte line, four loads in flight at once) in registers.
__device__ __forceinline__ uint32_t last_le(const uint32_t* __restrict__ a, const uint32_t* s,
                                            uint32_t v) {
  uint32_t lo = 0, hi = SAMPLE;  // last k with s[k] <= v, in [lo, hi)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (s[mid] <= v) lo = mid; else hi = mid;
  }
  const uint4* blk = reinterpret_cast<const uint4*>(a + 16 * lo);
  const uint4 q0 = blk[0], q1 = blk[1], q2 = blk[2], q3 = blk[3];
  const uint32_t e[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                          q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
  uint32_t n = 0;  // entries <= v (e[0] = s[lo] <= v; nondecreasing)
#pragma unroll
  for (int i = 1; i < 16; i++) n += e[i] <= v ? 1u : 0u;
  return 16 * lo + n;
}

#ifndef B2F_LK_NT
#define B2F_LK_NT 3  // non-temporal stores: 1 the columns, 2 the factors, 3 both (permute pass
                     // 552 us write-back, 546 columns only, 358 both: the write-back lines
                     // evicted the gathered tables)
#endif
// The four columns and the grand product's factors, a lane per row (grid-stride over 64-row
// groups): A = Tx[x], S = Tx[p] (row 0's value past the table), A' = Ts[r] for the run r holding
// p (binary search of pos: the top 12 levels in the workgroup's LDS sample), S' = A' at a run
// start, else leftover item L - 1 - j for the j-th repeated row (halo2 hands leftovers out in
// ascending order, each to the last open repeated row), found by binary search of LP. Each
// column's 64 values of a wave go out as 1 KiB non-temporal stores (gp::wave_store_rows), the
// factors to their chunk-interleaved slots (gp::wave_store_slots). Measured the searches cost
// about what a separate rank-expansion pass (run-start / leftover marks and wave max-scans)
// did, so they stay: r04e, 1.319 vs 1.321-1.332 ms per call.
template <class F>
__global__ __launch_bounds__(256) void lk_permute_kernel(
    const uint32_t* __restrict__ adv, uint64_t total_rows, const uint64_t* __restrict__ row_begin,
    uint32_t c0, uint64_t usable, const Fe* __restrict__ Tx, const Fe* __restrict__ Ts,
    bool mont, uint64_t* __restrict__ out, uint64_t out_rows, Chal ch, Fe* __restrict__ num,
    Fe* __restrict__ den, const uint32_t* __restrict__ pos, const uint32_t* __restrict__ dcnt,
    const uint32_t* __restrict__ lp, const uint32_t* __restrict__ samp) {
  __shared__ uint4 stage[4][128];
  const uint32_t c = blockIdx.y, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  __shared__ uint32_t sP[SAMPLE], sL[SAMPLE];
  {
    const uint4* sa = reinterpret_cast<const uint4*>(samp + (uint64_t)c * 2 * SAMPLE);
    uint4* sp4 = reinterpret_cast<uint4*>(sP);
    uint4* sl4 = reinterpret_cast<uint4*>(sL);
    for (uint32_t i = threadIdx.x; i < (uint32_t)SAMPLE / 4; i += 256) {
      sp4[i] = sa[i];
      sl4[i] = sa[SAMPLE / 4 + i];
    }
  }
  __syncthreads();
  uint4* st = stage[wv];
  const Fe beta = field::to_mont<F>(field::load_words(ch.beta));
  const Fe gamma = field::to_mont<F>(field::load_words(ch.gamma));
  Fe* nm = num + (uint64_t)c * gp::elems(usable);
  Fe* dn = den + (uint64_t)c * gp::elems(usable);
  const Circ k = circ(row_begin, total_rows, usable, c0 + c);
  const uint32_t* P = pos + (uint64_t)c * TROWS;
  const uint32_t* D = dcnt + (uint64_t)c * TROWS;
  const uint32_t* L = lp + (uint64_t)c * TROWS;
  const uint32_t n_left = (uint32_t)usable - D[TROWS - 1];  // repeated rows = leftover items
  uint64_t* o = out + (uint64_t)(c0 + c) * 5 * out_rows * 4;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t base = (uint64_t)blockIdx.x * 256 + 64 * wv; base < usable; base += stride) {
    const uint64_t p = base + lane;
    const bool in = p < usable;
    const uint32_t nv = (uint32_t)(usable - base < 64 ? usable - base : 64);
    const uint32_t x = p < k.n_in ? (adv[total_rows + k.first + p] & 0xffffu) : 0u;
    uint2 r = make_uint2(0u, 0u);  // ranks of A'[p] and S'[p]
    if (in) {
      r.x = last_le(P, sP, (uint32_t)p);
      r.y = P[r.x] == (uint32_t)p ? r.x : last_le(L, sL, n_left - 1u - ((uint32_t)p - D[r.x]));
    }
#ifndef B2F_LK_ABL
#define B2F_LK_ABL 0  // diagnostics (variant builds only): 1 no gathers, 2 no products, 4 no column stores
#endif
#if B2F_LK_ABL & 1
    Fe a = beta, sv = gamma, ap = beta, sp = gamma;
    a.w[0] ^= x; sv.w[0] ^= (uint32_t)p; ap.w[0] ^= r.x; sp.w[0] ^= r.y;
#else
    const Fe a = Tx[x];
    const Fe sv = Tx[p < (uint64_t)TROWS ? (uint32_t)p : 0u];
    const Fe ap = Ts[r.x];
    const Fe sp = Ts[r.y];
#endif
    if (!(B2F_LK_ABL & 4)) {
      gp::wave_store_rows<B2F_LK_NT & 1>(o + 4 * base, st, lane, out_form<F>(a, mont), nv);
      gp::wave_store_rows<B2F_LK_NT & 1>(o + (out_rows + base) * 4, st, lane, out_form<F>(sv, mont), nv);
      gp::wave_store_rows<B2F_LK_NT & 1>(o + (2 * out_rows + base) * 4, st, lane, out_form<F>(ap, mont), nv);
      gp::wave_store_rows<B2F_LK_NT & 1>(o + (3 * out_rows + base) * 4, st, lane, out_form<F>(sp, mont), nv);
    }
    // the grand product's factors (A + beta)(S + gamma) / ((A' + beta)(S' + gamma)); rows past
    // `usable` land in slots of the last tile that the grand product never reads
    const uint64_t sb = (base / (gp::ZC * gp::ZC)) * (gp::ZC * gp::ZC) + (base / gp::ZC) % gp::ZC;
    if (B2F_LK_ABL & 2) {
      gp::wave_store_slots<(B2F_LK_NT >> 1) & 1>(nm + sb, st, lane, field::add<F>(field::add<F>(a, beta), field::add<F>(sv, gamma)));
      gp::wave_store_slots<(B2F_LK_NT >> 1) & 1>(dn + sb, st, lane, field::add<F>(field::add<F>(ap, beta), field::add<F>(sp, gamma)));
    } else {
      gp::wave_store_slots<(B2F_LK_NT >> 1) & 1>(nm + sb, st, lane, field::mul<F>(field::add<F>(a, beta), field::add<F>(sv, gamma)));
      gp::wave_store_slots<(B2F_LK_NT >> 1) & 1>(dn + sb, st, lane, field::mul<F>(field::add<F>(ap, beta), field::add<F>(sp, gamma)));
    }
  }
}

using gp::ZC;

struct Carve {
  Fe* Tx;
  Fe* Ts;
  uint64_t* key;   // 4 x TROWS canonical limbs
  uint64_t* kout;  // TROWS
  uint32_t* perm;  // TROWS
  uint32_t* perm2;
  uint32_t* count;  // group x TROWS
  uint32_t* pos;
  uint32_t* dcnt;
  uint32_t* lp;
  uint32_t* samp;  // group x 2 x SAMPLE
  uint32_t* part;  // group x SC_PARTS x 3 (rank-scan part totals)
  Fe* num;  // group x usable
  Fe* den;
  Fe* zs;  // group x gp::scratch_elems
  Fe* dpart;  // (group + 1) x DP_PARTS (lk_dtot_kernel)
  void* sort_tmp;
  size_t sort_bytes;
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
  k.Tx = (Fe*)take(sizeof(Fe) * TROWS);
  k.Ts = (Fe*)take(sizeof(Fe) * TROWS);
  k.key = (uint64_t*)take(8ull * 4 * TROWS);
  k.kout = (uint64_t*)take(8ull * TROWS);
  k.perm = (uint32_t*)take(4ull * TROWS);
  k.perm2 = (uint32_t*)take(4ull * TROWS);
  k.count = (uint32_t*)take(4ull * TROWS * group);
  k.pos = (uint32_t*)take(4ull * TROWS * group);
  k.dcnt = (uint32_t*)take(4ull * TROWS * group);
  k.lp = (uint32_t*)take(4ull * TROWS * group);
  k.samp = (uint32_t*)take(8ull * SAMPLE * group);
  k.part = (uint32_t*)take(12ull * SC_PARTS * group);
  k.num = (Fe*)take(sizeof(Fe) * gp::elems(usable) * group);  // chunk-interleaved (b2f_gprod.h)
  k.den = (Fe*)take(sizeof(Fe) * gp::elems(usable) * group);
  k.zs = (Fe*)take(sizeof(Fe) * gp::scratch_elems(usable) * group);
  k.dpart = (Fe*)take(sizeof(Fe) * DP_PARTS * (group + 1));
  k.sort_bytes = sort_temp_bytes();
  k.sort_tmp = take(k.sort_bytes);
  k.total = off;
  return k;
}

template <class F>
hipError_t run_lookup(const uint32_t* d_advice, uint64_t total_rows, const uint64_t* d_row_begin,
                      uint32_t n_circuits, uint64_t usable_rows, const Chal& ch, bool mont,
                      uint64_t* d_out, uint64_t out_rows, uint64_t* d_first_bad, void* scratch,
                      uint32_t group, int* sticky, const gp::Side& side, hipStream_t s) {
  Carve k = carve(scratch, group, usable_rows);
  const dim3 tb(TROWS / 256);
  hipLaunchKernelGGL(lk_table_kernel<F>, tb, dim3(256), 0, s, ch, k.Tx, k.key, k.perm);
  // one radix sort by the top limb of the canonical value (< 2^63: both moduli are < 2^255),
  // then ties in the top limb ordered by the lower limbs
  uint32_t* pa = k.perm2;
  {
    size_t bytes = k.sort_bytes;
    hipError_t e = rocprim::radix_sort_pairs(k.sort_tmp, bytes, k.key + 3ull * TROWS, k.kout, k.perm, pa,
                                             (size_t)TROWS, 0, 63, s);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(lk_tie_fix_kernel, tb, dim3(256), 0, s, k.key, k.kout, pa);
  hipLaunchKernelGGL(lk_rank_kernel, tb, dim3(256), 0, s, k.Tx, pa, k.Ts);
  hipError_t e = hipMemsetAsync(d_first_bad, 0xff, 8ull * n_circuits, s);
  if (e != hipSuccess) return e;
  // Per group: the count / scan / permute passes over all its circuits at once (a workgroup
  // count per circuit that fills the chip), then the grand products. The den totals' inverses
  // D^-1 come from the rows on the side stream (lk_dtot_kernel, lk_dinv_kernel), forked at the
  // group's start (after the previous group's gp_write, which read the same D^-1 slots), so the
  // inversions' latency hides behind the count, scan and permute passes. (r04m: with D taken from
  // the den chunk totals, each half of the group's inversion still held its gp_write 25-52 us
  // after two-way pipelining, 1.24-1.27 ms per call.)
  for (uint32_t c0 = 0; c0 < n_circuits; c0 += group) {
    const uint32_t g = n_circuits - c0 < group ? n_circuits - c0 : group;
    const gp::Scratch zk = gp::scratch_of(k.zs, g, usable_rows);
    if ((e = hipEventRecord(side.fork, s)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(side.s2, side.fork, 0)) != hipSuccess) return e;
    hipLaunchKernelGGL(lk_dtot_kernel<F>, dim3(DP_PARTS, g + 1), dim3(DP_THREADS), 0, side.s2, d_advice,
                       total_rows, d_row_begin, c0, g, usable_rows, k.Tx, ch, k.dpart);
    hipLaunchKernelGGL(lk_dinv_kernel<F>, dim3(g), dim3(DP_PARTS), 0, side.s2, k.dpart, g, zk.dt, sticky);
    if ((e = hipEventRecord(side.join, side.s2)) != hipSuccess) return e;
    hipLaunchKernelGGL(lk_count_kernel, dim3(CNT_SPLIT, g), dim3(CNT_THREADS), 0, s, d_advice,
                       total_rows, d_row_begin, c0, usable_rows, k.count, d_first_bad);
    hipLaunchKernelGGL(lk_scan_sums, dim3(SC_PARTS, g), dim3(SC_THREADS), 0, s, pa, k.count, usable_rows, k.part);
    hipLaunchKernelGGL(lk_scan_write, dim3(SC_PARTS, g), dim3(SC_THREADS), 0, s, pa, k.count, usable_rows,
                       k.part, k.pos, k.dcnt, k.lp, k.samp);
    // permute: ~4096 rows per workgroup
    const uint32_t px = (uint32_t)((usable_rows + 4095) / 4096);
    hipLaunchKernelGGL(lk_permute_kernel<F>, dim3(px, g), dim3(256), 0, s, d_advice, total_rows,
                       d_row_begin, c0, usable_rows, k.Tx, k.Ts, mont, d_out, out_rows, ch, k.num,
                       k.den, k.pos, k.dcnt, k.lp, k.samp);
    e = gp::run_begin<F>(g, usable_rows, k.num, k.den, k.zs, sticky, side, s, false, true);
    if (e == hipSuccess)
      e = gp::run_end<F>(g, usable_rows, mont, d_out + ((uint64_t)c0 * 5 + 4) * out_rows * 4, 5 * out_rows * 4,
                         k.num, k.den, k.zs, nullptr, nullptr, s, nullptr, side);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

size_t lookup_scratch_bytes(uint32_t group, uint64_t usable_rows) {
  return carve(nullptr, group, usable_rows).total;
}

hipError_t launch_lookup(const uint32_t* d_advice, uint64_t total_rows,
                         const uint64_t* d_row_begin, uint32_t n_circuits, uint64_t usable_rows,
                         const uint64_t* theta, const uint64_t* beta, const uint64_t* gamma,
                         uint32_t form, uint64_t* d_out, uint64_t out_rows, uint64_t* d_first_bad,
                         void* scratch, uint32_t group, int* sticky, hipStream_t s2,
                         hipEvent_t ev_fork, hipEvent_t ev_join, hipStream_t s) {
  const gp::Side side{s2, ev_fork, ev_join};
  Chal ch;
  for (int i = 0; i < 4; i++) {
    ch.theta[i] = theta[i];
    ch.beta[i] = beta[i];
    ch.gamma[i] = gamma[i];
  }
  const bool mont = (form & 1u) != 0;
  if (form >> 1)
    return run_lookup<field::Bn254>(d_advice, total_rows, d_row_begin, n_circuits, usable_rows, ch,
                                    mont, d_out, out_rows, d_first_bad, scratch, group, sticky, side, s);
  return run_lookup<field::Pallas>(d_advice, total_rows, d_row_begin, n_circuits, usable_rows, ch,
                                   mont, d_out, out_rows, d_first_bad, scratch, group, sticky, side, s);
}

}  // namespace b2f

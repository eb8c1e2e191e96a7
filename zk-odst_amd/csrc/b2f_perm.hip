// b2f_perm.hip -- permutation-argument prover columns of the equality columns a_1..a_8
// (table16.rs:312-314; halo2_proofs 0.3.0 plonk/permutation: keygen.rs Assembly::copy +
// build_pk's permutation polynomials, prover.rs commit; restated in oracle/permutation.py).
//
// One circuit = whole instances of a batch, circuit row = trace row - the first instance's
// offset. Keygen's cycle structure comes from the structure alone and is the same for every
// instance of a given `rounds`: the host replays halo2's Assembly::copy over one instance's
// copy list (b2f_kernels.hip, perm_mapping) and this file expands the resulting mapping
// pattern over the circuit:
//   sigma_j(w^i) = delta^c' w^r'   with (c', r') = mapping[j][i] (identity off the cycles);
//   for each set of chunk_len columns, the grand product with
//     num_i = prod_j (v_j(i) + beta delta^j w^i + gamma),
//     den_i = prod_j (v_j(i) + beta sigma_j(w^i) + gamma),
//   z[0] = the previous set's last z (1 for the first), z[i + 1] = z[i] num_i / den_i
//   (b2f_gprod.h), rows 0 .. usable (the blinding rows after it are the prover's).
// delta^c w^r = OL[c][r mod 1024] OH[r / 1024]: two table reads and one product per value
// (OL, BL = beta OL: 8 x 1024 entries; OH: 2^k / 1024 entries), built per call.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/b2f.h"
#include "b2f_field.h"
#include "b2f_gprod.h"

namespace b2f {

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

namespace {

using field::Fe;
constexpr int NCOL = 8;    // equality columns a_1..a_8, permutation column j = a_{j+1}
constexpr int LO = 1024;   // low table
constexpr uint32_t ROW_BITS = 29;  // mapping entries: (column << 29) | instance-relative row

struct Params {
  uint64_t omega[4], delta[4], beta[4], gamma[4];
};

template <class F>
__device__ Fe pow_u64(Fe b, uint64_t e) {
  Fe r = field::one<F>();
  while (e) {
    if (e & 1) r = field::mul<F>(r, b);
    b = field::mul<F>(b, b);
    e >>= 1;
  }
  return r;
}

// OL[c][lo] = delta^c w^lo, BL[c][lo] = beta OL[c][lo] (c < 8, lo < 1024); OH[h] = w^(1024 h);
// G = gamma (Montgomery form, converted once here rather than per row)
template <class F>
__global__ __launch_bounds__(256) void pm_table_kernel(Params prm, uint64_t n_hi, Fe* __restrict__ OL,
                                                       Fe* __restrict__ BL, Fe* __restrict__ OH,
                                                       Fe* __restrict__ G) {
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i == 0) G[0] = field::to_mont<F>(field::load_words(prm.gamma));
  const Fe w = field::to_mont<F>(field::load_words(prm.omega));
  if (i < (uint64_t)NCOL * LO) {
    const uint32_t c = (uint32_t)(i / LO), lo = (uint32_t)(i % LO);
    const Fe d = field::to_mont<F>(field::load_words(prm.delta));
    const Fe b = field::to_mont<F>(field::load_words(prm.beta));
    const Fe v = field::mul<F>(pow_u64<F>(d, c), pow_u64<F>(w, lo));
    OL[i] = v;
    BL[i] = field::mul<F>(b, v);
  }
  if (i < n_hi) OH[i] = pow_u64<F>(pow_u64<F>(w, LO), i);
}

// the instance holding circuit row r: last i with start[i] <= r (start[0] = 0 <= r), n if
// r >= start[n]
__device__ __forceinline__ uint32_t inst_of(const uint64_t* __restrict__ start, uint32_t n, uint64_t r) {
  if (r >= start[n]) return n;
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (start[mid] <= r) lo = mid; else hi = mid;
  }
  return lo;
}

// d_inst: per instance (circuit start row, pool offset of its rounds' pattern), n + 1 starts
struct Inst {
  const uint64_t* start;  // n + 1
  const uint64_t* pat;    // n: pool offset (u32 units) of the [8][R] pattern
  uint32_t n;
};

// the instance holding row r of a wave whose first row is `base` (wave-uniform: one search per
// wave, scalar loads), then a lane's forward steps past the instance starts up to its row (an
// instance has at least 228 rows, so a 64-row wave crosses at most one start)
__device__ __forceinline__ uint32_t inst_of_wave(const Inst& I, uint64_t base, uint64_t r) {
  uint32_t ii = __builtin_amdgcn_readfirstlane(inst_of(I.start, I.n, base));
  while (ii < I.n && I.start[ii + 1] <= r) ii++;
  return ii;
}

// mapping of cell (j, r) -> circuit (c', r')
__device__ __forceinline__ void mapped(const Inst& I, const uint32_t* __restrict__ pool, uint32_t ii,
                                       uint32_t j, uint64_t r, uint32_t& c2, uint64_t& r2) {
  if (ii >= I.n) {
    c2 = j;
    r2 = r;
    return;
  }
  const uint64_t s = I.start[ii], R = I.start[ii + 1] - s;
  const uint32_t m = pool[I.pat[ii] + j * R + (r - s)];
  c2 = m >> ROW_BITS;
  r2 = s + (m & ((1u << ROW_BITS) - 1));
}

template <class F>
__device__ __forceinline__ Fe dw(const Fe* __restrict__ T, const Fe* __restrict__ OH, uint32_t c,
                                 uint64_t r) {
  return field::mul<F>(T[c * LO + (uint32_t)(r & (LO - 1))], OH[r >> 10]);
}

// sigma_j(w^r) for every row r < 2^k (keygen: the permutation polynomials' values); a wave per
// 64 rows, each column's 64 values stored through LDS as 1 KiB runs (gp::wave_store_rows)
template <class F>
__global__ __launch_bounds__(256) void pm_sigma_kernel(Inst I, const uint32_t* __restrict__ pool,
                                                       uint64_t n_rows, const Fe* __restrict__ OL,
                                                       const Fe* __restrict__ OH, bool mont,
                                                       uint64_t* __restrict__ out, uint64_t out_rows) {
  __shared__ uint4 stage[4][128];
  const uint32_t lane = threadIdx.x & 63u, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t base = (uint64_t)blockIdx.x * 256 + 64 * wv;
  if (base >= n_rows) return;
  const uint64_t r = base + lane;
  const uint32_t nv = (uint32_t)(n_rows - base < 64 ? n_rows - base : 64);
  const uint64_t rr = r < n_rows ? r : base;
  const uint32_t ii = inst_of_wave(I, base, rr);
#pragma unroll 1
  for (uint32_t j = 0; j < NCOL; j++) {
    uint32_t c2;
    uint64_t r2;
    mapped(I, pool, ii, j, rr, c2, r2);
    gp::wave_store_rows<true>(out + ((uint64_t)j * out_rows + base) * 4, stage[wv], lane,
                              gp::out_form<F>(dw<F>(OL, OH, c2, r2), mont), nv);
  }
}

// num/den of every column set for rows r < usable: a wave per 64 rows (the instance lookup and
// the cell loads shared by the sets), the factors stored through LDS to their slots
// (gp::wave_store_slots, non-temporal)
template <class F>
__global__ __launch_bounds__(256) void pm_factor_kernel(Inst I, const uint32_t* __restrict__ pool,
                                                        const uint32_t* __restrict__ adv,
                                                        uint64_t total_rows, uint64_t row0,
                                                        uint64_t usable, uint32_t chunk_len,
                                                        const Fe* __restrict__ BL,
                                                        const Fe* __restrict__ OH, const Fe* __restrict__ G,
                                                        Fe* __restrict__ num, Fe* __restrict__ den) {
  __shared__ uint4 stage[4][128];
  const uint32_t lane = threadIdx.x & 63u, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t base = (uint64_t)blockIdx.x * 256 + 64 * wv;
  if (base >= usable) return;
  const uint64_t r0 = base + lane;
  const uint64_t r = r0 < usable ? r0 : base;  // lanes past the end repeat row base (slots unused)
  const uint32_t set = blockIdx.y;  // column set: columns [j0, j1)
  const uint32_t j0 = set * chunk_len, j1 = j0 + chunk_len < (uint32_t)NCOL ? j0 + chunk_len : NCOL;
  num += (uint64_t)set * gp::elems(usable);
  den += (uint64_t)set * gp::elems(usable);
  const Fe gamma = G[0];
  const uint32_t ii = inst_of_wave(I, base, r);
  const uint64_t used = I.start[I.n];
  Fe n, d;  // the first column's factors, then one product per further column
#pragma unroll 1
  for (uint32_t j = j0; j < j1; j++) {
    // advice column a_{j+1}; cells past the circuit's instances are unassigned (zero)
    const uint32_t x = r < used ? adv[(uint64_t)(j + 1) * total_rows + row0 + r] : 0u;
    const Fe vg = field::add<F>(field::from_u32<F>(x), gamma);
    uint32_t c2;
    uint64_t r2;
    mapped(I, pool, ii, j, r, c2, r2);
    const Fe fn = field::add<F>(vg, dw<F>(BL, OH, j, r));
    // a cell on no copy cycle maps to itself (about 2/3 of the cells): sigma = delta^j w^r
    const Fe fd = (c2 == j && r2 == r) ? fn : field::add<F>(vg, dw<F>(BL, OH, c2, r2));
    n = j == j0 ? fn : field::mul<F>(n, fn);
    d = j == j0 ? fd : field::mul<F>(d, fd);
  }
  const uint64_t sb = gp::slot_base64(base);
  gp::wave_store_slots<true>(num + sb, stage[wv], lane, n);
  gp::wave_store_slots<true>(den + sb, stage[wv], lane, d);
}

constexpr uint32_t PM_CL = 3;  // pm_chunk_kernel's column sets: chunk_len <= 3 (halo2's usual 3)
// waves per SIMD pm_chunk_kernel is compiled for: BN254 fits 4 (119 VGPRs, no scratch; 147 at
// the default budget, 3 waves); pasta's form spills at 128, so it keeps 3
template <class F> struct PmWaves { static constexpr int v = 3; };
#ifndef B2F_PM_WAVES_BN254
#define B2F_PM_WAVES_BN254 4
#endif
template <> struct PmWaves<field::Bn254> { static constexpr int v = B2F_PM_WAVES_BN254; };
// The factors fused with the grand product's chunk pass (replaces pm_factor_kernel + gp_chunk):
// a lane per 16-row chunk walks its rows -- per row the set's num / den factors as
// pm_factor_kernel forms them, the running num prefix Nloc written over num and the den factor
// to den (gp::slot_of, non-temporal) -- then the workgroup's block scan (gp::block_scan). The
// factors never make the round trip through HBM that pm_factor_kernel -> gp_chunk took (64
// bytes written, 64 read and 32 rewritten per row and set).
template <class F>
__global__ __launch_bounds__(gp::BLK) __attribute__((amdgpu_waves_per_eu(PmWaves<F>::v))) void pm_chunk_kernel(Inst I, const uint32_t* __restrict__ pool,
                                                           const uint32_t* __restrict__ adv,
                                                           uint64_t total_rows, uint64_t row0,
                                                           uint64_t usable, uint32_t chunk_len,
                                                           const Fe* __restrict__ BL,
                                                           const Fe* __restrict__ OH,
                                                           const Fe* __restrict__ G,
                                                           Fe* __restrict__ num, Fe* __restrict__ den,
                                                           Fe* __restrict__ zs) {
  __shared__ Fe sn[gp::BLK], sd[gp::BLK];
  const uint32_t t = threadIdx.x, set = blockIdx.y, sets = gridDim.y;
  const uint32_t j0 = set * chunk_len, j1 = j0 + chunk_len < (uint32_t)NCOL ? j0 + chunk_len : NCOL;
  const uint64_t nq = gp::n_chunks(usable), nb = gp::n_blocks(usable);
  const gp::Scratch k = gp::scratch_of(zs, sets, usable);
  Fe* nm = num + (uint64_t)set * gp::elems(usable);
  Fe* dn = den + (uint64_t)set * gp::elems(usable);
  const uint64_t q = (uint64_t)blockIdx.x * gp::BLK + t;
  const Fe gamma = G[0];
  const uint64_t used = I.start[I.n];
  Fe pn = field::one<F>(), pd = field::one<F>();
  {
    // the wave's first row -> its instance (one search per wave), then this lane's first row
    const uint64_t wq = __builtin_amdgcn_readfirstlane((uint32_t)(blockIdx.x * gp::BLK + (t & ~63u)));
    const uint64_t rb = q * gp::ZC, re = rb + gp::ZC < usable ? rb + gp::ZC : usable;
    uint32_t ii = inst_of_wave(I, wq * gp::ZC < usable ? wq * gp::ZC : 0, rb < usable ? rb : 0);
    // the lane's instance context, refreshed when its rows cross an instance start (an instance
    // has >= 228 rows, so at most once per chunk)
    uint64_t s_lo = ~0ull, s_hi = ~0ull, pat = 0;
    if (ii < I.n) {
      s_lo = I.start[ii];
      s_hi = I.start[ii + 1];
      pat = I.pat[ii];
    }
    // one row's loads (the set's cells and mapping entries), issued a row ahead of their use:
    // a lane walks its 16 rows in order, so without the prefetch every row waited for its loads
    struct RowIn {
      uint32_t x[PM_CL], m[PM_CL];
    };
#define PM_FETCH(v, rr)                                                                          \
    do {                                                                                         \
      const uint64_t r_ = (rr);                                                                  \
      if (r_ >= s_hi && ii < I.n) {                                                              \
        ii++;                                                                                    \
        s_lo = s_hi;                                                                             \
        if (ii < I.n) {                                                                          \
          s_hi = I.start[ii + 1];                                                                \
          pat = I.pat[ii];                                                                       \
        } else {                                                                                 \
          s_lo = s_hi = ~0ull;                                                                   \
        }                                                                                        \
      }                                                                                          \
      _Pragma("unroll") for (uint32_t jj = 0; jj < PM_CL; jj++) {                                \
        const uint32_t j_ = j0 + jj < j1 ? j0 + jj : j0;                                         \
        v.x[jj] = r_ < used ? adv[(uint64_t)(j_ + 1) * total_rows + row0 + r_] : 0u;             \
        v.m[jj] = ii < I.n ? pool[pat + j_ * (s_hi - s_lo) + (r_ - s_lo)]                        \
                           : (j_ << ROW_BITS) | 0x1fffffffu;                                     \
      }                                                                                          \
    } while (0)
    RowIn cur;
    PM_FETCH(cur, rb < usable ? rb : 0);
    uint64_t cur_lo = s_lo;
#pragma unroll 1
    for (uint64_t r = rb; r < re; r++) {
      RowIn nxt;
      PM_FETCH(nxt, r + 1 < re ? r + 1 : r);
      const uint64_t nxt_lo = s_lo;
      Fe n = field::one<F>(), d = field::one<F>();
#pragma unroll
      for (uint32_t jj = 0; jj < PM_CL; jj++) {
        const uint32_t j = j0 + jj;
        if (j >= j1) continue;  // a shorter last set (uniform)
        const Fe vg = field::add<F>(field::from_u32<F>(cur.x[jj]), gamma);
        // the mapping entry (c' << 29 | instance-relative r'), or the identity past the instances
        const uint32_t mm = cur.m[jj];
        const bool ident_enc = (mm & 0x1fffffffu) == 0x1fffffffu;
        const uint32_t c2 = ident_enc ? j : mm >> ROW_BITS;
        const uint64_t r2 = ident_enc ? r : cur_lo + (mm & ((1u << ROW_BITS) - 1));
#ifdef B2F_PM_NOIDENT  // diagnostics (results wrong): no identity coset product
        const Fe fn = vg;
#else
        const Fe fn = field::add<F>(vg, dw<F>(BL, OH, j, r));
#endif
#ifdef B2F_PM_NOSIGMA  // diagnostics (results wrong): no sigma product, as if sigma were loaded
        const Fe fd = (c2 == j && r2 == r) ? fn : vg;
#else
        const Fe fd = (c2 == j && r2 == r) ? fn : field::add<F>(vg, dw<F>(BL, OH, c2, r2));
#endif
        n = jj == 0 ? fn : field::mul<F>(n, fn);
        d = jj == 0 ? fd : field::mul<F>(d, fd);
      }
      pn = r == rb ? n : field::mul<F>(pn, n);
      pd = r == rb ? d : field::mul<F>(pd, d);
      const uint64_t sl = gp::slot_of(r, nq);
      uint4* pnp = reinterpret_cast<uint4*>(nm + sl);
      uint4* dnp = reinterpret_cast<uint4*>(dn + sl);
      gp::nt_store(pnp, make_uint4(pn.w[0], pn.w[1], pn.w[2], pn.w[3]));
      gp::nt_store(pnp + 1, make_uint4(pn.w[4], pn.w[5], pn.w[6], pn.w[7]));
      gp::nt_store(dnp, make_uint4(d.w[0], d.w[1], d.w[2], d.w[3]));
      gp::nt_store(dnp + 1, make_uint4(d.w[4], d.w[5], d.w[6], d.w[7]));
      cur = nxt;
      cur_lo = nxt_lo;
    }
#undef PM_FETCH
  }
  gp::block_scan<F>(sn, sd, t, q, nq, nb, set, pn, pd, k.zn, k.zd, k.tn, k.td);
}

struct Carve {
  Fe* OL;
  Fe* BL;
  Fe* OH;
  Fe* num;
  Fe* den;
  Fe* zs;
  Fe* seed;  // chained grand products: closing values and seeds, NCOL each
  Fe* gm;    // gamma, Montgomery form
  size_t total;
};

// num, den and the grand-product scratch hold one slice per column set: ceil(8 / chunk_len)
// of them (3 for halo2's usual chunk_len 3), not one per column
Carve carve(void* base, uint32_t k, uint64_t usable, uint32_t sets) {
  Carve m;
  char* p = (char*)base;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    void* r = p ? p + off : nullptr;
    off += (bytes + 255) & ~(size_t)255;
    return r;
  };
  const uint64_t n_hi = ((1ull << k) + LO - 1) / LO;
  m.OL = (Fe*)take(sizeof(Fe) * NCOL * LO);
  m.BL = (Fe*)take(sizeof(Fe) * NCOL * LO);
  m.OH = (Fe*)take(sizeof(Fe) * n_hi);
  m.num = (Fe*)take(sizeof(Fe) * gp::elems(usable) * sets);
  m.den = (Fe*)take(sizeof(Fe) * gp::elems(usable) * sets);
  m.zs = (Fe*)take(sizeof(Fe) * gp::scratch_elems(usable) * sets);
  m.seed = (Fe*)take(sizeof(Fe) * 2 * sets);
  m.gm = (Fe*)take(sizeof(Fe));
  m.total = off;
  return m;
}

template <class F>
hipError_t run_perm(const uint32_t* d_advice, uint64_t total_rows, uint64_t row0, const Inst& I,
                    const uint32_t* d_pool, uint32_t k, uint64_t usable, const Params& prm,
                    const uint64_t* gamma, uint32_t chunk_len, bool mont, uint64_t* d_sigma,
                    uint64_t* d_z, uint64_t out_rows, void* scratch, int* sticky, gp::Side side,
                    hipStream_t s) {
  const uint32_t sets = (NCOL + chunk_len - 1) / chunk_len;
  Carve m = carve(scratch, k, usable, sets);
  const uint64_t n_rows = 1ull << k, n_hi = n_rows / LO;
  const uint64_t tab = n_hi > (uint64_t)NCOL * LO ? n_hi : (uint64_t)NCOL * LO;
  hipLaunchKernelGGL(pm_table_kernel<F>, dim3((uint32_t)((tab + 255) / 256)), dim3(256), 0, s, prm,
                     n_hi, m.OL, m.BL, m.OH, m.gm);
  // every column set's factors in one launch, then their grand products side by side, chained
  // (set c starts where set c - 1 closed); the sigma columns go between the two halves of the
  // grand product, beside its inversions on the side stream
#ifdef B2F_PM_SEPARATE  // diagnostics: the factor pass and gp_chunk as two launches
  const bool fused = false;
#else
  const bool fused = chunk_len <= PM_CL;  // longer column sets: the two-launch form
#endif
  if (fused)
    hipLaunchKernelGGL(pm_chunk_kernel<F>, dim3((uint32_t)gp::n_blocks(usable), sets), dim3(gp::BLK), 0, s,
                       I, d_pool, d_advice, total_rows, row0, usable, chunk_len, m.BL, m.OH, m.gm, m.num,
                       m.den, m.zs);
  else
    hipLaunchKernelGGL(pm_factor_kernel<F>, dim3((uint32_t)((usable + 255) / 256), sets), dim3(256), 0, s,
                       I, d_pool, d_advice, total_rows, row0, usable, chunk_len, m.BL, m.OH, m.gm, m.num,
                       m.den);
  hipError_t e = gp::run_begin<F>(sets, usable, m.num, m.den, m.zs, sticky, side, s, fused);
  if (e != hipSuccess) return e;
  if (d_sigma)
    hipLaunchKernelGGL(pm_sigma_kernel<F>, dim3((uint32_t)((n_rows + 255) / 256)), dim3(256), 0, s, I,
                       d_pool, n_rows, m.OL, m.OH, mont, d_sigma, out_rows);
  e = gp::run_end<F>(sets, usable, mont, d_z, out_rows * 4, m.num, m.den, m.zs, nullptr, nullptr, s,
                     m.seed, side);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}

// keygen: the sigma columns alone (the tables they read, then pm_sigma_kernel)
template <class F>
hipError_t run_perm_sigma(const Inst& I, const uint32_t* d_pool, uint32_t k, const Params& prm, bool mont,
                          uint64_t* d_sigma, uint64_t out_rows, void* scratch, hipStream_t s) {
  Carve m = carve(scratch, k, 0, 1);
  const uint64_t n_rows = 1ull << k, n_hi = n_rows / LO;
  const uint64_t tab = n_hi > (uint64_t)NCOL * LO ? n_hi : (uint64_t)NCOL * LO;
  hipLaunchKernelGGL(pm_table_kernel<F>, dim3((uint32_t)((tab + 255) / 256)), dim3(256), 0, s, prm,
                     n_hi, m.OL, m.BL, m.OH, m.gm);
  hipLaunchKernelGGL(pm_sigma_kernel<F>, dim3((uint32_t)((n_rows + 255) / 256)), dim3(256), 0, s, I,
                     d_pool, n_rows, m.OL, m.OH, mont, d_sigma, out_rows);
  return hipGetLastError();
}

}  // namespace

size_t perm_sigma_scratch_bytes(uint32_t k) { return carve(nullptr, k, 0, 1).total; }

hipError_t launch_permutation_sigma(const uint64_t* d_inst, size_t n_inst, const uint32_t* d_pool, uint32_t k,
                                    const uint64_t* omega, const uint64_t* delta, uint32_t form,
                                    uint64_t* d_sigma, uint64_t out_rows, void* scratch, hipStream_t s) {
  Params prm;
  for (int i = 0; i < 4; i++) {
    prm.omega[i] = omega[i];
    prm.delta[i] = delta[i];
    prm.beta[i] = i == 0;  // BL (beta times the coset table) is not used by the sigma pass
    prm.gamma[i] = 0;
  }
  Inst I;
  I.start = d_inst;
  I.pat = d_inst + n_inst + 1;
  I.n = (uint32_t)n_inst;
  const bool mont = (form & 1u) != 0;
  if (form >> 1) return run_perm_sigma<field::Bn254>(I, d_pool, k, prm, mont, d_sigma, out_rows, scratch, s);
  return run_perm_sigma<field::Pallas>(I, d_pool, k, prm, mont, d_sigma, out_rows, scratch, s);
}

size_t perm_scratch_bytes(uint32_t k, uint64_t usable_rows, size_t, uint32_t chunk_len) {
  return carve(nullptr, k, usable_rows, (NCOL + chunk_len - 1) / chunk_len).total;
}

// d_inst: n + 1 circuit start rows, then n pool offsets
hipError_t launch_permutation(const uint32_t* d_advice, uint64_t total_rows, uint64_t row0,
                              const uint64_t* d_inst, size_t n_inst, const uint32_t* d_pool,
                              uint32_t k, uint64_t usable_rows, const uint64_t* omega,
                              const uint64_t* delta, const uint64_t* beta, const uint64_t* gamma,
                              uint32_t chunk_len, uint32_t form, uint64_t* d_sigma, uint64_t* d_z,
                              uint64_t out_rows, void* scratch, int* sticky, hipStream_t s2,
                              hipEvent_t ev_fork, hipEvent_t ev_join, hipStream_t s) {
  const gp::Side side{s2, ev_fork, ev_join};
  Params prm;
  for (int i = 0; i < 4; i++) {
    prm.omega[i] = omega[i];
    prm.delta[i] = delta[i];
    prm.beta[i] = beta[i];
    prm.gamma[i] = gamma[i];
  }
  Inst I;
  I.start = d_inst;
  I.pat = d_inst + n_inst + 1;
  I.n = (uint32_t)n_inst;
  const bool mont = (form & 1u) != 0;
  if (form >> 1)
    return run_perm<field::Bn254>(d_advice, total_rows, row0, I, d_pool, k, usable_rows, prm, gamma,
                                  chunk_len, mont, d_sigma, d_z, out_rows, scratch, sticky, side, s);
  return run_perm<field::Pallas>(d_advice, total_rows, row0, I, d_pool, k, usable_rows, prm, gamma,
                                 chunk_len, mont, d_sigma, d_z, out_rows, scratch, sticky, side, s);
}

}  // namespace b2f

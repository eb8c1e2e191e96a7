// b2f_gprod.h -- the grand product z[0] = seed, z[p + 1] = z[p] num_p / den_p over `usable`
// rows, shared by the lookup argument (halo2_proofs 0.3.0 lookup/prover.rs commit_product,
// seed 1) and the permutation argument (permutation/prover.rs commit, seed = the previous
// column set's last z).
//
// z[p + 1] = seed N_p / D_p with N_p, D_p the prefix products through row p, and
// D_p^-1 = D^-1 prod_{i > p} den_i: ONE inversion per product (of the whole den product D),
// the rest prefix and suffix products. Three passes over ZC-row chunks (one lane walks one
// chunk):
//   gp_chunk:  the chunk's num prefix Nloc_p (written over num in place), the chunk totals of
//              num and den (2 products per row);
//   gp_scan:   K_q = seed N_before(q) D_end(q)^-1 per chunk, the inversion, and the closing
//              value seed N / D (= z[usable]) for a next product. Up to SCAN_THREADS x 4
//              chunks one workgroup per product scans them directly; beyond, three levels over
//              blocks of SCAN_THREADS chunks (gp_block_reduce: block totals; gp_scan over the
//              block totals; gp_block_down: in-block exclusive prefix / suffix combined with the
//              block's K), so the serial run per lane stays short at any size;
//   gp_write:  backward over the chunk: z[p + 1] = K_q Nloc_p prod_{p < i < e} den_i
//              (2 products per row), converted to the output form.
// Products are independent along blockIdx.y: product y reads num/den + y * elems(usable) and
// writes z column z_base + y * z_stride (u64 units, 4 per element).
#pragma once
#include "b2f_field.h"

namespace b2f {
namespace gp {
namespace {

using field::Fe;

constexpr uint32_t ZC = 16;           // rows per chunk
constexpr int SCAN_THREADS = 1024;    // one workgroup per product

__host__ __device__ inline uint64_t n_chunks(uint64_t usable) { return (usable + ZC - 1) / ZC; }

// num / den are stored chunk-interleaved: row p of a product at (p mod ZC) * nq + p / ZC, so
// that the lanes of a wave (consecutive chunks) walking their chunks read consecutive
// elements at every step -- a row-major layout put the lanes 512 bytes apart and turned each
// 32-byte read into a 128-byte line fetch. Writers (the factor passes) place rows this way;
// an array holds ZC * nq elements per product.
__host__ __device__ inline uint64_t slot_of(uint64_t p, uint64_t nq) { return (p % ZC) * nq + p / ZC; }
__host__ __device__ inline uint64_t elems(uint64_t usable) { return n_chunks(usable) * ZC; }

template <class F>
__device__ __forceinline__ Fe out_form(const Fe& a, bool mont) {
  return mont ? a : field::to_canonical<F>(a);
}

template <class F>
__global__ __launch_bounds__(256) void gp_chunk(uint64_t usable, Fe* __restrict__ num,
                                                const Fe* __restrict__ den, Fe* __restrict__ zn,
                                                Fe* __restrict__ zd) {
  const uint32_t c = blockIdx.y;
  const uint64_t nq = n_chunks(usable);
  const uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  Fe* nm = num + (uint64_t)c * elems(usable);
  const Fe* dn = den + (uint64_t)c * elems(usable);
  const uint64_t b = q * ZC, e = b + ZC < usable ? b + ZC : usable;
  Fe pn = nm[q], pd = dn[q];  // row b (slot 0 of chunk q)
  for (uint64_t p = b + 1; p < e; p++) {
    const uint64_t k = slot_of(p, nq);
    pn = field::mul<F>(pn, nm[k]);
    pd = field::mul<F>(pd, dn[k]);
    nm[k] = pn;
  }
  zn[(uint64_t)c * nq + q] = pn;
  zd[(uint64_t)c * nq + q] = pd;
}

// zn[q] <- K_q = seed N_before(q) D_end(q)^-1 with N_before(q) = prod_{q' < q} zn[q'],
// D_end(q)^-1 = D^-1 prod_{q' > q} zd[q']. Per-thread runs of chunks, Hillis-Steele scans
// of the run products in LDS (a prefix for num, a suffix for den), one inversion.
// seed: Montgomery elements per product (nullptr: 1); closing (nullable) <- seed N / D;
// sticky (nullable): the context's sticky error word, B2F_ERR_FIELD set when D = 0.
// T threads: SCAN_THREADS, or one wave when there are at most 64 chunk totals (the block totals
// of the three-level path) -- a 1,024-thread scan of 8 values spent ten levels of products on
// every thread.
template <class F, int T = SCAN_THREADS>
__global__ __launch_bounds__(T) void gp_scan(uint64_t nq, Fe* __restrict__ zn,
                                             const Fe* __restrict__ zd,
                                             const Fe* __restrict__ seed,
                                             Fe* __restrict__ closing, int* __restrict__ sticky) {
  const uint32_t c = blockIdx.x, t = threadIdx.x;
  const uint64_t per = (nq + T - 1) / T;
  __shared__ Fe sn[T], sd[T];
  __shared__ Fe dinv;
  Fe* an = zn + (uint64_t)c * nq;
  const Fe* ad = zd + (uint64_t)c * nq;
  const uint64_t b = t * per < nq ? t * per : nq, e = b + per < nq ? b + per : nq;
  Fe pn = field::one<F>(), pd = field::one<F>();
  for (uint64_t q = b; q < e; q++) {
    pn = field::mul<F>(pn, an[q]);
    pd = field::mul<F>(pd, ad[q]);
  }
  sn[t] = pn;
  sd[t] = pd;
  __syncthreads();
  for (int off = 1; off < T; off <<= 1) {  // inclusive: prefix of sn, suffix of sd
    Fe xn = pn, xd = pd;
    if (t >= (uint32_t)off) xn = field::mul<F>(sn[t - off], pn);
    if (t + off < (uint32_t)T) xd = field::mul<F>(pd, sd[t + off]);
    __syncthreads();
    sn[t] = pn = xn;
    sd[t] = pd = xd;
    __syncthreads();
  }
  const Fe s = seed ? seed[c] : field::one<F>();
  if (t == 0) {
#ifdef B2F_INV_EUCLID  // diagnostics: the plain binary extended Euclid
    dinv = field::inv<F>(sd[0]);  // sd[0] = D
#else
    dinv = field::inv_kaliski<F>(sd[0]);  // sd[0] = D
#endif
    // D = 0: some den factor is zero (a challenge collides with a cell value). halo2's
    // batch_invert would leave that entry zero and the proof would fail; here every z would
    // come from a meaningless inverse, so the call reports B2F_ERR_FIELD at b2f_sync instead.
    if (sticky && field::is_zero(sd[0])) atomicOr(sticky, 1 << B2F_ERR_FIELD);
    if (closing) closing[c] = field::mul<F>(field::mul<F>(s, sn[T - 1]), dinv);
  }
  __syncthreads();
  Fe rd = t + 1 < (uint32_t)T ? field::mul<F>(dinv, sd[t + 1]) : dinv;
  Fe rn = t ? field::mul<F>(s, sn[t - 1]) : s;
  for (uint64_t q = b; q < e; q++) {  // forward: seed times the exclusive num prefix
    const Fe vn = an[q];
    an[q] = rn;
    rn = field::mul<F>(rn, vn);
  }
  for (uint64_t q = e; q-- > b;) {  // backward: K_q
    an[q] = field::mul<F>(an[q], rd);
    rd = field::mul<F>(rd, ad[q]);
  }
}

// block b of product c: the products of its SCAN_THREADS chunks' zn and zd -> tn/td[c][b]
template <class F>
__global__ __launch_bounds__(SCAN_THREADS) void gp_block_reduce(uint64_t nq, const Fe* __restrict__ zn,
                                                                const Fe* __restrict__ zd,
                                                                Fe* __restrict__ tn, Fe* __restrict__ td) {
  const uint32_t b = blockIdx.x, c = blockIdx.y, t = threadIdx.x;
  const uint64_t nb = (nq + SCAN_THREADS - 1) / SCAN_THREADS;
  const uint64_t q = (uint64_t)b * SCAN_THREADS + t;
  __shared__ Fe sn[SCAN_THREADS], sd[SCAN_THREADS];
  Fe pn = q < nq ? zn[(uint64_t)c * nq + q] : field::one<F>();
  Fe pd = q < nq ? zd[(uint64_t)c * nq + q] : field::one<F>();
  for (uint32_t w = SCAN_THREADS / 2; w > 0; w >>= 1) {
    if (t >= w && t < 2 * w) {
      sn[t] = pn;
      sd[t] = pd;
    }
    __syncthreads();
    if (t < w) {
      pn = field::mul<F>(pn, sn[t + w]);
      pd = field::mul<F>(pd, sd[t + w]);
    }
    __syncthreads();
  }
  if (t == 0) {
    tn[(uint64_t)c * nb + b] = pn;
    td[(uint64_t)c * nb + b] = pd;
  }
}

// K_q = KB[b] * (exclusive in-block prefix of zn) * (exclusive in-block suffix of zd), KB[b] the
// block's K from gp_scan over the block totals. Work-efficient: DOWN_T threads, each owning
// DOWN_PER consecutive chunks of the block -- thread totals, a DOWN_T-wide scan of them, then a
// backward pass that leaves each chunk's exclusive zd suffix in zd (not read after this pass) and a
// forward pass that writes K -- about 90 products per thread instead of a 1,024-wide
// Hillis-Steele scan's 22 per chunk.
constexpr int DOWN_T = 64, DOWN_PER = SCAN_THREADS / DOWN_T;
template <class F>
__global__ __launch_bounds__(DOWN_T) void gp_block_down(uint64_t nq, Fe* __restrict__ zn,
                                                        Fe* __restrict__ zd,
                                                        const Fe* __restrict__ kb) {
  const uint32_t b = blockIdx.x, c = blockIdx.y, t = threadIdx.x;
  const uint64_t nb = (nq + SCAN_THREADS - 1) / SCAN_THREADS;
  const uint64_t q0 = (uint64_t)b * SCAN_THREADS + (uint64_t)t * DOWN_PER;
  Fe* an = zn + (uint64_t)c * nq;
  Fe* ad = zd + (uint64_t)c * nq;
  const uint32_t cnt = q0 >= nq ? 0u : (uint32_t)(nq - q0 < DOWN_PER ? nq - q0 : DOWN_PER);
  Fe tn = field::one<F>(), td = field::one<F>();
  for (uint32_t i = 0; i < cnt; i++) {
    tn = field::mul<F>(tn, an[q0 + i]);
    td = field::mul<F>(td, ad[q0 + i]);
  }
  __shared__ Fe sn[DOWN_T], sd[DOWN_T];
  sn[t] = tn;
  sd[t] = td;
  __syncthreads();
  Fe pn = tn, pd = td;
  for (int off = 1; off < DOWN_T; off <<= 1) {  // inclusive prefix of sn, suffix of sd
    Fe xn = pn, xd = pd;
    if (t >= (uint32_t)off) xn = field::mul<F>(sn[t - off], pn);
    if (t + off < (uint32_t)DOWN_T) xd = field::mul<F>(pd, sd[t + off]);
    __syncthreads();
    sn[t] = pn = xn;
    sd[t] = pd = xd;
    __syncthreads();
  }
  if (!cnt) return;
  const Fe k = kb[(uint64_t)c * nb + b];
  Fe e = t ? field::mul<F>(k, sn[t - 1]) : k;                               // KB x thread prefix
  Fe sf = t + 1 < (uint32_t)DOWN_T ? sd[t + 1] : field::one<F>();           // thread suffix
  for (uint32_t i = cnt; i-- > 0;) {  // backward: zd[q] <- exclusive in-block suffix of zd
    const Fe v = ad[q0 + i];
    ad[q0 + i] = sf;
    sf = field::mul<F>(sf, v);
  }
  for (uint32_t i = 0; i < cnt; i++) {  // forward: K_q
    const Fe v = an[q0 + i];
    an[q0 + i] = field::mul<F>(e, ad[q0 + i]);
    e = field::mul<F>(e, v);
  }
}

template <class F>
__global__ __launch_bounds__(256) void gp_write(uint64_t usable, bool mont, uint64_t* __restrict__ z_base,
                                                uint64_t z_stride, const Fe* __restrict__ num,
                                                const Fe* __restrict__ den,
                                                const Fe* __restrict__ zn,
                                                const Fe* __restrict__ seed,
                                                const Fe* __restrict__ post) {
  const uint32_t c = blockIdx.y;
  const uint64_t nq = n_chunks(usable);
  const uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  const Fe* nm = num + (uint64_t)c * elems(usable);  // Nloc, from gp_chunk
  const Fe* dn = den + (uint64_t)c * elems(usable);
  uint64_t* zcol = z_base + (uint64_t)c * z_stride;
  const uint64_t b = q * ZC, e = b + ZC < usable ? b + ZC : usable;
  // post: a factor applied here rather than in the scan (chained products: the seed of
  // product c is only known once the scans of products 0 .. c - 1 are done)
  const Fe s0 = post ? post[c] : (seed ? seed[c] : field::one<F>());
  if (q == 0) field::store(zcol, out_form<F>(s0, mont));
  Fe k = zn[(uint64_t)c * nq + q];
  if (post) k = field::mul<F>(k, post[c]);
  for (uint64_t p = e; p-- > b;) {
    const uint64_t sl = slot_of(p, nq);
    field::store(zcol + 4 * (p + 1), out_form<F>(field::mul<F>(nm[sl], k), mont));
    if (p > b) k = field::mul<F>(k, dn[sl]);
  }
}

// Chained products: S[0] = 1, S[c] = S[c - 1] T[c - 1] with T[c] product c's closing value
// for seed 1 (the permutation argument's column sets: each set's z starts where the previous
// one closed).
template <class F>
__global__ void gp_chain_seeds(const Fe* __restrict__ T, Fe* __restrict__ S, uint32_t g) {
  if (threadIdx.x != 0) return;
  Fe acc = field::one<F>();
  for (uint32_t c = 0; c < g; c++) {
    S[c] = acc;
    acc = field::mul<F>(acc, T[c]);
  }
}

// Scratch (Fe elements) gp::run needs per product: chunk products, and block totals + K.
__host__ __device__ inline uint64_t scratch_elems(uint64_t usable) {
  const uint64_t nq = n_chunks(usable), nb = (nq + SCAN_THREADS - 1) / SCAN_THREADS;
  return 2 * nq + 2 * nb;
}

// The passes for `g` products on `s`. zs: scratch of g * scratch_elems(usable). With `chain`
// (2 g elements of scratch) the products are chained -- product c starts from product c - 1's
// closing value, product 0 from 1 -- and still scanned side by side: their single inversions
// run in parallel, the seeds are applied in gp_write.
template <class F>
hipError_t run(uint32_t g, uint64_t usable, bool mont, uint64_t* z_base, uint64_t z_stride,
               Fe* num, const Fe* den, Fe* zs, const Fe* seed, Fe* closing, hipStream_t s,
               Fe* chain = nullptr, int* sticky = nullptr) {
  Fe* post = nullptr;
  if (chain) {
    seed = nullptr;
    closing = chain;  // T
    post = chain + g;  // S
  }
  const uint64_t nq = n_chunks(usable), nb = (nq + SCAN_THREADS - 1) / SCAN_THREADS;
  Fe* zn = zs;
  Fe* zd = zs + (uint64_t)g * nq;
  Fe* tn = zd + (uint64_t)g * nq;
  Fe* td = tn + (uint64_t)g * nb;
  const uint32_t zq = (uint32_t)((nq + 255) / 256);
  hipLaunchKernelGGL(gp_chunk<F>, dim3(zq, g), dim3(256), 0, s, usable, num, den, zn, zd);
  if (nq <= 64) {
    hipLaunchKernelGGL((gp_scan<F, 64>), dim3(g), dim3(64), 0, s, nq, zn, zd, seed, closing, sticky);
  } else if (nq <= 4ull * SCAN_THREADS) {
    hipLaunchKernelGGL(gp_scan<F>, dim3(g), dim3(SCAN_THREADS), 0, s, nq, zn, zd, seed, closing, sticky);
  } else {
    hipLaunchKernelGGL(gp_block_reduce<F>, dim3((uint32_t)nb, g), dim3(SCAN_THREADS), 0, s, nq, zn, zd,
                       tn, td);
    if (nb <= 64)
      hipLaunchKernelGGL((gp_scan<F, 64>), dim3(g), dim3(64), 0, s, nb, tn, td, seed, closing, sticky);
    else
      hipLaunchKernelGGL(gp_scan<F>, dim3(g), dim3(SCAN_THREADS), 0, s, nb, tn, td, seed, closing, sticky);
    hipLaunchKernelGGL(gp_block_down<F>, dim3((uint32_t)nb, g), dim3(DOWN_T), 0, s, nq, zn, zd, tn);
  }
  if (chain) hipLaunchKernelGGL(gp_chain_seeds<F>, dim3(1), dim3(64), 0, s, chain, post, g);
  hipLaunchKernelGGL(gp_write<F>, dim3(zq, g), dim3(256), 0, s, usable, mont, z_base, z_stride, num,
                     den, zn, seed, post);
  return hipGetLastError();
}

}  // namespace
}  // namespace gp
}  // namespace b2f

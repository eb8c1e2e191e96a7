// b2f_gprod.h -- the grand product z[0] = seed, z[p + 1] = z[p] num_p / den_p over `usable`
// rows, shared by the lookup argument (halo2_proofs 0.3.0 lookup/prover.rs commit_product,
// seed 1) and the permutation argument (permutation/prover.rs commit, seed = the previous
// column set's last z).
//
// z[p + 1] = seed N_p / D_p with N_p, D_p the prefix products through row p, and
// D_p^-1 = D^-1 prod_{i > p} den_i: ONE inversion per product (of the whole den product D),
// the rest prefix and suffix products. Chunks of ZC rows (one lane walks one chunk), blocks of
// BLK chunks (one workgroup):
//   gp_chunk:  the chunk's num prefix Nloc_p (written over num in place) and its num / den
//              totals (2 products per row); then, across the workgroup's BLK chunks, the
//              exclusive prefix of the num totals and exclusive suffix of the den totals (zn /
//              zd per chunk) and the block's totals (tn / td) -- Hillis-Steele in LDS;
//   gp_total:  the den total D from the block totals;
//   gp_inv:    D^-1 (one lane's divsteps inversion, b2f_safegcd.h) and the closing values.
//              It depends only on gp_total, so it runs on a second stream beside the scan;
//   gp_scan:   K'_b = seed N_before(b) prod_{b' > b} D_b' per block (K = K' D^-1) and seed N
//              (the closing value seed N / D = z[usable] before its D^-1);
//   gp_write:  backward over the chunk: z[p + 1] = K'_b zn_q zd_q D^-1 Nloc_p prod_{p < i < e}
//              den_i (2 products per row), converted to the output form and staged through LDS
//              so a wave's stores cover whole 128-byte row groups.
// (Round 3 reduced and down-swept 1,024-chunk blocks in two more passes, 124-151 us per lookup
// call of 64 circuits; the in-block scans now ride in gp_chunk, one product per row more.)
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

// num / den are stored interleaved by tiles of ZC chunks (ZC x ZC rows): row p = ZC q + j of chunk
// q = ZC Q + k sits at ZC^2 Q + ZC j + k. Readers (a lane per chunk, walking j) see 16 consecutive
// chunks' row j as 16 consecutive elements (512 contiguous bytes per 16 lanes); writers (a lane per
// row: the factor passes) see 64 consecutive rows as 16 runs of 4 elements (128-byte lines). Row-
// major put the readers' lanes 512 bytes apart; interleaving over ALL chunks ((p mod ZC) nq + p /
// ZC) put the writers' lanes nq x 32 bytes apart (every 32-byte store a partial line: the lookup's
// permute pass wrote its num / den at a fraction of the bandwidth). An array holds elems(usable)
// elements per product (whole tiles).
__host__ __device__ inline uint64_t slot_of(uint64_t p, uint64_t nq) {
  (void)nq;
  return (p / (ZC * ZC)) * (ZC * ZC) + (p % ZC) * ZC + (p / ZC) % ZC;
}
__host__ __device__ inline uint64_t elems(uint64_t usable) {
  return (usable + ZC * ZC - 1) / (ZC * ZC) * (ZC * ZC);
}

// A wave's 64 consecutive 32-byte elements (lane l holds element l) stored through the wave's
// 2 KiB of LDS (st: 128 x 16 B) so that each store instruction writes 1 KiB contiguous (lane l
// the 16-byte chunk l); a lane storing its own element writes 16 bytes every 32 per instruction.
// NT: non-temporal stores (data no later kernel of the call re-reads soon).
__device__ __forceinline__ void nt_store(uint4* p, const uint4& v) {
  __builtin_nontemporal_store(field::u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<field::u32x4*>(p));
}
template <bool NT>
__device__ __forceinline__ void put16(uint4* p, const uint4& v) {
  if (NT) nt_store(p, v); else *p = v;
}
__device__ __forceinline__ void wave_stage(uint4* st, uint32_t lane, const Fe& v) {
  st[2 * lane] = make_uint4(v.w[0], v.w[1], v.w[2], v.w[3]);
  st[2 * lane + 1] = make_uint4(v.w[4], v.w[5], v.w[6], v.w[7]);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void wave_unstage_done() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}
// elements 0 .. n - 1 of the staged 64 to dst (contiguous)
template <bool NT>
__device__ __forceinline__ void wave_store_rows(uint64_t* dst, uint4* st, uint32_t lane, const Fe& v,
                                                uint32_t n) {
  wave_stage(st, lane, v);
  const uint4 x = st[lane], y = st[64 + lane];
  wave_unstage_done();
  uint4* d = reinterpret_cast<uint4*>(dst);
  if ((lane >> 1) < n) put16<NT>(d + lane, x);
  if (32u + (lane >> 1) < n) put16<NT>(d + 64 + lane, y);
}
// The staged 64 rows base .. base + 63 (base a multiple of 64) to their slot_of slots: 16 runs of
// 4 elements (128 bytes) 512 bytes apart, 8 lanes per run. slots_base = the array + the slot of
// row base. Non-temporal by default: the lookup's permute pass wrote its factors 1.55x faster so
// (552 -> 358 us, the write-back stores' partial lines evicting the gathered tables).
template <bool NT>
__device__ __forceinline__ void wave_store_slots(Fe* slots_base, uint4* st, uint32_t lane, const Fe& v) {
  wave_stage(st, lane, v);
  const uint32_t c = lane & 7u, e = c >> 1, h = c & 1u, r = lane >> 3;
  const uint4 x = st[2 * (16 * e + r) + h], y = st[2 * (16 * e + r + 8) + h];
  wave_unstage_done();
  uint4* d = reinterpret_cast<uint4*>(slots_base);  // element (j * 16 + e), half h
  put16<NT>(d + 2 * (r * 16 + e) + h, x);
  put16<NT>(d + 2 * ((r + 8) * 16 + e) + h, y);
}
__host__ __device__ inline uint64_t slot_base64(uint64_t base) {  // slot of row base (64 | base)
  return (base / (ZC * ZC)) * (ZC * ZC) + (base / ZC) % ZC;
}

template <class F>
__device__ __forceinline__ Fe out_form(const Fe& a, bool mont) {
  return mont ? a : field::to_canonical<F>(a);
}

constexpr int BLK = 256;  // chunks per block = gp_chunk's workgroup
__host__ __device__ inline uint64_t n_blocks(uint64_t usable) { return (n_chunks(usable) + BLK - 1) / BLK; }

// The block scan of gp_chunk: chunk totals pn / pd of the workgroup's BLK chunks -> exclusive
// in-block num prefix (zn) / den suffix (zd) per chunk and the block totals (tn / td). Every
// thread of the workgroup calls it (chunks past the end with the identity).
template <class F>
__device__ __forceinline__ void block_scan(Fe* sn, Fe* sd, uint32_t t, uint64_t q, uint64_t nq, uint64_t nb,
                                           uint32_t c, Fe pn, Fe pd, Fe* __restrict__ zn,
                                           Fe* __restrict__ zd, Fe* __restrict__ tn, Fe* __restrict__ td) {
  // inclusive scans over the block: prefix of the num totals, suffix of the den totals
  sn[t] = pn;
  sd[t] = pd;
  __syncthreads();
  for (int off = 1; off < BLK; off <<= 1) {
    Fe xn = pn, xd = pd;
    if (t >= (uint32_t)off) xn = field::mul<F>(sn[t - off], pn);
    if (t + off < (uint32_t)BLK) xd = field::mul<F>(pd, sd[t + off]);
    __syncthreads();
    sn[t] = pn = xn;
    sd[t] = pd = xd;
    __syncthreads();
  }
  if (q < nq) {
    zn[(uint64_t)c * nq + q] = t ? sn[t - 1] : field::one<F>();
    zd[(uint64_t)c * nq + q] = t + 1 < (uint32_t)BLK ? sd[t + 1] : field::one<F>();
  }
  if (t == 0) {
    tn[(uint64_t)c * nb + blockIdx.x] = sn[BLK - 1];
    td[(uint64_t)c * nb + blockIdx.x] = sd[0];
  }
}

template <class F>
__global__ __launch_bounds__(BLK) void gp_chunk(uint64_t usable, Fe* __restrict__ num,
                                                const Fe* __restrict__ den, Fe* __restrict__ zn,
                                                Fe* __restrict__ zd, Fe* __restrict__ tn,
                                                Fe* __restrict__ td) {
  __shared__ Fe sn[BLK], sd[BLK];
  const uint32_t c = blockIdx.y, t = threadIdx.x;
  const uint64_t nq = n_chunks(usable), nb = n_blocks(usable);
  const uint64_t q = (uint64_t)blockIdx.x * BLK + t;
  Fe pn = field::one<F>(), pd = field::one<F>();  // chunks past the end: the identity
  if (q < nq) {
    Fe* nm = num + (uint64_t)c * elems(usable);
    const Fe* dn = den + (uint64_t)c * elems(usable);
    const uint64_t b = q * ZC, e = b + ZC < usable ? b + ZC : usable;
    pn = nm[slot_of(b, nq)];  // row b
    pd = dn[slot_of(b, nq)];
    // the next row's factors are loaded a row ahead (the prefix store to num would otherwise keep
    // the compiler from hoisting them: same array)
    Fe an = pn, ad = pd;
    if (b + 1 < e) {
      an = nm[slot_of(b + 1, nq)];
      ad = dn[slot_of(b + 1, nq)];
    }
    for (uint64_t p = b + 1; p < e; p++) {
      const uint64_t k = slot_of(p, nq);
      const Fe cn = an, cd = ad;
      if (p + 1 < e) {
        an = nm[slot_of(p + 1, nq)];
        ad = dn[slot_of(p + 1, nq)];
      }
      pn = field::mul<F>(pn, cn);
      pd = field::mul<F>(pd, cd);
      nm[k] = pn;
    }
  }
  block_scan<F>(sn, sd, t, q, nq, nb, c, pn, pd, zn, zd, tn, td);
}

// Over the block totals (zn = tn, zd = td, nq = the block count): zn[b] <- K'_b = seed
// N_before(b) prod_{b' > b} zd[b'] with N_before(b) = prod_{b' < b} zn[b'] (K_b = K'_b D^-1:
// gp_write applies D^-1). Per-thread runs of blocks, Hillis-Steele scans of the run products in
// LDS (a prefix for num, a suffix for den). seed: Montgomery elements per product (nullptr: 1);
// sn[c] <- seed N. T threads: SCAN_THREADS, or one wave for at most 64 blocks (a 1,024-thread
// scan of 8 values spent ten levels of products on every thread).
template <class F, int T = SCAN_THREADS>
__global__ __launch_bounds__(T) void gp_scan(uint64_t nq, Fe* __restrict__ zn,
                                             const Fe* __restrict__ zd,
                                             const Fe* __restrict__ seed,
                                             Fe* __restrict__ sn_out) {
  const uint32_t c = blockIdx.x, t = threadIdx.x;
  const uint64_t per = (nq + T - 1) / T;
  __shared__ Fe sn[T], sd[T];
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
  if (t == 0) sn_out[c] = field::mul<F>(s, sn[T - 1]);  // seed N (the closing value before D^-1)
  Fe rd = t + 1 < (uint32_t)T ? sd[t + 1] : field::one<F>();
  Fe rn = t ? field::mul<F>(s, sn[t - 1]) : s;
  for (uint64_t q = b; q < e; q++) {  // forward: seed times the exclusive num prefix
    const Fe vn = an[q];
    an[q] = rn;
    rn = field::mul<F>(rn, vn);
  }
  for (uint64_t q = e; q-- > b;) {  // backward: K'_q
    an[q] = field::mul<F>(an[q], rd);
    rd = field::mul<F>(rd, ad[q]);
  }
}

// D = the product of a product's den block totals (a few to a few thousand values), so D is ready
// right after gp_chunk and the inversion starts before the scan. (Over all chunk totals a
// workgroup's serial strides took 750 us at 2^22 rows.) One workgroup per product.
constexpr int TOT_T = 256;
template <class F>
__global__ __launch_bounds__(TOT_T) void gp_total(uint64_t n, const Fe* __restrict__ zd,
                                                  Fe* __restrict__ dt) {
  const uint32_t c = blockIdx.x, t = threadIdx.x;
  __shared__ Fe sp[TOT_T];
  Fe p = field::one<F>();
  for (uint64_t q = t; q < n; q += TOT_T) p = field::mul<F>(p, zd[(uint64_t)c * n + q]);
  for (uint32_t w = TOT_T / 2; w > 0; w >>= 1) {
    if (t >= w && t < 2 * w) sp[t] = p;
    __syncthreads();
    if (t < w) p = field::mul<F>(p, sp[t + w]);
    __syncthreads();
  }
  if (t == 0) dt[c] = p;
}

// D^-1 in place of D (one lane per product: divsteps, b2f_safegcd.h; it needs only gp_total,
// so it runs on the side stream beside the scans and gp_block_down). D = 0: some den factor is zero (a challenge
// collides with a cell value). halo2's batch_invert would leave that entry zero and the proof
// would fail; here every z would come from a meaningless inverse, so the call reports
// B2F_ERR_FIELD at b2f_sync instead.
template <class F>
__global__ __launch_bounds__(64) void gp_inv(Fe* __restrict__ dt, int* __restrict__ sticky) {
  const uint32_t c = blockIdx.x;
  if (threadIdx.x != 0) return;
  // the inversion is one lane's serial chain beside whole-chip passes on the other stream: top
  // issue priority on its SIMD (r04m: BN254 469 us beside the sigma pass, pasta 190-208 beside
  // the lookup's passes, ~110-125 alone)
  __builtin_amdgcn_s_setprio(3);
  const Fe D = dt[c];
  if (sticky && field::is_zero(D)) atomicOr(sticky, 1 << B2F_ERR_FIELD);
#if defined(B2F_INV_EUCLID)  // diagnostics: the plain binary extended Euclid
  dt[c] = field::inv<F>(D);
#elif defined(B2F_INV_KALISKI)  // diagnostics: Kaliski's almost-inverse (round 4's)
  dt[c] = field::inv_kaliski<F>(D);
#else
  bool ok;
  dt[c] = field::inv_safegcd<F>(D, ok);
  if (sticky && !ok) atomicOr(sticky, 1 << B2F_ERR_CHECK);
#endif
}

// closing[c] = seed N / D (the value z[usable] ends at), for a chained next product
template <class F>
__global__ void gp_close(const Fe* __restrict__ sn, const Fe* __restrict__ dinv, Fe* __restrict__ closing,
                         uint32_t g) {
  const uint32_t c = threadIdx.x;
  if (c < g) closing[c] = field::mul<F>(sn[c], dinv[c]);
}

// z rows go out through LDS in groups of GW_ROWS rows: each lane walks its chunk backward as
// before, stages the z values of GW_ROWS rows, and the wave then stores the group's rows of its
// 64 chunks so that every 8 lanes write one 128-byte run of rows (a lane storing its own rows
// straight away wrote 64 lines 512 bytes apart per store instruction).
constexpr int GW_ROWS = 4;
#ifndef B2F_GW_NT
#define B2F_GW_NT 0  // z stores non-temporal: measured slower (gp_write 263 -> 363 us Pallas, 389 -> 527 BN254)
#endif
constexpr bool GW_NT = B2F_GW_NT != 0;
static_assert(ZC % GW_ROWS == 0, "whole row groups per chunk");
template <class F>
__global__ __launch_bounds__(256) void gp_write(uint64_t usable, bool mont, uint64_t* __restrict__ z_base,
                                                uint64_t z_stride, const Fe* __restrict__ num,
                                                const Fe* __restrict__ den,
                                                const Fe* __restrict__ zn,
                                                const Fe* __restrict__ zd,
                                                const Fe* __restrict__ kb,
                                                const Fe* __restrict__ seed,
                                                const Fe* __restrict__ post,
                                                const Fe* __restrict__ dinv) {
  // a lane's GW_ROWS x 2 chunks padded to 9 (144 bytes): lanes 128 bytes apart hit the same
  // banks in pairs (4-way conflicts on the staging writes, 83 % of the LDS cycles)
  __shared__ uint4 stage[4][64][GW_ROWS * 2 + 1];
  const uint32_t c = blockIdx.y, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint64_t nq = n_chunks(usable);
  const uint64_t q0w = (uint64_t)blockIdx.x * 256 + 64 * wv;  // the wave's first chunk
  const uint64_t q = q0w + lane;
  const bool act = q < nq;
  const Fe* nm = num + (uint64_t)c * elems(usable);  // Nloc, from gp_chunk
  const Fe* dn = den + (uint64_t)c * elems(usable);
  uint64_t* zcol = z_base + (uint64_t)c * z_stride;
  const uint64_t b = q * ZC, e = !act ? b : (b + ZC < usable ? b + ZC : usable);
  // post: a factor applied here rather than in the scan (chained products: the seed of
  // product c is only known once the scans of products 0 .. c - 1 are done)
  const Fe s0 = post ? post[c] : (seed ? seed[c] : field::one<F>());
  if (q == 0) field::store(zcol, out_form<F>(s0, mont));
  Fe k = field::one<F>();
  if (act) {  // K'_q D^-1 = K'_b (exclusive in-block num prefix) (exclusive in-block den suffix) D^-1
    const uint64_t nb = n_blocks(usable);
    k = field::mul<F>(field::mul<F>(kb[(uint64_t)c * nb + q / BLK], zn[(uint64_t)c * nq + q]),
                      field::mul<F>(zd[(uint64_t)c * nq + q], dinv[c]));
    if (post) k = field::mul<F>(k, post[c]);
  }
  // row p's Nloc and den are loaded a row ahead of their use (the staging barriers every
  // GW_ROWS rows would otherwise hold each row's loads until its products)
  Fe an = field::one<F>(), ad = field::one<F>();
  if (b + ZC - 1 < e) {
    an = nm[slot_of(b + ZC - 1, nq)];
    ad = dn[slot_of(b + ZC - 1, nq)];
  }
#pragma unroll 1
  for (int j = ZC - 1; j >= 0; j--) {
    const uint64_t p = b + (uint64_t)j;
    const Fe cn = an, cd = ad;
    if (j > 0 && p - 1 < e) {
      const uint64_t sp = slot_of(p - 1, nq);
      an = nm[sp];
      ad = dn[sp];
    }
    if (p < e) {
      const Fe z = out_form<F>(field::mul<F>(cn, k), mont);
      stage[wv][lane][2 * (j % GW_ROWS)] = make_uint4(z.w[0], z.w[1], z.w[2], z.w[3]);
      stage[wv][lane][2 * (j % GW_ROWS) + 1] = make_uint4(z.w[4], z.w[5], z.w[6], z.w[7]);
      if (j > 0) k = field::mul<F>(k, cd);
    }
    if (j % GW_ROWS == 0) {  // rows b + j + 1 .. b + j + GW_ROWS of the wave's 64 chunks
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int i = 0; i < 64 * GW_ROWS * 2 / 64; i++) {
        const uint32_t u = 64u * i + lane, ch = u / (2 * GW_ROWS), rr = (u >> 1) % GW_ROWS, h = u & 1u;
        const uint64_t cq = q0w + ch, pr = cq * ZC + (uint64_t)j + rr;  // the row p whose z[p + 1] this is
        if (cq < nq && pr < usable && pr < cq * ZC + ZC) {
          const uint4 v = stage[wv][ch][2 * rr + h];
          put16<GW_NT>(reinterpret_cast<uint4*>(zcol + 4 * (pr + 1) + 2 * h), v);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
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
  const uint64_t nq = n_chunks(usable), nb = n_blocks(usable);
  return 2 * nq + 2 * nb + 2;  // in-block chunk prefixes / suffixes, block totals, (seed N, D / D^-1)
}

struct Side {
  hipStream_t s2;
  hipEvent_t fork, join;
};
struct Scratch {  // the carve of zs for g products
  Fe *zn, *zd, *tn, *td, *sn, *dt;
};
__host__ __device__ inline Scratch scratch_of(Fe* zs, uint32_t g, uint64_t usable) {
  const uint64_t nq = n_chunks(usable), nb = n_blocks(usable);
  Scratch k;
  k.zn = zs;
  k.zd = zs + (uint64_t)g * nq;
  k.tn = k.zd + (uint64_t)g * nq;
  k.td = k.tn + (uint64_t)g * nb;
  k.sn = k.td + (uint64_t)g * nb;  // g: seed N per product (gp_scan)
  k.dt = k.sn + g;                  // g: D, then D^-1 (gp_total, gp_inv)
  return k;
}
// First half of the passes: chunk products and block scans, the den total D, and D^-1 -- on the
// side stream when `side` has one (forked after gp_total, joined by run_end), so whatever the
// caller launches on `s` between run_begin and run_end overlaps the inversion's ~100 us of
// latency (the lookup's other half of its circuits, the permutation's sigma columns).
// chunked: the caller's factor pass already wrote what gp_chunk writes (Nloc over num, zn / zd,
// tn / td: the permutation's pm_chunk_kernel). have_dinv: the caller computes D^-1 into
// scratch_of(zs).dt itself, on side.s2, recording side.join when done (the lookup: D from the
// histogram, before its factor pass) -- only gp_chunk runs here.
template <class F>
hipError_t run_begin(uint32_t g, uint64_t usable, Fe* num, const Fe* den, Fe* zs, int* sticky,
                     Side side, hipStream_t s, bool chunked = false, bool have_dinv = false) {
  const uint64_t nb = n_blocks(usable);
  const Scratch k = scratch_of(zs, g, usable);
  hipError_t e;
  if (!chunked)
    hipLaunchKernelGGL(gp_chunk<F>, dim3((uint32_t)nb, g), dim3(BLK), 0, s, usable, num, den, k.zn, k.zd,
                       k.tn, k.td);
  if (have_dinv) return hipGetLastError();
  hipLaunchKernelGGL(gp_total<F>, dim3(g), dim3(TOT_T), 0, s, nb, k.td, k.dt);
  if (side.s2) {
    if ((e = hipEventRecord(side.fork, s)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(side.s2, side.fork, 0)) != hipSuccess) return e;
  }
  hipLaunchKernelGGL(gp_inv<F>, dim3(g), dim3(64), 0, side.s2 ? side.s2 : s, k.dt, sticky);
  if (side.s2 && (e = hipEventRecord(side.join, side.s2)) != hipSuccess) return e;
  return hipGetLastError();
}
// Second half: the block scan, the join with the inversion, closing values / chained seeds, and
// z. With `chain` (2 g elements of scratch) the products are chained -- product c starts from
// product c - 1's closing value, product 0 from 1 -- and still scanned side by side: their single
// inversions run in parallel, the seeds are applied in gp_write.
template <class F>
hipError_t run_end(uint32_t g, uint64_t usable, bool mont, uint64_t* z_base, uint64_t z_stride,
                   Fe* num, const Fe* den, Fe* zs, const Fe* seed, Fe* closing, hipStream_t s,
                   Fe* chain, Side side) {
  Fe* post = nullptr;
  if (chain) {
    seed = nullptr;
    closing = chain;  // T
    post = chain + g;  // S
  }
  const uint64_t nq = n_chunks(usable), nb = n_blocks(usable);
  const Scratch k = scratch_of(zs, g, usable);
  hipError_t e;
  if (nb <= 64)
    hipLaunchKernelGGL((gp_scan<F, 64>), dim3(g), dim3(64), 0, s, nb, k.tn, k.td, seed, k.sn);
  else
    hipLaunchKernelGGL(gp_scan<F>, dim3(g), dim3(SCAN_THREADS), 0, s, nb, k.tn, k.td, seed, k.sn);
  if (side.s2 && (e = hipStreamWaitEvent(s, side.join, 0)) != hipSuccess) return e;
  if (closing) hipLaunchKernelGGL(gp_close<F>, dim3(1), dim3(256), 0, s, k.sn, k.dt, closing, g);
  if (chain) hipLaunchKernelGGL(gp_chain_seeds<F>, dim3(1), dim3(64), 0, s, chain, post, g);
  hipLaunchKernelGGL(gp_write<F>, dim3((uint32_t)((nq + 255) / 256), g), dim3(256), 0, s, usable, mont,
                     z_base, z_stride, num, den, k.zn, k.zd, k.tn, seed, post, k.dt);
  return hipGetLastError();
}
// The passes for `g` products on `s` (zs: g * scratch_elems(usable) elements).
template <class F>
hipError_t run(uint32_t g, uint64_t usable, bool mont, uint64_t* z_base, uint64_t z_stride,
               Fe* num, const Fe* den, Fe* zs, const Fe* seed, Fe* closing, hipStream_t s,
               Fe* chain = nullptr, int* sticky = nullptr, Side side = Side{nullptr, nullptr, nullptr}) {
  hipError_t e = run_begin<F>(g, usable, num, den, zs, sticky, side, s);
  if (e != hipSuccess) return e;
  return run_end<F>(g, usable, mont, z_base, z_stride, num, den, zs, seed, closing, s, chain, side);
}

}  // namespace
}  // namespace gp
}  // namespace b2f

// b2f_lookup.hip -- lookup-argument prover columns of the spread lookup (SURVEY.md §8(f)
// row 4): for circuits cut from the trace (usable rows each), halo2_proofs 0.3.0's
// compressed input A, compressed table S, permuted input A', permuted table S' and the
// grand product z (lookup/prover.rs: commit_permuted, permute_expression_pair,
// commit_product; restated in oracle/lookup.py).
//
// halo2 sorts the compressed inputs and walks a BTreeMap of table values. Here every input
// is a table row, so the sort is a counting sort over the 2^16 table rows in the order of
// their compressed values:
//   table pass (once per theta): T[x] = theta^2 tag(x) + theta x + spread(x) for x < 2^16,
//     sorted by canonical value (four stable LSD passes of a 64-bit radix sort), giving the
//     rank order x_of_rank[r] and Ts[r] = T[x_of_rank[r]];
//   count:   histogram of the dense cell (a_1) over the circuit's rows, with the row check
//            (tag, dense, spread) in table (first failing row reported);
//   scan:    in rank order, run starts pos[r] (exclusive prefix of counts), D[r] (runs up to
//            and including r) and LP[r] (exclusive prefix of leftover table multiplicities);
//   permute: row p of A' is Ts[r] for the run r holding p (binary search of pos); a run
//            start gets S'[p] = Ts[r]; the j-th repeated row gets leftover item L - 1 - j
//            (halo2 hands leftovers out in ascending order, each to the last open repeated
//            row), found by binary search of LP;
//   z:       the permute pass also writes each row's factors num = (A + beta)(S + gamma) and
//            den = (A' + beta)(S' + gamma); per 64-row chunk the products of num and of den;
//            exclusive product scans over the chunks; then each chunk's z rows N_p / D_p
//            with one inversion per chunk (batch inversion, N_p staged in the z column).
// Field arithmetic: pasta Fp, 4 x 64-bit limbs, Montgomery (R = 2^256) CIOS multiply.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "../../include/b2f.h"

namespace b2f {

size_t lookup_scratch_bytes(uint32_t group, uint64_t usable_rows);
hipError_t launch_lookup(const uint32_t* d_advice, uint64_t total_rows,
                         const uint64_t* d_row_begin, uint32_t n_circuits, uint64_t usable_rows,
                         const uint64_t* theta, const uint64_t* beta, const uint64_t* gamma,
                         uint32_t form, uint64_t* d_out, uint64_t out_rows, uint64_t* d_first_bad,
                         void* scratch, uint32_t group, hipStream_t s);

namespace {

typedef unsigned __int128 u128;
constexpr int TROWS = 1 << 16;
constexpr uint64_t FP_P0 = 0x992d30ed00000001ull, FP_P1 = 0x224698fc094cf91bull,
                   FP_P3 = 0x4000000000000000ull;
constexpr uint64_t FP_INV = 0x992d30ecffffffffull;  // -p^-1 mod 2^64

struct Fp {
  uint64_t v[4];
};
struct Chal {
  uint64_t theta[4], beta[4], gamma[4];
};

__device__ __forceinline__ Fp fp_make(uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
  Fp r;
  r.v[0] = a; r.v[1] = b; r.v[2] = c; r.v[3] = d;
  return r;
}
__device__ __forceinline__ Fp fp_one() {  // R mod p
  return fp_make(0x34786d38fffffffdull, 0x992c350be41914adull, 0xffffffffffffffffull,
                 0x3fffffffffffffffull);
}
__device__ __forceinline__ Fp fp_r2() {  // R^2 mod p
  return fp_make(0x8c78ecb30000000full, 0xd7d30dbd8b0de0e7ull, 0x7797a99bc3c95d18ull,
                 0x096d41af7b9cb714ull);
}

// t (< 2p) -> t mod p
__device__ __forceinline__ Fp fp_reduce1(uint64_t t0, uint64_t t1, uint64_t t2, uint64_t t3) {
  u128 d = (u128)t0 - FP_P0;
  uint64_t r0 = (uint64_t)d, b = (uint64_t)(d >> 64) & 1;
  d = (u128)t1 - FP_P1 - b;
  uint64_t r1 = (uint64_t)d;
  b = (uint64_t)(d >> 64) & 1;
  d = (u128)t2 - b;
  uint64_t r2 = (uint64_t)d;
  b = (uint64_t)(d >> 64) & 1;
  d = (u128)t3 - FP_P3 - b;
  uint64_t r3 = (uint64_t)d;
  b = (uint64_t)(d >> 64) & 1;
  return b ? fp_make(t0, t1, t2, t3) : fp_make(r0, r1, r2, r3);
}

// Montgomery product a * b / 2^256 mod p (CIOS; p2 = 0 and p3 = 2^62 fold into the constants)
__device__ __forceinline__ Fp fp_mul(const Fp& a, const Fp& b) {
  uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t bi = b.v[i];
    u128 c = (u128)a.v[0] * bi + t0;
    t0 = (uint64_t)c;
    c = (u128)a.v[1] * bi + t1 + (uint64_t)(c >> 64);
    t1 = (uint64_t)c;
    c = (u128)a.v[2] * bi + t2 + (uint64_t)(c >> 64);
    t2 = (uint64_t)c;
    c = (u128)a.v[3] * bi + t3 + (uint64_t)(c >> 64);
    t3 = (uint64_t)c;
    u128 c4 = (u128)t4 + (uint64_t)(c >> 64);
    t4 = (uint64_t)c4;
    const uint64_t t5 = (uint64_t)(c4 >> 64);
    const uint64_t m = t0 * FP_INV;
    c = (u128)m * FP_P0 + t0;
    c = (u128)m * FP_P1 + t1 + (uint64_t)(c >> 64);
    t0 = (uint64_t)c;
    c = (u128)t2 + (uint64_t)(c >> 64);
    t1 = (uint64_t)c;
    c = (u128)m * FP_P3 + t3 + (uint64_t)(c >> 64);
    t2 = (uint64_t)c;
    c = (u128)t4 + (uint64_t)(c >> 64);
    t3 = (uint64_t)c;
    t4 = t5 + (uint64_t)(c >> 64);
  }
  return fp_reduce1(t0, t1, t2, t3);
}

__device__ __forceinline__ Fp fp_add(const Fp& a, const Fp& b) {  // a, b < p < 2^255
  u128 c = (u128)a.v[0] + b.v[0];
  uint64_t s0 = (uint64_t)c;
  c = (u128)a.v[1] + b.v[1] + (uint64_t)(c >> 64);
  uint64_t s1 = (uint64_t)c;
  c = (u128)a.v[2] + b.v[2] + (uint64_t)(c >> 64);
  uint64_t s2 = (uint64_t)c;
  uint64_t s3 = a.v[3] + b.v[3] + (uint64_t)(c >> 64);
  return fp_reduce1(s0, s1, s2, s3);
}

__device__ __forceinline__ Fp fp_small(uint32_t x) {  // Montgomery form of a small integer
  return fp_mul(fp_make(x, 0, 0, 0), fp_r2());
}

// a^(p-2): left-to-right square and multiply over the fixed exponent
__device__ Fp fp_inv(const Fp& a) {
  const uint64_t e[4] = {FP_P0 - 2, FP_P1, 0, FP_P3};
  Fp r = a;  // bit 254 (the top bit of e)
#pragma unroll 1
  for (int bit = 253; bit >= 0; bit--) {
    r = fp_mul(r, r);
    if ((e[bit >> 6] >> (bit & 63)) & 1) r = fp_mul(r, a);
  }
  return r;
}

__device__ __forceinline__ Fp fp_out(const Fp& a, uint32_t form) {
  return form == B2F_FP_CANONICAL ? fp_mul(a, fp_make(1, 0, 0, 0)) : a;
}

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void fp_store(uint64_t* p, const Fp& a) {
  u64x2* q = reinterpret_cast<u64x2*>(p);
  q[0] = u64x2{a.v[0], a.v[1]};
  q[1] = u64x2{a.v[2], a.v[3]};
}
__device__ __forceinline__ Fp fp_load(const uint64_t* p) {
  const u64x2* q = reinterpret_cast<const u64x2*>(p);
  u64x2 x = q[0], y = q[1];
  return fp_make(x.x, x.y, y.x, y.y);
}

__device__ __forceinline__ uint32_t spread16(uint32_t x) {
  x = (x | (x << 8)) & 0x00FF00FFu;
  x = (x | (x << 4)) & 0x0F0F0F0Fu;
  x = (x | (x << 2)) & 0x33333333u;
  x = (x | (x << 1)) & 0x55555555u;
  return x;
}
__device__ __forceinline__ uint32_t tag16(uint32_t x) { return x < 256u ? 0u : (x < 32768u ? 1u : 2u); }

__device__ __forceinline__ Fp chal(const uint64_t* c) { return fp_make(c[0], c[1], c[2], c[3]); }

// ------------------------------------------------------------------ table pass (per theta)
__global__ __launch_bounds__(256) void lk_table_kernel(Chal ch, Fp* __restrict__ Tx,
                                                       uint64_t* __restrict__ key,
                                                       uint32_t* __restrict__ perm) {
  const uint32_t x = blockIdx.x * 256 + threadIdx.x;
  const Fp th = fp_mul(chal(ch.theta), fp_r2());
  const Fp th2 = fp_mul(th, th);
  Fp t = fp_add(fp_add(fp_mul(th2, fp_small(tag16(x))), fp_mul(th, fp_small(x))),
                fp_small(spread16(x)));
  Tx[x] = t;
  const Fp c = fp_mul(t, fp_make(1, 0, 0, 0));
#pragma unroll
  for (int k = 0; k < 4; k++) key[(uint64_t)k * TROWS + x] = c.v[k];
  perm[x] = x;
}

__global__ __launch_bounds__(256) void lk_gather_key_kernel(const uint64_t* __restrict__ limb,
                                                            const uint32_t* __restrict__ perm,
                                                            uint64_t* __restrict__ out) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  out[i] = limb[perm[i]];
}

__global__ __launch_bounds__(256) void lk_rank_kernel(const Fp* __restrict__ Tx,
                                                      const uint32_t* __restrict__ perm,
                                                      Fp* __restrict__ Ts) {
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

__global__ __launch_bounds__(256) void lk_count_kernel(
    const uint32_t* __restrict__ adv, uint64_t total_rows, const uint64_t* __restrict__ row_begin,
    uint32_t c0, uint64_t usable, uint32_t* __restrict__ count, uint64_t* __restrict__ first_bad) {
  const uint32_t c = blockIdx.y;
  const Circ k = circ(row_begin, total_rows, usable, c0 + c);
  uint32_t* cnt = count + (uint64_t)c * TROWS;
  if (blockIdx.x == 0 && threadIdx.x == 0 && usable > k.n_in)
    atomicAdd(cnt, (uint32_t)(usable - k.n_in));  // zero rows past the trace: table row 0
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t base = (uint64_t)blockIdx.x * 256; base < k.n_in; base += stride) {
    const uint64_t p = base + threadIdx.x;
    const bool act = p < k.n_in;
    uint32_t a0 = 0, a1 = 0, a2 = 0;
    if (act) {
      const uint64_t row = k.first + p;
      a0 = adv[row];
      a1 = adv[total_rows + row];
      a2 = adv[2 * total_rows + row];
    }
    const bool ok = a1 < (uint32_t)TROWS && a0 == tag16(a1) && a2 == spread16(a1);
    if (act && !ok) atomicMin((unsigned long long*)first_bad + c0 + c, (unsigned long long)p);
    const bool zero = act && ok && a1 == 0;
    const uint64_t zb = __ballot(zero);
    if (zb && (threadIdx.x & 63) == (uint32_t)__builtin_ctzll(zb))
      atomicAdd(cnt, (uint32_t)__builtin_popcountll(zb));
    if (act && ok && a1 != 0) atomicAdd(cnt + a1, 1u);
  }
}

// one workgroup per circuit: 1024 threads x 64 ranks
__global__ __launch_bounds__(1024) void lk_scan_kernel(const uint32_t* __restrict__ perm,
                                                       const uint32_t* __restrict__ count,
                                                       uint64_t usable, uint32_t* __restrict__ pos,
                                                       uint32_t* __restrict__ dcnt,
                                                       uint32_t* __restrict__ lp) {
  const uint32_t c = blockIdx.x, t = threadIdx.x;
  const uint32_t* cnt = count + (uint64_t)c * TROWS;
  uint32_t sc = 0, sd = 0, sl = 0;
  for (int i = 0; i < 64; i++) {
    const uint32_t x = perm[t * 64 + i];
    const uint32_t n = cnt[x];
    const uint32_t mult = x == 0 ? (uint32_t)(usable - TROWS + 1) : 1u;
    sc += n;
    sd += n ? 1u : 0u;
    sl += mult - (n ? 1u : 0u);
  }
  __shared__ uint32_t s[3][1024];
  s[0][t] = sc; s[1][t] = sd; s[2][t] = sl;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // inclusive Hillis-Steele
    uint32_t a = 0, b = 0, d = 0;
    if (t >= (uint32_t)off) { a = s[0][t - off]; b = s[1][t - off]; d = s[2][t - off]; }
    __syncthreads();
    s[0][t] += a; s[1][t] += b; s[2][t] += d;
    __syncthreads();
  }
  uint32_t ec = s[0][t] - sc, ed = s[1][t] - sd, el = s[2][t] - sl;  // exclusive
  uint32_t* P = pos + (uint64_t)c * TROWS;
  uint32_t* D = dcnt + (uint64_t)c * TROWS;
  uint32_t* L = lp + (uint64_t)c * TROWS;
  for (int i = 0; i < 64; i++) {
    const uint32_t r = t * 64 + i;
    const uint32_t x = perm[r];
    const uint32_t n = cnt[x];
    const uint32_t mult = x == 0 ? (uint32_t)(usable - TROWS + 1) : 1u;
    P[r] = ec;
    ed += n ? 1u : 0u;
    D[r] = ed;
    L[r] = el;
    ec += n;
    el += mult - (n ? 1u : 0u);
  }
}

// last index r with a[r] <= v (a nondecreasing, a[0] <= v)
__device__ __forceinline__ uint32_t last_le(const uint32_t* a, uint32_t v) {
  uint32_t lo = 0, hi = TROWS;  // answer in [lo, hi)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid; else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void lk_permute_kernel(
    const uint32_t* __restrict__ adv, uint64_t total_rows, const uint64_t* __restrict__ row_begin,
    uint32_t c0, uint64_t usable, const Fp* __restrict__ Tx, const Fp* __restrict__ Ts,
    const uint32_t* __restrict__ pos, const uint32_t* __restrict__ dcnt,
    const uint32_t* __restrict__ lp, uint32_t form, uint64_t* __restrict__ out, uint64_t out_rows,
    Chal ch, Fp* __restrict__ num, Fp* __restrict__ den) {
  const uint32_t c = blockIdx.y;
  const Fp beta = fp_mul(chal(ch.beta), fp_r2()), gamma = fp_mul(chal(ch.gamma), fp_r2());
  Fp* nm = num + (uint64_t)c * usable;
  Fp* dn = den + (uint64_t)c * usable;
  const Circ k = circ(row_begin, total_rows, usable, c0 + c);
  const uint32_t* P = pos + (uint64_t)c * TROWS;
  const uint32_t* D = dcnt + (uint64_t)c * TROWS;
  const uint32_t* L = lp + (uint64_t)c * TROWS;
  const uint32_t n_left = (uint32_t)usable - D[TROWS - 1];
  uint64_t* o = out + (uint64_t)(c0 + c) * 5 * out_rows * 4;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < usable; p += stride) {
    const uint32_t x = p < k.n_in ? (adv[total_rows + k.first + p] & 0xffffu) : 0u;
    const Fp a = Tx[x];
    const Fp sv = Tx[p < (uint64_t)TROWS ? (uint32_t)p : 0u];
    const uint32_t r = last_le(P, (uint32_t)p);
    const Fp ap = Ts[r];
    Fp sp;
    if (P[r] == (uint32_t)p) {
      sp = ap;
    } else {
      const uint32_t j = (uint32_t)p - D[r];
      sp = Ts[last_le(L, n_left - 1 - j)];
    }
    fp_store(o + 4 * p, fp_out(a, form));
    fp_store(o + (out_rows + p) * 4, fp_out(sv, form));
    fp_store(o + (2 * out_rows + p) * 4, fp_out(ap, form));
    fp_store(o + (3 * out_rows + p) * 4, fp_out(sp, form));
    // the grand product's factors (A + beta)(S + gamma) / ((A' + beta)(S' + gamma))
    fp_store(nm[p].v, fp_mul(fp_add(a, beta), fp_add(sv, gamma)));
    fp_store(dn[p].v, fp_mul(fp_add(ap, beta), fp_add(sp, gamma)));
  }
}

constexpr uint32_t ZC = 64;  // rows per z chunk (one inversion per chunk)

// per chunk: products of num and den
__global__ __launch_bounds__(256) void lk_zchunk_kernel(uint64_t usable, const Fp* __restrict__ num,
                                                        const Fp* __restrict__ den,
                                                        Fp* __restrict__ zn, Fp* __restrict__ zd) {
  const uint32_t c = blockIdx.y;
  const uint64_t nq = (usable + ZC - 1) / ZC;
  const uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  const Fp* nm = num + (uint64_t)c * usable;
  const Fp* dn = den + (uint64_t)c * usable;
  Fp pn = fp_one(), pd = fp_one();
  const uint64_t e = (q + 1) * ZC < usable ? (q + 1) * ZC : usable;
  for (uint64_t p = q * ZC; p < e; p++) {
    pn = fp_mul(pn, fp_load(nm[p].v));
    pd = fp_mul(pd, fp_load(dn[p].v));
  }
  zn[(uint64_t)c * nq + q] = pn;
  zd[(uint64_t)c * nq + q] = pd;
}

// exclusive product scans of zn and zd over a circuit's chunks (one workgroup per circuit):
// per-thread runs of chunks, then a Hillis-Steele scan of the 1024 run products in LDS (both
// arrays at once: two independent multiply chains)
constexpr int ZS_THREADS = 1024;
__global__ __launch_bounds__(ZS_THREADS) void lk_zscan_kernel(uint64_t usable, Fp* __restrict__ zn,
                                                              Fp* __restrict__ zd) {
  const uint32_t c = blockIdx.x, t = threadIdx.x;
  const uint64_t nq = (usable + ZC - 1) / ZC;
  const uint64_t per = (nq + ZS_THREADS - 1) / ZS_THREADS;
  __shared__ Fp sn[ZS_THREADS], sd[ZS_THREADS];
  Fp* an = zn + (uint64_t)c * nq;
  Fp* ad = zd + (uint64_t)c * nq;
  const uint64_t b = t * per < nq ? t * per : nq, e = b + per < nq ? b + per : nq;
  Fp pn = fp_one(), pd = fp_one();
  for (uint64_t q = b; q < e; q++) {
    pn = fp_mul(pn, an[q]);
    pd = fp_mul(pd, ad[q]);
  }
  sn[t] = pn;
  sd[t] = pd;
  __syncthreads();
  for (int off = 1; off < ZS_THREADS; off <<= 1) {  // inclusive
    Fp xn = pn, xd = pd;
    if (t >= (uint32_t)off) {
      xn = fp_mul(sn[t - off], pn);
      xd = fp_mul(sd[t - off], pd);
    }
    __syncthreads();
    sn[t] = pn = xn;
    sd[t] = pd = xd;
    __syncthreads();
  }
  Fp rn = t ? sn[t - 1] : fp_one(), rd = t ? sd[t - 1] : fp_one();
  for (uint64_t q = b; q < e; q++) {
    const Fp vn = an[q], vd = ad[q];
    an[q] = rn;
    ad[q] = rd;
    rn = fp_mul(rn, vn);
    rd = fp_mul(rd, vd);
  }
}

// z rows of chunk q: with N_p, D_p the prefix products of num and den through row p,
// z[p + 1] = N_p / D_p. Forward: N_p staged in z[p + 1], D running; one inversion of the
// chunk's last D; backward: z[p + 1] = N_p (1 / D_p), 1 / D_{p-1} = (1 / D_p) den_p.
__global__ __launch_bounds__(256) void lk_zwrite_kernel(uint32_t c0, uint64_t usable, uint32_t form,
                                                        uint64_t* __restrict__ out, uint64_t out_rows,
                                                        const Fp* __restrict__ num,
                                                        const Fp* __restrict__ den,
                                                        const Fp* __restrict__ zn,
                                                        const Fp* __restrict__ zd) {
  const uint32_t c = blockIdx.y;
  const uint64_t nq = (usable + ZC - 1) / ZC;
  const uint64_t q = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= nq) return;
  const Fp* nm = num + (uint64_t)c * usable;
  const Fp* dn = den + (uint64_t)c * usable;
  uint64_t* zcol = out + ((uint64_t)(c0 + c) * 5 + 4) * out_rows * 4;
  const uint64_t b = q * ZC, e = (q + 1) * ZC < usable ? (q + 1) * ZC : usable;
  Fp n = zn[(uint64_t)c * nq + q], d = zd[(uint64_t)c * nq + q];
  if (q == 0) fp_store(zcol, fp_out(fp_one(), form));
  for (uint64_t p = b; p < e; p++) {
    n = fp_mul(n, fp_load(nm[p].v));
    d = fp_mul(d, fp_load(dn[p].v));
    fp_store(zcol + 4 * (p + 1), n);
  }
  Fp inv = fp_inv(d);
  for (uint64_t p = e; p-- > b;) {
    fp_store(zcol + 4 * (p + 1), fp_out(fp_mul(fp_load(zcol + 4 * (p + 1)), inv), form));
    inv = fp_mul(inv, fp_load(dn[p].v));
  }
}

struct Carve {
  Fp* Tx;
  Fp* Ts;
  uint64_t* key;   // 4 x TROWS canonical limbs
  uint64_t* kin;   // TROWS
  uint64_t* kout;  // TROWS
  uint32_t* perm;  // TROWS
  uint32_t* perm2;
  uint32_t* count;  // group x TROWS
  uint32_t* pos;
  uint32_t* dcnt;
  uint32_t* lp;
  Fp* num;  // group x usable
  Fp* den;
  Fp* zn;  // group x nq
  Fp* zd;
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
  const uint64_t nq = (usable + ZC - 1) / ZC;
  k.Tx = (Fp*)take(sizeof(Fp) * TROWS);
  k.Ts = (Fp*)take(sizeof(Fp) * TROWS);
  k.key = (uint64_t*)take(8ull * 4 * TROWS);
  k.kin = (uint64_t*)take(8ull * TROWS);
  k.kout = (uint64_t*)take(8ull * TROWS);
  k.perm = (uint32_t*)take(4ull * TROWS);
  k.perm2 = (uint32_t*)take(4ull * TROWS);
  k.count = (uint32_t*)take(4ull * TROWS * group);
  k.pos = (uint32_t*)take(4ull * TROWS * group);
  k.dcnt = (uint32_t*)take(4ull * TROWS * group);
  k.lp = (uint32_t*)take(4ull * TROWS * group);
  k.num = (Fp*)take(sizeof(Fp) * usable * group);
  k.den = (Fp*)take(sizeof(Fp) * usable * group);
  k.zn = (Fp*)take(sizeof(Fp) * nq * group);
  k.zd = (Fp*)take(sizeof(Fp) * nq * group);
  k.sort_bytes = sort_temp_bytes();
  k.sort_tmp = take(k.sort_bytes);
  k.total = off;
  return k;
}

}  // namespace

size_t lookup_scratch_bytes(uint32_t group, uint64_t usable_rows) {
  return carve(nullptr, group, usable_rows).total;
}

hipError_t launch_lookup(const uint32_t* d_advice, uint64_t total_rows,
                         const uint64_t* d_row_begin, uint32_t n_circuits, uint64_t usable_rows,
                         const uint64_t* theta, const uint64_t* beta, const uint64_t* gamma,
                         uint32_t form, uint64_t* d_out, uint64_t out_rows, uint64_t* d_first_bad,
                         void* scratch, uint32_t group, hipStream_t s) {
  Carve k = carve(scratch, group, usable_rows);
  Chal ch;
  for (int i = 0; i < 4; i++) {
    ch.theta[i] = theta[i];
    ch.beta[i] = beta[i];
    ch.gamma[i] = gamma[i];
  }
  const dim3 tb(TROWS / 256);
  hipLaunchKernelGGL(lk_table_kernel, tb, dim3(256), 0, s, ch, k.Tx, k.key, k.perm);
  // stable LSD over the four 64-bit limbs of the canonical value
  uint32_t* pa = k.perm;
  uint32_t* pb = k.perm2;
  for (int limb = 0; limb < 4; limb++) {
    hipLaunchKernelGGL(lk_gather_key_kernel, tb, dim3(256), 0, s, k.key + (uint64_t)limb * TROWS,
                       pa, k.kin);
    size_t bytes = k.sort_bytes;
    hipError_t e = rocprim::radix_sort_pairs(k.sort_tmp, bytes, k.kin, k.kout, pa, pb,
                                             (size_t)TROWS, 0, limb == 3 ? 63 : 64, s);
    if (e != hipSuccess) return e;
    uint32_t* t = pa;
    pa = pb;
    pb = t;
  }
  hipLaunchKernelGGL(lk_rank_kernel, tb, dim3(256), 0, s, k.Tx, pa, k.Ts);
  hipError_t e = hipMemsetAsync(d_first_bad, 0xff, 8ull * n_circuits, s);
  if (e != hipSuccess) return e;
  const uint64_t nq = (usable_rows + ZC - 1) / ZC;
  for (uint32_t c0 = 0; c0 < n_circuits; c0 += group) {
    const uint32_t g = n_circuits - c0 < group ? n_circuits - c0 : group;
    e = hipMemsetAsync(k.count, 0, 4ull * TROWS * g, s);
    if (e != hipSuccess) return e;
    const uint32_t bx = (uint32_t)((usable_rows + 255) / 256 < 512 ? (usable_rows + 255) / 256 : 512);
    hipLaunchKernelGGL(lk_count_kernel, dim3(bx, g), dim3(256), 0, s, d_advice, total_rows,
                       d_row_begin, c0, usable_rows, k.count, d_first_bad);
    hipLaunchKernelGGL(lk_scan_kernel, dim3(g), dim3(1024), 0, s, pa, k.count, usable_rows, k.pos,
                       k.dcnt, k.lp);
    hipLaunchKernelGGL(lk_permute_kernel, dim3(bx, g), dim3(256), 0, s, d_advice, total_rows,
                       d_row_begin, c0, usable_rows, k.Tx, k.Ts, k.pos, k.dcnt, k.lp, form, d_out,
                       out_rows, ch, k.num, k.den);
    const uint32_t zq = (uint32_t)((nq + 255) / 256);
    hipLaunchKernelGGL(lk_zchunk_kernel, dim3(zq, g), dim3(256), 0, s, usable_rows, k.num, k.den,
                       k.zn, k.zd);
    hipLaunchKernelGGL(lk_zscan_kernel, dim3(g), dim3(ZS_THREADS), 0, s, usable_rows, k.zn, k.zd);
    hipLaunchKernelGGL(lk_zwrite_kernel, dim3(zq, g), dim3(256), 0, s, c0, usable_rows, form, d_out,
                       out_rows, k.num, k.den, k.zn, k.zd);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace b2f

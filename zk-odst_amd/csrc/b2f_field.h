// b2f_field.h -- the prime fields of the prover columns, on the device.
//
//   Pallas: pallas::Base = pasta_curves 0.5.1 Fp (Cargo.lock:1334-1337), the field of
//           halo2_proofs 0.3.0's own tests;
//   Bn254:  halo2curves 0.3.2 bn256::Fr (Cargo.lock:859-861), the field the reference
//           instantiates its circuit in (blake2f.rs:283,293; blake2f_circuit_bench.rs:10,34).
// Both keep elements in Montgomery form with R = 2^256, four little-endian u64 limbs -- here
// eight u32 words in the same byte order, so an element is stored exactly as the crates hold
// it in memory.
//
// Multiply: Montgomery product by product scanning (Comba) over 8 x 32-bit words: each column
// of the 512-bit sum of a_i b_j and m_i p_j accumulates in a 64-bit VGPR pair by
// v_mad_u64_u32 whose carry goes into a third word by v_addc. `mul` is that product as one
// generated inline-asm block per field (b2f_mont_asm.h, tools/gen_mont_asm.py: the accumulator
// in two fixed VGPR pairs, pallas' p_0 = 1 and p_7 = 2^30 words without multiplies); mul_comba
// is the same scheme as per-step asm (round 4) and mul_cios the operand-scanning form before it,
// both kept as tools/mulbench.hip's cross-checks. Both moduli have a top word below 2^31 - 1, so
// the result is < 2p and one conditional subtraction finishes it (the oracle and halo2 use the
// textbook form; the result is the same canonical residue).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "b2f_safegcd.h"

namespace b2f {
namespace field {

struct Pallas {
  static constexpr uint32_t P[8] = {0x00000001u, 0x992d30edu, 0x094cf91bu, 0x224698fcu,
                                    0x00000000u, 0x00000000u, 0x00000000u, 0x40000000u};
  static constexpr uint32_t R[8] = {0xfffffffdu, 0x34786d38u, 0xe41914adu, 0x992c350bu,
                                    0xffffffffu, 0xffffffffu, 0xffffffffu, 0x3fffffffu};
  static constexpr uint32_t R2[8] = {0x0000000fu, 0x8c78ecb3u, 0x8b0de0e7u, 0xd7d30dbdu,
                                     0xc3c95d18u, 0x7797a99bu, 0x7b9cb714u, 0x096d41afu};
  static constexpr uint32_t R3[8] = {0x3a9e10f9u, 0xf185a599u, 0x6ac5b1d1u, 0xf6a68f3bu,
                                     0x353fd42cu, 0xdf8d1014u, 0x2d2d9910u, 0x2ae30922u};
  static constexpr uint32_t NP = 0xffffffffu;  // -p^-1 mod 2^32
  static constexpr uint64_t RQ = 0xffffffffffffffffull;  // floor(R 2^64 / p), R = 2^256 mod p
};

struct Bn254 {
  static constexpr uint32_t P[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t R[8] = {0x4ffffffbu, 0xac96341cu, 0x9f60cd29u, 0x36fc7695u,
                                    0x7879462eu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr uint32_t R2[8] = {0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u,
                                     0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u};
  static constexpr uint32_t R3[8] = {0xb4bf0040u, 0x5e94d8e1u, 0x1cfbb6b8u, 0x2a489cbeu,
                                     0xa19fcfedu, 0x893cc664u, 0x7fcc657cu, 0x0cf8594bu};
  static constexpr uint32_t NP = 0xefffffffu;
  static constexpr uint64_t RQ = 0x4a47462623a04a7aull;
};

static_assert(Pallas::P[7] < 0x7ffffffeu && Bn254::P[7] < 0x7ffffffeu, "no-carry CIOS needs a spare top bit");

struct Fe {
  uint32_t w[8];
};

__device__ __forceinline__ Fe fe_zero() {
  Fe r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.w[i] = 0;
  return r;
}

template <class F>
__device__ __forceinline__ Fe fe_const(const uint32_t (&c)[8]) {
  Fe r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.w[i] = c[i];
  return r;
}

template <class F>
__device__ __forceinline__ Fe one() {  // Montgomery form of 1
  return fe_const<F>(F::R);
}

// t (< 2p, 8 words) -> t mod p
template <class F>
__device__ __forceinline__ Fe reduce_once(const Fe& t) {
  Fe d;
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t x = (uint64_t)t.w[i] - F::P[i] - borrow;
    d.w[i] = (uint32_t)x;
    borrow = (uint32_t)(x >> 63);
  }
  return borrow ? t : d;
}

#include "b2f_mont_asm.h"

// Montgomery product a b / 2^256 mod p (a, b < p), product scanning (Comba): column k of the
// 512-bit sum of a_i b_j and m_i p_j (i + j = k; m_k chosen so column k < 8 ends in a zero word)
// accumulates in a 64-bit VGPR pair by v_mad_u64_u32, whose carry out of the 64-bit add goes
// straight into a third word by v_addc (acc_madd): two instructions per word product. The
// constant words of p are SGPR operands and fold (pallas has three zero words). The compiler's
// form of the operand-scanning CIOS (add-with-carry fed addends, kept below as mul_cios) took
// about three instructions and a wait state per word product: tools/mulbench.hip, gfx950,
// profiles/r04h_mulbench.txt: pallas 141-144 vs 111-113 G products/s, BN254 121-124 vs 104-105,
// identical results on 4.2 M random products of each field.
__device__ __forceinline__ void acc_madd(uint64_t& acc, uint32_t& ov, uint32_t x, uint32_t y) {
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(ov)
      : "v"(x), "v"(y)
      : "vcc");
}
__device__ __forceinline__ void acc_maddc(uint64_t& acc, uint32_t& ov, uint32_t x, uint32_t y) {  // y uniform
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(ov)
      : "v"(x), "s"(y)
      : "vcc");
}
// a_i b_j and m_i p_j of one column step in one asm block: the compiler puts a wait state
// after every inline asm block, so two word products per block halve them (mulbench, r04l:
// pallas 147-150 vs 140-142 G products/s, BN254 128 vs 122-125, bit-identical)
__device__ __forceinline__ void acc_madd2(uint64_t& acc, uint32_t& ov, uint32_t x0, uint32_t y0,
                                          uint32_t x1, uint32_t y1) {  // y1 uniform
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
      "v_mad_u64_u32 %0, vcc, %4, %5, %0\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "+v"(acc), "+v"(ov)
      : "v"(x0), "v"(y0), "v"(x1), "s"(y1)
      : "vcc");
}
template <class F>
__device__ __forceinline__ Fe mul_comba(const Fe& a, const Fe& b) {
  uint32_t m[8], r[8];
  uint64_t acc = 0;
  uint32_t ov = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
#pragma unroll
    for (int i = 0; i < k; i++) {
      if (F::P[k - i]) acc_madd2(acc, ov, a.w[i], b.w[k - i], m[i], F::P[k - i]);
      else acc_madd(acc, ov, a.w[i], b.w[k - i]);
    }
    acc_madd(acc, ov, a.w[k], b.w[0]);
    m[k] = (uint32_t)acc * F::NP;
    acc_maddc(acc, ov, m[k], F::P[0]);  // the low word is now zero
    acc = (acc >> 32) | ((uint64_t)ov << 32);
    ov = 0;
  }
#pragma unroll
  for (int k = 8; k < 15; k++) {
#pragma unroll
    for (int i = k - 7; i < 8; i++) {
      if (F::P[k - i]) acc_madd2(acc, ov, a.w[i], b.w[k - i], m[i], F::P[k - i]);
      else acc_madd(acc, ov, a.w[i], b.w[k - i]);
    }
    r[k - 8] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)ov << 32);
    ov = 0;
  }
  r[7] = (uint32_t)acc;  // the result is < 2p < 2^256: nothing above this word
  Fe o;
#pragma unroll
  for (int j = 0; j < 8; j++) o.w[j] = r[j];
  return reduce_once<F>(o);
}

// The product the kernels use: the same product scanning as one generated asm block per field
// (b2f_mont_asm.h, tools/gen_mont_asm.py): the column accumulator stays in two fixed VGPR pairs
// and pallas' p_0 = 1 and p_7 = 2^30 words cost no multiplies (88 v_mad_u64_u32 against 104;
// BN254 128). mul_comba above is the per-step form it replaced (mulbench variant 0 vs 4,
// profiles/r05m_mulbench.txt: pallas 162 vs 153 G products/s, BN254 133-135 vs 126; in the
// kernels: lookup call 1.27 vs 1.31 ms, permutation z call 2.13 vs 2.21, r05m).
template <class F>
__device__ __forceinline__ Fe mul(const Fe& a, const Fe& b) {
#ifdef B2F_MUL_COMBA  // A/B builds only (tools/build_variant.sh)
  return mul_comba<F>(a, b);
#else
  return mul_asm<F>(a, b);
#endif
}

// The operand-scanning CIOS form the product had before (kept as the cross-check of mul in
// tools/mulbench.hip). The 32-bit sums that feed each
// v_mad_u64_u32 addend are formed with add-with-carry (the carry becomes the addend's high
// word) instead of 64-bit adds of zero-extended words: 20 % fewer instructions, ~1.25x the
// throughput on gfx950 (tools/mulbench.hip: 114 vs 90 G products/s chip-wide).
template <class F>
__device__ __forceinline__ Fe mul_cios(const Fe& a, const Fe& b) {
  uint32_t t[8];
#pragma unroll
  for (int j = 0; j < 8; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t bi = b.w[i];
    uint64_t x = (uint64_t)a.w[0] * bi + t[0];
    uint32_t A = (uint32_t)(x >> 32);
    const uint32_t t0 = (uint32_t)x;
    const uint32_t m = t0 * F::NP;
    uint64_t y = (uint64_t)m * F::P[0] + t0;
    uint32_t C = (uint32_t)(y >> 32);
#pragma unroll
    for (int j = 1; j < 8; j++) {
      unsigned co;
      const uint32_t s1 = __builtin_addc(t[j], A, 0u, &co);  // t_j + A
      x = (uint64_t)a.w[j] * bi + (((uint64_t)co << 32) | s1);
      A = (uint32_t)(x >> 32);
      const uint32_t s2 = __builtin_addc((uint32_t)x, C, 0u, &co);  // x_lo + C
      y = (uint64_t)m * F::P[j] + (((uint64_t)co << 32) | s2);
      C = (uint32_t)(y >> 32);
      t[j - 1] = (uint32_t)y;
    }
    t[7] = C + A;
  }
  Fe r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.w[j] = t[j];
  return reduce_once<F>(r);
}

template <class F>
__device__ __forceinline__ Fe add(const Fe& a, const Fe& b) {  // a + b < 2p < 2^256
  Fe s;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t x = (uint64_t)a.w[i] + b.w[i] + c;
    s.w[i] = (uint32_t)x;
    c = (uint32_t)(x >> 32);
  }
  return reduce_once<F>(s);
}

// Montgomery form of a small integer, x R mod p, without a Montgomery product: with c = R mod p
// (F::R), x c < 2^32 p, so the quotient fits 32 bits and q' = floor(x RQ / 2^64) is q or q - 1
// (x c / p - x RQ / 2^64 < x / 2^64 < 1). x c - q' p is in [0, 2p): computed mod 2^256 as 16
// word products, then one conditional subtraction (the generic route, mont(x, R^2), is 72).
template <class F>
__device__ __forceinline__ Fe from_u32(uint32_t x) {
  const uint32_t q = (uint32_t)__umul64hi((uint64_t)x, F::RQ);
  Fe w;
  uint64_t ca = 0, cb = 0;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t ta = (uint64_t)x * F::R[i] + ca;
    const uint64_t tb = (uint64_t)q * F::P[i] + cb;
    ca = ta >> 32;
    cb = tb >> 32;
    const uint64_t td = (uint64_t)(uint32_t)ta - (uint32_t)tb - br;
    w.w[i] = (uint32_t)td;
    br = (uint32_t)(td >> 63);
  }
  return reduce_once<F>(w);
}

// Montgomery form of a canonical element (< p)
template <class F>
__device__ __forceinline__ Fe to_mont(const Fe& a) {
  return mul<F>(a, fe_const<F>(F::R2));
}

// canonical value of a Montgomery-form element (PrimeField::to_repr as integer words)
template <class F>
__device__ __forceinline__ Fe to_canonical(const Fe& a) {
  Fe one_c = fe_zero();
  one_c.w[0] = 1;
  return mul<F>(a, one_c);
}

// a^(p-2) = a^-1 (a != 0): left-to-right square and multiply over the fixed exponent
// (~380 dependent products; kept as the cross-check of inv())
template <class F>
__device__ Fe inv_fermat(const Fe& a) {
  uint32_t e[8];  // p - 2
  uint32_t borrow = 2;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t x = (uint64_t)F::P[i] - borrow;
    e[i] = (uint32_t)x;
    borrow = (uint32_t)(x >> 63);
  }
  int top = 255;
  while (!((e[top >> 5] >> (top & 31)) & 1)) top--;
  Fe r = a;
#pragma unroll 1
  for (int bit = top - 1; bit >= 0; bit--) {
    r = mul<F>(r, r);
    if ((e[bit >> 5] >> (bit & 31)) & 1) r = mul<F>(r, a);
  }
  return r;
}

namespace detail {
__device__ __forceinline__ void shr1(uint32_t (&u)[8], uint32_t top) {  // u = (top:u) >> 1
#pragma unroll
  for (int i = 0; i < 7; i++) u[i] = (u[i] >> 1) | (u[i + 1] << 31);
  u[7] = (u[7] >> 1) | (top << 31);
}
// x / 2 mod p (x < p)
template <class F>
__device__ __forceinline__ void half_mod(uint32_t (&x)[8]) {
  uint32_t c = 0;
  if (x[0] & 1u) {  // x + p < 2p < 2^256
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint64_t s = (uint64_t)x[i] + F::P[i] + c;
      x[i] = (uint32_t)s;
      c = (uint32_t)(s >> 32);
    }
  }
  shr1(x, c);
}
// a = a - b; returns the borrow
__device__ __forceinline__ uint32_t sub_to(uint32_t (&a)[8], const uint32_t (&b)[8]) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t d = (uint64_t)a[i] - b[i] - br;
    a[i] = (uint32_t)d;
    br = (uint32_t)(d >> 63);
  }
  return br;
}
template <class F>
__device__ __forceinline__ void sub_mod(uint32_t (&a)[8], const uint32_t (&b)[8]) {
  if (sub_to(a, b)) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint64_t s = (uint64_t)a[i] + F::P[i] + c;
      a[i] = (uint32_t)s;
      c = (uint32_t)(s >> 32);
    }
  }
}
__device__ __forceinline__ bool is_one(const uint32_t (&u)[8]) {
  uint32_t o = u[0] ^ 1u;
#pragma unroll
  for (int i = 1; i < 8; i++) o |= u[i];
  return o == 0;
}
__device__ __forceinline__ bool geq(const uint32_t (&a)[8], const uint32_t (&b)[8]) {
  uint32_t t[8];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = a[i];
  return sub_to(t, b) == 0;
}
}  // namespace detail

// Montgomery-form inverse (a != 0): binary extended Euclid on the integer A = aR
// (u = A, v = p; x1 A = u, x2 A = v mod p), giving A^-1 = a^-1 R^-1, then one product with
// R^3: a^-1 R^-1 R^3 / R = a^-1 R. About 2 x 256 shift/subtract steps of 8-word integer work
// instead of ~380 field products; meant for one lane (its branches diverge per element).
template <class F>
__device__ Fe inv(const Fe& a) {
  using namespace detail;
  uint32_t u[8], v[8], x1[8], x2[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    u[i] = a.w[i];
    v[i] = F::P[i];
    x1[i] = 0;
    x2[i] = 0;
  }
  x1[0] = 1;
#pragma unroll 1
  while (!is_one(u) && !is_one(v)) {
#pragma unroll 1
    while (!(u[0] & 1u)) {
      shr1(u, 0);
      half_mod<F>(x1);
    }
#pragma unroll 1
    while (!(v[0] & 1u)) {
      shr1(v, 0);
      half_mod<F>(x2);
    }
    if (geq(u, v)) {
      sub_to(u, v);
      sub_mod<F>(x1, x2);
    } else {
      sub_to(v, u);
      sub_mod<F>(x2, x1);
    }
  }
  Fe r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.w[i] = is_one(u) ? x1[i] : x2[i];
  return mul<F>(r, fe_const<F>(F::R3));
}

namespace detail {
// (hi:u) >> sh for 0 < sh < 32, in place (funnel shifts)
__device__ __forceinline__ void shr_n(uint32_t (&u)[8], uint32_t sh) {
#pragma unroll
  for (int i = 0; i < 7; i++) u[i] = __builtin_amdgcn_alignbit(u[i + 1], u[i], sh);
  u[7] >>= sh;
}
// u << sh for 0 < sh < 32 (no carry out: callers keep u < 2^(256 - sh))
__device__ __forceinline__ void shl_n(uint32_t (&u)[8], uint32_t sh) {
#pragma unroll
  for (int i = 7; i > 0; i--) u[i] = __builtin_amdgcn_alignbit(u[i], u[i - 1], 32 - sh);
  u[0] <<= sh;
}
__device__ __forceinline__ void add_to(uint32_t (&a)[8], const uint32_t (&b)[8]) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t x = (uint64_t)a[i] + b[i] + c;
    a[i] = (uint32_t)x;
    c = (uint32_t)(x >> 32);
  }
}
__device__ __forceinline__ bool nonzero(const uint32_t (&u)[8]) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= u[i];
  return o != 0;
}
}  // namespace detail

// Montgomery-form inverse (a != 0) by Kaliski's almost-inverse with multi-bit shifts: on the
// integer A = aR, u = p, v = A, r = 0, s = 1 (invariant u s + v r = p, so r, s <= p < 2^255):
// an even u or v loses all its trailing zeros (up to 31) in one step while s or r doubles as
// often; otherwise the larger of u, v becomes (u - v) / 2 and r, s are updated. It ends with
// r = p - A^-1 2^k mod p, k in [255, 510] the halvings counted. Then x = A^-1 2^k, and two
// Montgomery products undo the powers of two: x 2^(512-k) R^-1 = A^-1 R = a^-1, times R2 R^-1
// = a^-1 R. About 270 steps of 8-word shift / add / subtract work per inverse against ~530 for
// the plain binary extended Euclid below, whose halvings each need a conditional add of p.
template <class F>
__device__ Fe inv_kaliski(const Fe& a) {
  using namespace detail;
  uint32_t u[8], v[8], r[8], s[8], pm[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    pm[i] = F::P[i];
    u[i] = F::P[i];
    v[i] = a.w[i];
    r[i] = 0;
    s[i] = 0;
  }
  s[0] = 1;
  uint32_t k = 0;
  // every step adds at least 1 to k <= 2 log2(p) < 512: the bound only guards the wave
#pragma unroll 1
  for (uint32_t it = 0; it < 512 && nonzero(v); it++) {
    if (!(u[0] & 1u)) {
      const uint32_t tz = u[0] ? (uint32_t)__builtin_ctz(u[0]) : 31u;
      shr_n(u, tz);
      shl_n(s, tz);
      k += tz;
    } else if (!(v[0] & 1u)) {
      const uint32_t tz = v[0] ? (uint32_t)__builtin_ctz(v[0]) : 31u;
      shr_n(v, tz);
      shl_n(r, tz);
      k += tz;
    } else if (!geq(v, u)) {  // u > v (u = v = 1 must take the other branch: v -> 0 ends)
      sub_to(u, v);
      shr_n(u, 1);
      add_to(r, s);
      shl_n(s, 1);
      k += 1;
    } else {
      sub_to(v, u);
      shr_n(v, 1);
      add_to(s, r);
      shl_n(r, 1);
      k += 1;
    }
  }
  // x = p - (r mod p)
  if (geq(r, pm)) sub_to(r, pm);
  uint32_t x[8];
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = pm[i];
  sub_to(x, r);
  // y = 2^(512 - k) mod p: 2^min(j, 253) (< p for both moduli), then doublings mod p
  const uint32_t j = 512u - k;
  const uint32_t j0 = j < 253u ? j : 253u;
  uint32_t y[8];
#pragma unroll
  for (int i = 0; i < 8; i++) y[i] = (uint32_t)(i == (int)(j0 >> 5)) << (j0 & 31u);
#pragma unroll 1
  for (uint32_t d = j0; d < j; d++) {
    shl_n(y, 1);  // y < p < 2^255: no carry out
    if (geq(y, pm)) sub_to(y, pm);
  }
  Fe X, Y;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    X.w[i] = x[i];
    Y.w[i] = y[i];
  }
  return mul<F>(mul<F>(X, Y), fe_const<F>(F::R2));
}

// Montgomery-form inverse by Bernstein-Yang divsteps (b2f_safegcd.h) on the integer A = aR:
// A^-1 = a^-1 R^-1, then one product with R^3 gives a^-1 R. About 20 steps of 30 divsteps and
// two 2x2-matrix updates of 9-limb vectors against Kaliski's ~270 single-bit steps of 8-word
// work (inv_kaliski, kept as a cross-check); one lane, a = 0 gives 0. `ok` is cleared when the
// divsteps did not converge (never for a < p; the callers raise B2F_ERR_CHECK on it).
template <class F>
__device__ Fe inv_safegcd(const Fe& a, bool& ok) {
  uint32_t x[8], pw[8], o[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x[i] = a.w[i];
    pw[i] = F::P[i];
  }
  ok = sgcd::inverse(x, pw, o);
  Fe r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.w[i] = o[i];
  return mul<F>(r, fe_const<F>(F::R3));
}

__device__ __forceinline__ bool is_zero(const Fe& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a.w[i];
  return o == 0;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void store(uint64_t* p, const Fe& a) {
  u32x4* q = reinterpret_cast<u32x4*>(p);
  q[0] = u32x4{a.w[0], a.w[1], a.w[2], a.w[3]};
  q[1] = u32x4{a.w[4], a.w[5], a.w[6], a.w[7]};
}
__device__ __forceinline__ Fe load(const uint64_t* p) {
  const u32x4* q = reinterpret_cast<const u32x4*>(p);
  const u32x4 x = q[0], y = q[1];
  Fe r;
  r.w[0] = x.x; r.w[1] = x.y; r.w[2] = x.z; r.w[3] = x.w;
  r.w[4] = y.x; r.w[5] = y.y; r.w[6] = y.z; r.w[7] = y.w;
  return r;
}
__device__ __forceinline__ Fe load_words(const uint64_t* c) {  // 4 LE u64 limbs
  Fe r;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    r.w[2 * i] = (uint32_t)c[i];
    r.w[2 * i + 1] = (uint32_t)(c[i] >> 32);
  }
  return r;
}

}  // namespace field
}  // namespace b2f

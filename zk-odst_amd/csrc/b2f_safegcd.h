// b2f_safegcd.h -- modular inversion by Bernstein-Yang divsteps ("safegcd", variable-time form),
// for the one-lane inversions of the grand products (b2f_gprod.h gp_inv, the lookup's
// lk_nscan_kernel). Plain C++ on 32-bit limbs, __host__ __device__ so tools/ can check it
// against big-integer arithmetic on the CPU.
//
// Numbers are signed-30 limb vectors: value = sum v[i] 2^(30 i), i < 9 (270 bits). One outer
// step runs 30 divsteps on the low 32 bits of f and g only, collecting them in a 2x2 matrix
// t (entries < 2^30 in magnitude, scaled by 2^30), then applies t to the full f, g (exact
// division by 2^30) and to d, e (mod p: a multiple of p is added so the division is exact).
// Divsteps (Bernstein, Yang, "Fast constant-time gcd computation and modular inversion", 2019),
// in the eta = -delta form with zero runs taken at once and up to 8 low bits of g cancelled per
// step by a multiple of f (an inverse of f mod 2^8 by Newton iteration). The invariants
// (f odd; u f0 + v g0 = f 2^k, q f0 + r g0 = g 2^k after k divsteps; d x = f, e x = g mod p
// up to the accumulated powers of two, which the exact divisions by 2^30 remove) end with
// g = 0, f = +-1 and d = +-x^-1 mod p. About 20 outer steps for a 256-bit modulus against
// 2 x 256 single-bit steps of Kaliski's almost-inverse.
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#ifndef __host__
#define __host__
#endif
#ifndef __device__
#define __device__
#endif
#endif

namespace b2f {
namespace sgcd {

struct S30 {
  int32_t v[9];
};
struct T2 {
  int32_t u, v, q, r;
};
constexpr uint32_t M30 = 0x3fffffffu;

__host__ __device__ inline int ctz32(uint32_t x) { return __builtin_ctz(x); }

// 8 words little-endian (< 2^256) <-> signed-30 limbs (all limbs in [0, 2^30) but the top)
__host__ __device__ inline S30 from_words(const uint32_t (&w)[8]) {
  S30 r;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int bit = 30 * i, k = bit >> 5, sh = bit & 31;
    uint64_t x = (uint64_t)w[k < 8 ? k : 7] >> sh;
    if (k >= 8) x = 0;
    if (k + 1 < 8) x |= (uint64_t)w[k + 1] << (32 - sh);
    r.v[i] = (int32_t)(x & M30);
  }
  return r;
}
__host__ __device__ inline void to_words(const S30& a, uint32_t (&w)[8]) {
  // a is normalised: limbs in [0, 2^30), value < 2^256
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int bit = 32 * k, i = bit / 30, sh = bit % 30;
    uint64_t x = (uint64_t)(uint32_t)a.v[i] >> sh;
    if (i + 1 < 9) x |= (uint64_t)(uint32_t)a.v[i + 1] << (30 - sh);
    if (i + 2 < 9) x |= (uint64_t)(uint32_t)a.v[i + 2] << (60 - sh);
    w[k] = (uint32_t)x;
  }
}

// 30 divsteps on the low bits of f, g (f odd); returns the new eta
__host__ __device__ inline int32_t divsteps_30(int32_t eta, uint32_t f0, uint32_t g0, T2& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1, f = f0, g = g0;
  int i = 30;
  for (;;) {
    // a sentinel bit counts zeros only up to i: that many divsteps just halve g
    const int zeros = ctz32(g | (0xffffffffu << i));
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    // f, g odd: if eta < 0, (f, g) <- (g, -f) with the matrix rows swapped and negated
    if (eta < 0) {
      uint32_t tmp;
      eta = -eta;
      tmp = f; f = g; g = 0u - tmp;
      tmp = u; u = q; q = 0u - tmp;
      tmp = v; v = r; r = 0u - tmp;
    }
    // cancel up to min(eta + 1, i, 8) low bits of g with a multiple w of f
    const int limit = (eta + 1) > i ? i : (eta + 1);
    const uint32_t m = (0xffffffffu >> (32 - limit)) & 255u;
    uint32_t x = f;               // f^-1 mod 2^8: 3 correct bits (f odd), Newton doubles them
    x *= 2u - f * x;
    x *= 2u - f * x;
    const uint32_t w = (0u - g * x) & m;
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t.u = (int32_t)u;
  t.v = (int32_t)v;
  t.q = (int32_t)q;
  t.r = (int32_t)r;
  return eta;
}

// [f, g] <- t [f, g] / 2^30 (exact)
__host__ __device__ inline void update_fg(S30& f, S30& g, const T2& t) {
  const int64_t u = t.u, v = t.v, q = t.q, r = t.r;
  int64_t cf = u * f.v[0] + v * g.v[0];
  int64_t cg = q * f.v[0] + r * g.v[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    const int64_t fi = f.v[i], gi = g.v[i];
    cf += u * fi + v * gi;
    cg += q * fi + r * gi;
    f.v[i - 1] = (int32_t)((uint32_t)cf & M30);
    g.v[i - 1] = (int32_t)((uint32_t)cg & M30);
    cf >>= 30;
    cg >>= 30;
  }
  f.v[8] = (int32_t)cf;
  g.v[8] = (int32_t)cg;
}

// [d, e] <- (t [d, e] + p [md, me]) / 2^30 with md, me making the low 30 bits zero (d, e stay
// in (-2p, p)); pinv30 = p^-1 mod 2^30
__host__ __device__ inline void update_de(S30& d, S30& e, const T2& t, const S30& p, uint32_t pinv30) {
  const int32_t u = t.u, v = t.v, q = t.q, r = t.r;
  const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
  int32_t md = (u & sd) + (v & se);
  int32_t me = (q & sd) + (r & se);
  int64_t cd = (int64_t)u * d.v[0] + (int64_t)v * e.v[0];
  int64_t ce = (int64_t)q * d.v[0] + (int64_t)r * e.v[0];
  md -= (int32_t)((pinv30 * (uint32_t)cd + (uint32_t)md) & M30);
  me -= (int32_t)((pinv30 * (uint32_t)ce + (uint32_t)me) & M30);
  cd += (int64_t)p.v[0] * md;
  ce += (int64_t)p.v[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    const int64_t di = d.v[i], ei = e.v[i];
    cd += (int64_t)u * di + (int64_t)v * ei + (int64_t)p.v[i] * md;
    ce += (int64_t)q * di + (int64_t)r * ei + (int64_t)p.v[i] * me;
    d.v[i - 1] = (int32_t)((uint32_t)cd & M30);
    e.v[i - 1] = (int32_t)((uint32_t)ce & M30);
    cd >>= 30;
    ce >>= 30;
  }
  d.v[8] = (int32_t)cd;
  e.v[8] = (int32_t)ce;
}

// r in (-2p, p), negated when sign < 0, to [0, p) with limbs in [0, 2^30)
__host__ __device__ inline void normalize(S30& r, int32_t sign, const S30& p) {
  int32_t c = r.v[8] >> 31;  // add p if negative
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] += p.v[i] & c;
  const int32_t neg = sign >> 31;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = (r.v[i] ^ neg) - neg;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.v[i + 1] += r.v[i] >> 30;
    r.v[i] &= (int32_t)M30;
  }
  c = r.v[8] >> 31;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] += p.v[i] & c;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.v[i + 1] += r.v[i] >> 30;
    r.v[i] &= (int32_t)M30;
  }
}

// x^-1 mod p (x < p, as 8 words; x = 0 gives 0), p odd < 2^256 as 8 words. Returns whether the
// divsteps converged -- g reached 0 with f = +-1 (gcd 1; for x = 0, f = +-p and out = 0) --
// within the 40 outer steps: ~25 suffice for 256 bits, so false means an input outside the
// contract (x >= p, a modulus change) and `out` is not an inverse.
__host__ __device__ inline bool inverse(const uint32_t (&x)[8], const uint32_t (&pw)[8], uint32_t (&out)[8]) {
  const S30 p = from_words(pw);
  uint32_t pinv = pw[0];  // p^-1 mod 2^32 by Newton (p odd)
  for (int i = 0; i < 5; i++) pinv *= 2u - pw[0] * pinv;
  const uint32_t pinv30 = pinv & M30;
  S30 d = {{0, 0, 0, 0, 0, 0, 0, 0, 0}}, e = {{1, 0, 0, 0, 0, 0, 0, 0, 0}};
  S30 f = p, g = from_words(x);
  int32_t eta = -1;
  bool done = false;
  for (int it = 0; it < 40 && !done; it++) {  // 25 steps suffice for 256 bits (<= 750 divsteps)
    T2 t;
    eta = divsteps_30(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], t);
    update_de(d, e, t, p, pinv30);
    update_fg(f, g, t);
    int32_t nz = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) nz |= g.v[i];
    done = nz == 0;
  }
  // f = +-1 (x invertible; -1 is limbs 0..7 = 2^30 - 1, limb 8 = -1) or +-p (x = 0, d stays 0)
  int32_t one = f.v[0] == 1 && f.v[8] == 0, mone = f.v[0] == (int32_t)M30 && f.v[8] == -1, zx = 1;
#pragma unroll
  for (int i = 1; i < 8; i++) {
    one &= f.v[i] == 0;
    mone &= f.v[i] == (int32_t)M30;
  }
  const int32_t unit = one | mone;
#pragma unroll
  for (int i = 0; i < 9; i++) zx &= d.v[i] == 0;
  normalize(d, f.v[8], p);
  to_words(d, out);
  return done && (unit || zx);
}

}  // namespace sgcd
}  // namespace b2f

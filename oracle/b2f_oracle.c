/*
 * b2f_oracle.c -- CPU restatement (TEST INFRASTRUCTURE ONLY; see b2f_oracle.h).
 *
 * The fill follows the reference's region-assignment style: every block is an
 * `assign_region`-like helper that writes lookup rows (SpreadVar::with_lookup,
 * spread_table.rs:257-285), operand cells through `copy_advice` (table16.rs:431-433) and
 * enables selectors (compression_util.rs:214), one instance at a time
 * (CompressionConfig::{initialize_with_iv, compress, digest}, compression.rs:1078-1149).
 * The same synthesize routine runs in "structure" mode (no witness values, like halo2
 * keygen) to enumerate the copy constraints the eval checks.
 */
#include "b2f_oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { A0, A1, A2, A3, A4, A5, A6, A7, A8, A9 };
enum {
    S_ABCD = 0, S_EFGH, S_IJKL, S_A1, S_B1, S_C1, S_D1, S_A2, S_B2, S_C2, S_D2,
    S_DIGEST, S_XOR, S_XOR3, S_CONST, S_FMASK
};

/* table16.rs:47-56 */
static const uint64_t IV[8] = {
    0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
    0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
    0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

/* table16.rs:32-44 (ROUND_CONSTANTS = SIGMA) */
static const uint8_t SIGMA[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

/* README.md:42-51: the four column Mixes then the four diagonal Mixes */
static const uint8_t GIDX[8][4] = {{0, 4, 8, 12}, {1, 5, 9, 13}, {2, 6, 10, 14}, {3, 7, 11, 15},
                                   {0, 5, 10, 15}, {1, 6, 11, 12}, {2, 7, 8, 13}, {3, 4, 9, 14}};

#define INIT_ROWS 164u
#define ROUND_ROWS 416u
#define FINAL_ROWS 64u

static inline uint64_t rotr64(uint64_t x, unsigned n) { return (x >> n) | (x << (64 - n)); }
static inline uint32_t limb(uint64_t w, unsigned k) { return (uint32_t)((w >> (16 * k)) & 0xffff); }

/* util.rs:61-75 spread_bits: bit i of the input goes to bit 2i. */
static uint32_t spread16(uint32_t x) {
    uint32_t s = 0;
    for (int b = 0; b < 16; b++) s |= ((x >> b) & 1u) << (2 * b);
    return s;
}

/* spread_table.rs:213-222 */
static uint32_t get_tag(uint32_t x) { return x < (1u << 8) ? 0u : (x < (1u << 15) ? 1u : 2u); }

uint64_t orc_rows(uint32_t rounds) {
    return (uint64_t)INIT_ROWS + (uint64_t)ROUND_ROWS * rounds + FINAL_ROWS;
}

void orc_offsets(const orc_input* in, size_t n, uint64_t* offsets) {
    offsets[0] = 0;
    for (size_t i = 0; i < n; i++) offsets[i + 1] = offsets[i] + orc_rows(in[i].rounds);
}

void orc_compress(uint32_t rounds, const uint64_t h[8], const uint64_t m[16],
                  const uint64_t t[2], uint32_t f, uint64_t out[8]) {
    uint64_t v[16];
    for (int i = 0; i < 8; i++) { v[i] = h[i]; v[i + 8] = IV[i]; }
    v[12] ^= t[0];
    v[13] ^= t[1];
    if (f) v[14] = ~v[14];
    for (uint32_t r = 0; r < rounds; r++) {
        const uint8_t* s = SIGMA[r % 10];
        for (int g = 0; g < 8; g++) {
            int a = GIDX[g][0], b = GIDX[g][1], c = GIDX[g][2], d = GIDX[g][3];
            v[a] = v[a] + v[b] + m[s[2 * g]];
            v[d] = rotr64(v[d] ^ v[a], 32);
            v[c] = v[c] + v[d];
            v[b] = rotr64(v[b] ^ v[c], 24);
            v[a] = v[a] + v[b] + m[s[2 * g + 1]];
            v[d] = rotr64(v[d] ^ v[a], 16);
            v[c] = v[c] + v[d];
            v[b] = rotr64(v[b] ^ v[c], 63);
        }
    }
    for (int i = 0; i < 8; i++) out[i] = h[i] ^ v[i] ^ v[i + 8];
}

/* ------------------------------------------------------------------ region model */

typedef struct { uint32_t row; uint8_t col; } cell_t;
typedef struct {
    uint64_t val;
    cell_t d[4]; /* canonical dense cell of limb k */
    cell_t s[4]; /* canonical spread cell of limb k */
} word_t;

typedef struct {
    uint32_t* adv;      /* column-major, NULL in structure mode */
    uint32_t* fixed;    /* NULL in structure mode */
    uint64_t stride;    /* total rows */
    uint64_t base;      /* first global row of the instance */
    uint32_t* copies;   /* structure mode: (dst_row, dst_col, src_row, src_col) */
    size_t ncopies, cap;
    int record;         /* structure mode: count (and store up to cap) copy pairs */
    /* test-only tampering (orc_fill_tampered): 1 = the ADD block at tamper_row adds
     * tamper_delta to its sum and leaves its selector off; 2 = the CONST block at tamper_row
     * uses IV ^ tamper_delta (advice and k_0 alike) */
    int tamper_kind;
    uint32_t tamper_row;
    uint64_t tamper_delta;
} region_t;

static inline void put(region_t* R, int col, uint32_t row, uint32_t v) {
    if (R->adv) R->adv[(uint64_t)col * R->stride + R->base + row] = v;
}
static inline uint32_t get(const region_t* R, int col, uint32_t row) {
    return R->adv ? R->adv[(uint64_t)col * R->stride + R->base + row] : 0u;
}
static inline void enable(region_t* R, int sel, uint32_t row) {
    if (R->fixed) R->fixed[R->base + row] |= 1u << sel;
}
static inline void set_const(region_t* R, uint32_t row, uint32_t k) {
    if (R->fixed) R->fixed[R->base + row] |= k << 16;
}
/* copy_advice: the destination takes the source cell's value and the pair is recorded. */
static void copy_cell(region_t* R, int dcol, uint32_t drow, cell_t src) {
    put(R, dcol, drow, get(R, src.col, src.row));
    if (R->record) {
        if (R->copies && R->ncopies < R->cap) {
            uint32_t* q = R->copies + 4 * R->ncopies;
            q[0] = drow; q[1] = (uint32_t)dcol; q[2] = src.row; q[3] = src.col;
        }
        R->ncopies++;
    }
}
/* SpreadVar::with_lookup (spread_table.rs:257-285) */
static void lookup_row(region_t* R, uint32_t row, uint32_t x) {
    put(R, A0, row, get_tag(x));
    put(R, A1, row, x);
    put(R, A2, row, spread16(x));
}
static cell_t C(uint32_t row, int col) { cell_t c = {row, (uint8_t)col}; return c; }

/* ------------------------------------------------------------------ blocks (LAYOUT.md §4) */

static word_t blk_inw(region_t* R, uint32_t r0, uint64_t w) {
    word_t o; o.val = w;
    for (unsigned k = 0; k < 4; k++) {
        lookup_row(R, r0 + k, limb(w, k));
        o.d[k] = C(r0 + k, A1); o.s[k] = C(r0 + k, A2);
    }
    put(R, A7, r0, (uint32_t)w);
    put(R, A8, r0, (uint32_t)(w >> 32));
    enable(R, S_ABCD, r0);
    return o;
}

static word_t blk_const(region_t* R, uint32_t r0, uint64_t w) {
    if (R->tamper_kind == 2 && r0 == R->tamper_row) w ^= R->tamper_delta;
    word_t o; o.val = w;
    for (unsigned k = 0; k < 4; k++) {
        lookup_row(R, r0 + k, limb(w, k));
        set_const(R, r0 + k, limb(w, k));
        enable(R, S_CONST, r0 + k);
        o.d[k] = C(r0 + k, A1); o.s[k] = C(r0 + k, A2);
    }
    return o;
}

static word_t blk_fmask(region_t* R, uint32_t r0, uint32_t f) {
    word_t o; o.val = f ? ~0ULL : 0ULL;
    for (unsigned k = 0; k < 4; k++) {
        lookup_row(R, r0 + k, f ? 0xffffu : 0u);
        o.d[k] = C(r0 + k, A1); o.s[k] = C(r0 + k, A2);
    }
    put(R, A5, r0, f ? 1u : 0u);
    enable(R, S_FMASK, r0);
    return o;
}

/* XOR with rotation rho in {0, 16, 32}: output is a relabelling of the z limbs. */
static word_t blk_xor(region_t* R, uint32_t r0, const word_t* X, const word_t* Y, int sel,
                      unsigned rho) {
    uint64_t z = X->val ^ Y->val, a = X->val & Y->val;
    for (unsigned k = 0; k < 4; k++) {
        lookup_row(R, r0 + 2 * k, limb(z, k));
        lookup_row(R, r0 + 2 * k + 1, limb(a, k));
        copy_cell(R, A3, r0 + 2 * k, X->s[k]);
        copy_cell(R, A4, r0 + 2 * k, Y->s[k]);
    }
    enable(R, sel, r0);
    word_t o; o.val = rho ? rotr64(z, rho) : z;
    for (unsigned k = 0; k < 4; k++) {
        uint32_t src = r0 + 2 * ((k + rho / 16) & 3);
        o.d[k] = C(src, A1); o.s[k] = C(src, A2);
    }
    return o;
}

static word_t blk_xor24(region_t* R, uint32_t r0, const word_t* X, const word_t* Y) {
    uint64_t z = X->val ^ Y->val, a = X->val & Y->val, w = rotr64(z, 24);
    word_t o; o.val = w;
    for (unsigned k = 0; k < 4; k++) {
        uint32_t zk = limb(z, k), wk = limb(w, k);
        lookup_row(R, r0 + 3 * k, zk & 0xff);
        lookup_row(R, r0 + 3 * k + 1, zk >> 8);
        lookup_row(R, r0 + 3 * k + 2, limb(a, k));
        copy_cell(R, A3, r0 + 3 * k, X->s[k]);
        copy_cell(R, A4, r0 + 3 * k, Y->s[k]);
        put(R, A7, r0 + 3 * k, wk);
        put(R, A8, r0 + 3 * k, spread16(wk));
        o.d[k] = C(r0 + 3 * k, A7); o.s[k] = C(r0 + 3 * k, A8);
    }
    enable(R, S_B1, r0);
    enable(R, S_EFGH, r0);
    return o;
}

static word_t blk_xor63(region_t* R, uint32_t r0, const word_t* X, const word_t* Y) {
    uint64_t z = X->val ^ Y->val, a = X->val & Y->val, w = rotr64(z, 63);
    word_t o; o.val = w;
    for (unsigned k = 0; k < 4; k++) {
        uint32_t zk = limb(z, k), wk = limb(w, k);
        lookup_row(R, r0 + 2 * k, zk & 0x7fff);
        lookup_row(R, r0 + 2 * k + 1, limb(a, k));
        copy_cell(R, A3, r0 + 2 * k, X->s[k]);
        copy_cell(R, A4, r0 + 2 * k, Y->s[k]);
        put(R, A6, r0 + 2 * k, zk >> 15);
        put(R, A7, r0 + 2 * k, wk);
        put(R, A8, r0 + 2 * k, spread16(wk));
        o.d[k] = C(r0 + 2 * k, A7); o.s[k] = C(r0 + 2 * k, A8);
    }
    enable(R, S_B2, r0);
    enable(R, S_IJKL, r0);
    return o;
}

static word_t blk_add(region_t* R, uint32_t r0, const word_t* A, const word_t* B,
                      const word_t* M, int sel) {
    unsigned __int128 full = (unsigned __int128)A->val + B->val + (M ? M->val : 0);
    uint64_t s = (uint64_t)full;
    const int tampered = R->tamper_kind == 1 && r0 == R->tamper_row;
    if (tampered) s += R->tamper_delta;
    word_t o; o.val = s;
    for (unsigned k = 0; k < 4; k++) {
        lookup_row(R, r0 + k, limb(s, k));
        copy_cell(R, A3, r0 + k, A->d[k]);
        copy_cell(R, A4, r0 + k, B->d[k]);
        if (M) copy_cell(R, A5, r0 + k, M->d[k]);
        o.d[k] = C(r0 + k, A1); o.s[k] = C(r0 + k, A2);
    }
    put(R, A9, r0, (uint32_t)(full >> 64));
    if (!tampered) enable(R, sel, r0);
    return o;
}

static uint64_t blk_xor3(region_t* R, uint32_t r0, const word_t* H, const word_t* V,
                         const word_t* U) {
    uint64_t e = H->val ^ V->val ^ U->val;
    uint64_t j = (H->val & V->val) | (H->val & U->val) | (V->val & U->val);
    for (unsigned k = 0; k < 4; k++) {
        lookup_row(R, r0 + 2 * k, limb(e, k));
        lookup_row(R, r0 + 2 * k + 1, limb(j, k));
        copy_cell(R, A3, r0 + 2 * k, H->s[k]);
        copy_cell(R, A4, r0 + 2 * k, V->s[k]);
        copy_cell(R, A5, r0 + 2 * k, U->s[k]);
    }
    put(R, A7, r0, (uint32_t)e);
    put(R, A8, r0, (uint32_t)(e >> 32));
    enable(R, S_XOR3, r0);
    enable(R, S_DIGEST, r0);
    return e;
}

/* One instance: initialize (subregion_initial.rs:11-52 intent), compress, digest. */
static void synthesize(region_t* R, const orc_input* in, uint64_t out[8]) {
    static const orc_input zero;
    if (!in) in = &zero;
    word_t h[8], m[16], v[16], iv[8];
    for (int i = 0; i < 8; i++) h[i] = blk_inw(R, 4 * i, in->h[i]);
    for (int j = 0; j < 16; j++) m[j] = blk_inw(R, 32 + 4 * j, in->m[j]);
    word_t t0 = blk_inw(R, 96, in->t[0]);
    word_t t1 = blk_inw(R, 100, in->t[1]);
    word_t fm = blk_fmask(R, 104, in->f);
    for (int i = 0; i < 8; i++) iv[i] = blk_const(R, 108 + 4 * i, IV[i]);
    for (int i = 0; i < 8; i++) v[i] = h[i];
    for (int i = 0; i < 4; i++) v[8 + i] = iv[i];
    v[15] = iv[7];
    v[12] = blk_xor(R, 140, &iv[4], &t0, S_XOR, 0);
    v[13] = blk_xor(R, 148, &iv[5], &t1, S_XOR, 0);
    v[14] = blk_xor(R, 156, &iv[6], &fm, S_XOR, 0);
    for (uint32_t r = 0; r < in->rounds; r++) {
        const uint8_t* s = SIGMA[r % 10];
        uint32_t base = INIT_ROWS + ROUND_ROWS * r;
        for (int g = 0; g < 8; g++) {
            int ia = GIDX[g][0], ib = GIDX[g][1], ic = GIDX[g][2], id = GIDX[g][3];
            uint32_t gb = base + 52 * g;
            word_t a = blk_add(R, gb + 0, &v[ia], &v[ib], &m[s[2 * g]], S_A1);
            word_t d = blk_xor(R, gb + 4, &v[id], &a, S_D1, 32);
            word_t c = blk_add(R, gb + 12, &v[ic], &d, NULL, S_C1);
            word_t b = blk_xor24(R, gb + 16, &v[ib], &c);
            word_t a2 = blk_add(R, gb + 28, &a, &b, &m[s[2 * g + 1]], S_A2);
            word_t d2 = blk_xor(R, gb + 32, &d, &a2, S_D2, 16);
            word_t c2 = blk_add(R, gb + 40, &c, &d2, NULL, S_C2);
            word_t b2 = blk_xor63(R, gb + 44, &b, &c2);
            v[ia] = a2; v[ib] = b2; v[ic] = c2; v[id] = d2;
        }
    }
    uint32_t fb = INIT_ROWS + ROUND_ROWS * in->rounds;
    for (int i = 0; i < 8; i++) {
        uint64_t e = blk_xor3(R, fb + 8 * i, &h[i], &v[i], &v[i + 8]);
        if (out) out[i] = e;
    }
}

/* Structure-mode synthesize: the rounds value is the only input the structure depends on. */
size_t orc_copies(uint32_t rounds, uint32_t* out4, size_t cap) {
    orc_input in;
    memset(&in, 0, sizeof in);
    in.rounds = rounds;
    region_t R;
    memset(&R, 0, sizeof R);
    R.copies = out4;
    R.cap = out4 ? cap : 0;
    R.record = 1;
    synthesize(&R, &in, NULL);
    return R.ncopies;
}

/* Structure-mode synthesize of the fixed column of one instance (rows [0, R(rounds))). */
static void fixed_structure(uint32_t rounds, uint32_t* fixed) {
    orc_input in;
    memset(&in, 0, sizeof in);
    in.rounds = rounds;
    memset(fixed, 0, orc_rows(rounds) * sizeof(uint32_t));
    region_t R;
    memset(&R, 0, sizeof R);
    R.fixed = fixed;
    synthesize(&R, &in, NULL);
}

static int rows_ok(uint64_t R) {
    return R >= INIT_ROWS + FINAL_ROWS && (R - INIT_ROWS - FINAL_ROWS) % ROUND_ROWS == 0;
}

int orc_fixed(const uint64_t* offsets, size_t n, uint64_t total_rows, uint32_t* fixed) {
    if (offsets[0] != 0 || offsets[n] > total_rows) return -1;
    for (size_t i = 0; i < n; i++)
        if (offsets[i + 1] < offsets[i] || !rows_ok(offsets[i + 1] - offsets[i])) return -1;
    memset(fixed, 0, total_rows * sizeof(uint32_t));
    for (size_t i = 0; i < n; i++)
        fixed_structure((uint32_t)((offsets[i + 1] - offsets[i] - INIT_ROWS - FINAL_ROWS) / ROUND_ROWS),
                        fixed + offsets[i]);
    return 0;
}

/* ---------------------------------------------------------------- Fp export (§8(f) row 1)
 * Two prime fields, both in-memory Montgomery form with R = 2^256:
 *   pallas::Base of pasta_curves 0.5.1 (Cargo.lock:1334-1337);
 *   BN254 Fr of halo2curves 0.3.2 (Cargo.lock:859-861; the reference's circuit field,
 *   blake2f.rs:283,293, blake2f_circuit_bench.rs:10,34).
 * Textbook restatement: R^2 mod p by 512 modular doublings of 1, n0 = -p^-1 mod 2^64 by
 * Newton iteration, mont(x) = CIOS(x, R^2) with the full carry word. */
static const uint64_t FP_MODULI[2][4] = {
    {0x992d30ed00000001ull, 0x224698fc094cf91bull, 0ull, 0x4000000000000000ull},
    {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull, 0x30644e72e131a029ull}};

static int fp_geq(const uint64_t a[4], const uint64_t b[4]) {
    for (int i = 3; i >= 0; i--) {
        if (a[i] != b[i]) return a[i] > b[i];
    }
    return 1;
}

static void fp_sub(uint64_t a[4], const uint64_t b[4]) {
    unsigned __int128 borrow = 0;
    for (int i = 0; i < 4; i++) {
        unsigned __int128 d = (unsigned __int128)a[i] - b[i] - borrow;
        a[i] = (uint64_t)d;
        borrow = (d >> 64) ? 1 : 0;
    }
}

static void fp_consts(const uint64_t p[4], uint64_t r2[4], uint64_t* n0) {
    uint64_t v[4] = {1, 0, 0, 0};
    for (int k = 0; k < 512; k++) { /* v = 2v mod p; v < p < 2^255 so 2v fits */
        uint64_t c = 0;
        for (int i = 0; i < 4; i++) {
            uint64_t nc = v[i] >> 63;
            v[i] = (v[i] << 1) | c;
            c = nc;
        }
        if (fp_geq(v, p)) fp_sub(v, p);
    }
    memcpy(r2, v, sizeof v);
    uint64_t inv = 1;
    for (int i = 0; i < 6; i++) inv *= 2 - p[0] * inv;
    *n0 = 0 - inv;
}

/* CIOS Montgomery product a*b*2^-256 mod p */
static void fp_mont_mul(const uint64_t p[4], const uint64_t a[4], const uint64_t b[4], uint64_t n0,
                        uint64_t out[4]) {
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; i++) {
        unsigned __int128 c = 0;
        for (int j = 0; j < 4; j++) {
            c += (unsigned __int128)a[j] * b[i] + t[j];
            t[j] = (uint64_t)c;
            c >>= 64;
        }
        c += t[4];
        t[4] = (uint64_t)c;
        t[5] = (uint64_t)(c >> 64);
        uint64_t m = t[0] * n0;
        c = (unsigned __int128)m * p[0] + t[0];
        c >>= 64;
        for (int j = 1; j < 4; j++) {
            c += (unsigned __int128)m * p[j] + t[j];
            t[j - 1] = (uint64_t)c;
            c >>= 64;
        }
        c += t[4];
        t[3] = (uint64_t)c;
        t[4] = t[5] + (uint64_t)(c >> 64);
    }
    uint64_t r[4] = {t[0], t[1], t[2], t[3]};
    if (t[4] || fp_geq(r, p)) fp_sub(r, p);
    memcpy(out, r, sizeof r);
}

/* field 0 = pasta Fp, 1 = BN254 Fr */
void orc_fp_mont(uint32_t field, uint32_t x, uint64_t out[4]) {
    const uint64_t* p = FP_MODULI[field & 1];
    uint64_t r2[4], n0;
    fp_consts(p, r2, &n0);
    uint64_t a[4] = {x, 0, 0, 0};
    fp_mont_mul(p, a, r2, n0, out);
}

/* form: bit 0 = Montgomery, bit 1 = BN254 Fr (B2F_FP_*) */
void orc_export_fp(const uint32_t* advice, uint64_t total_rows, uint64_t row_begin,
                   uint64_t nrows, uint32_t form, uint64_t* out, uint64_t out_rows) {
    static const int a_of_h[10] = {5, 3, 4, 6, 7, 8, 9, 0, 1, 2}; /* table16.rs:281-294 */
    const uint64_t* p = FP_MODULI[(form >> 1) & 1];
    uint64_t r2[4], n0;
    fp_consts(p, r2, &n0);
    for (int h = 0; h < 10; h++) {
        const uint32_t* src = advice + (uint64_t)a_of_h[h] * total_rows + row_begin;
        uint64_t* dst = out + (uint64_t)h * out_rows * 4;
        for (uint64_t r = 0; r < nrows; r++) {
            uint64_t a[4] = {src[r], 0, 0, 0};
            if (form & 1) fp_mont_mul(p, a, r2, n0, dst + 4 * r);
            else memcpy(dst + 4 * r, a, sizeof a);
        }
    }
}

int orc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

static int fill_impl(const orc_input* in, size_t n, const uint64_t* offsets, uint64_t total_rows,
                     uint32_t* advice, uint32_t* fixed, uint64_t* h_out, int nthreads,
                     size_t t_inst, int t_kind, uint32_t t_row, uint64_t t_delta) {
    for (size_t i = 0; i < n; i++)
        if (offsets[i + 1] - offsets[i] != orc_rows(in[i].rounds)) return -1;
    if (offsets[n] > total_rows) return -1;
    /* rows past the last instance (if any) are left zero */
    for (int c = 0; c < ORC_NCOLS; c++)
        memset(advice + (uint64_t)c * total_rows + offsets[n], 0,
               (total_rows - offsets[n]) * sizeof(uint32_t));
    memset(fixed + offsets[n], 0, (total_rows - offsets[n]) * sizeof(uint32_t));
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads)
#endif
    for (long long i = 0; i < (long long)n; i++) {
        uint64_t rows = offsets[i + 1] - offsets[i];
        for (int c = 0; c < ORC_NCOLS; c++)
            memset(advice + (uint64_t)c * total_rows + offsets[i], 0, rows * sizeof(uint32_t));
        memset(fixed + offsets[i], 0, rows * sizeof(uint32_t));
        region_t R;
        memset(&R, 0, sizeof R);
        R.adv = advice; R.fixed = fixed; R.stride = total_rows; R.base = offsets[i];
        if ((size_t)i == t_inst) {
            R.tamper_kind = t_kind; R.tamper_row = t_row; R.tamper_delta = t_delta;
        }
        uint64_t out[8];
        synthesize(&R, &in[i], out);
        if (h_out) memcpy(h_out + 8 * i, out, sizeof out);
    }
    (void)nthreads;
    return 0;
}

int orc_fill(const orc_input* in, size_t n, const uint64_t* offsets, uint64_t total_rows,
             uint32_t* advice, uint32_t* fixed, uint64_t* h_out, int nthreads) {
    return fill_impl(in, n, offsets, total_rows, advice, fixed, h_out, nthreads, (size_t)-1, 0, 0, 0);
}

int orc_fill_tampered(const orc_input* in, size_t n, const uint64_t* offsets,
                      uint64_t total_rows, uint32_t* advice, uint32_t* fixed, uint64_t* h_out,
                      size_t inst, int kind, uint32_t row, uint64_t delta) {
    return fill_impl(in, n, offsets, total_rows, advice, fixed, h_out, 1, inst, kind, row, delta);
}

/* ------------------------------------------------------------------ eval (LAYOUT.md §6) */

typedef __int128 i128;

typedef struct {
    const uint32_t* adv;
    const uint32_t* fixed;
    uint64_t total;
    uint64_t row; /* selector row */
} gctx;

static inline i128 cv(const gctx* g, int col, unsigned j) {
    uint64_t r = g->row + j;
    if (r >= g->total) return 0;
    return (i128)g->adv[(uint64_t)col * g->total + r];
}

static int gate_fails(const gctx* g, int sel) {
    const i128 P16 = (i128)1 << 16, P64 = (i128)1 << 64;
    switch (sel) {
    case S_ABCD:
        return (cv(g, A7, 0) - cv(g, A1, 0) - P16 * cv(g, A1, 1)) != 0 ||
               (cv(g, A8, 0) - cv(g, A1, 2) - P16 * cv(g, A1, 3)) != 0;
    case S_DIGEST:
        return (cv(g, A7, 0) - cv(g, A1, 0) - P16 * cv(g, A1, 2)) != 0 ||
               (cv(g, A8, 0) - cv(g, A1, 4) - P16 * cv(g, A1, 6)) != 0;
    case S_EFGH:
        for (unsigned k = 0; k < 4; k++) {
            unsigned k1 = (k + 1) & 3, k2 = (k + 2) & 3;
            if (cv(g, A7, 3 * k) - cv(g, A1, 3 * k1 + 1) - 256 * cv(g, A1, 3 * k2) != 0) return 1;
            if (cv(g, A8, 3 * k) - cv(g, A2, 3 * k1 + 1) - P16 * cv(g, A2, 3 * k2) != 0) return 1;
        }
        return 0;
    case S_IJKL:
        for (unsigned k = 0; k < 4; k++) {
            unsigned k3 = (k + 3) & 3;
            if (cv(g, A7, 2 * k) - cv(g, A6, 2 * k3) - 2 * cv(g, A1, 2 * k) != 0) return 1;
            if (cv(g, A8, 2 * k) - cv(g, A6, 2 * k3) - 4 * cv(g, A2, 2 * k) != 0) return 1;
        }
        return 0;
    case S_A1:
    case S_A2: {
        i128 s = 0;
        for (unsigned k = 0; k < 4; k++)
            s += (cv(g, A3, k) + cv(g, A4, k) + cv(g, A5, k) - cv(g, A1, k)) * ((i128)1 << (16 * k));
        i128 c = cv(g, A9, 0);
        return (s - P64 * c) != 0 || c * (c - 1) * (c - 2) != 0;
    }
    case S_C1:
    case S_C2: {
        i128 s = 0;
        for (unsigned k = 0; k < 4; k++)
            s += (cv(g, A3, k) + cv(g, A4, k) - cv(g, A1, k)) * ((i128)1 << (16 * k));
        i128 c = cv(g, A9, 0);
        return (s - P64 * c) != 0 || c * (c - 1) != 0;
    }
    case S_B1:
        for (unsigned k = 0; k < 4; k++) {
            if (cv(g, A3, 3 * k) + cv(g, A4, 3 * k) - cv(g, A2, 3 * k) -
                    P16 * cv(g, A2, 3 * k + 1) - 2 * cv(g, A2, 3 * k + 2) != 0)
                return 1;
            if (cv(g, A0, 3 * k) != 0 || cv(g, A0, 3 * k + 1) != 0) return 1;
        }
        return 0;
    case S_D1:
    case S_D2:
    case S_XOR:
        for (unsigned k = 0; k < 4; k++)
            if (cv(g, A3, 2 * k) + cv(g, A4, 2 * k) - cv(g, A2, 2 * k) -
                    2 * cv(g, A2, 2 * k + 1) != 0)
                return 1;
        return 0;
    case S_B2:
        for (unsigned k = 0; k < 4; k++) {
            i128 t = cv(g, A0, 2 * k), b = cv(g, A6, 2 * k);
            if (cv(g, A3, 2 * k) + cv(g, A4, 2 * k) - cv(g, A2, 2 * k) - ((i128)1 << 30) * b -
                    2 * cv(g, A2, 2 * k + 1) != 0)
                return 1;
            if (t * (t - 1) != 0 || b * (b - 1) != 0) return 1;
        }
        return 0;
    case S_XOR3:
        for (unsigned k = 0; k < 4; k++)
            if (cv(g, A3, 2 * k) + cv(g, A4, 2 * k) + cv(g, A5, 2 * k) - cv(g, A2, 2 * k) -
                    2 * cv(g, A2, 2 * k + 1) != 0)
                return 1;
        return 0;
    case S_CONST:
        return cv(g, A1, 0) - (i128)(g->fixed[g->row] >> 16) != 0;
    case S_FMASK: {
        i128 f = cv(g, A5, 0);
        if (f * (f - 1) != 0) return 1;
        for (unsigned k = 0; k < 4; k++)
            if (cv(g, A1, k) - 65535 * f != 0) return 1;
        return 0;
    }
    }
    return 0;
}

static inline void note(orc_report* r, uint64_t row, unsigned code) {
    uint64_t key = (row << 8) | code;
    if (key < r->first_failure) r->first_failure = key;
}

int orc_eval(const uint32_t* advice, const uint32_t* fixed, const uint64_t* offsets, size_t n,
             uint64_t total_rows, orc_report* rep, int nthreads) {
    for (size_t i = 0; i < n; i++) {
        uint64_t R = offsets[i + 1] - offsets[i];
        if (R < INIT_ROWS + FINAL_ROWS || (R - INIT_ROWS - FINAL_ROWS) % ROUND_ROWS) return -1;
    }
    if (offsets[n] > total_rows) return -1;
    memset(rep, 0, sizeof *rep);
    rep->first_failure = UINT64_MAX;
    rep->rows_checked = total_rows;
    const uint32_t* A[ORC_NCOLS];
    for (int c = 0; c < ORC_NCOLS; c++) A[c] = advice + (uint64_t)c * total_rows;

#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
#endif
    {
        orc_report loc;
        memset(&loc, 0, sizeof loc);
        loc.first_failure = UINT64_MAX;
        uint32_t* cp = NULL;
        size_t cap = 0;
        uint32_t cp_rounds = UINT32_MAX;
        size_t ncp = 0;
        uint32_t* fx = NULL; /* keygen fixed column of cp_rounds */
        /* Rows and gates: chunk the global rows (independent of instance boundaries). */
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4096)
#endif
        for (long long rr = 0; rr < (long long)total_rows; rr++) {
            uint64_t row = (uint64_t)rr;
            uint32_t tag = A[A0][row], dense = A[A1][row], spread = A[A2][row];
            if (!(dense < 65536u && tag == get_tag(dense) && spread == spread16(dense))) {
                loc.lookup_failures++;
                note(&loc, row, ORC_CODE_LOOKUP);
            }
            uint32_t sel = fixed[row] & 0xffffu;
            if (sel) {
                gctx g = {advice, fixed, total_rows, row};
                for (int s = 0; s < ORC_NGATES; s++)
                    if (((sel >> s) & 1u) && gate_fails(&g, s)) {
                        loc.gate_failures[s]++;
                        note(&loc, row, (unsigned)s);
                    }
            }
        }
        /* Copy constraints: per instance, from the structure-mode synthesis. */
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
        for (long long i = 0; i < (long long)n; i++) {
            uint32_t rounds =
                (uint32_t)((offsets[i + 1] - offsets[i] - INIT_ROWS - FINAL_ROWS) / ROUND_ROWS);
            if (rounds != cp_rounds) {
                size_t need = orc_copies(rounds, NULL, 0);
                if (need > cap) {
                    free(cp);
                    cap = need;
                    cp = (uint32_t*)malloc(4 * cap * sizeof(uint32_t));
                }
                ncp = orc_copies(rounds, cp, cap);
                free(fx);
                fx = (uint32_t*)malloc(orc_rows(rounds) * sizeof(uint32_t));
                fixed_structure(rounds, fx);
                cp_rounds = rounds;
            }
            uint64_t base = offsets[i];
            /* the fixed column against the keygen structure (halo2 fixes it at keygen) */
            for (uint64_t r = 0; r < orc_rows(rounds); r++)
                if (fixed[base + r] != fx[r]) {
                    loc.fixed_failures++;
                    note(&loc, base + r, ORC_CODE_FIXED);
                }
            for (size_t q = 0; q < ncp; q++) {
                const uint32_t* e = cp + 4 * q;
                if (A[e[1]][base + e[0]] != A[e[3]][base + e[2]]) {
                    loc.copy_failures++;
                    note(&loc, base + e[0], ORC_CODE_COPY);
                }
            }
        }
        free(cp);
        free(fx);
        /* rows past the last instance carry no selector or constant */
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (long long rr = (long long)offsets[n]; rr < (long long)total_rows; rr++)
            if (fixed[rr]) {
                loc.fixed_failures++;
                note(&loc, (uint64_t)rr, ORC_CODE_FIXED);
            }
#ifdef _OPENMP
#pragma omp critical
#endif
        {
            for (int s = 0; s < ORC_NGATES; s++) rep->gate_failures[s] += loc.gate_failures[s];
            rep->lookup_failures += loc.lookup_failures;
            rep->copy_failures += loc.copy_failures;
            rep->fixed_failures += loc.fixed_failures;
            if (loc.first_failure < rep->first_failure) rep->first_failure = loc.first_failure;
        }
    }
    (void)nthreads;
    return 0;
}

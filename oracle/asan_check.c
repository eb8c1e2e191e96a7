/* Host sanitizer run of the CPU oracle (test infrastructure; VERDICT r1 aux item "host ASan
 * build of the oracle"): `make -C oracle asan` builds this driver and b2f_oracle.c with
 * AddressSanitizer + UndefinedBehaviorSanitizer into _asan/asan_check; tests/test_oracle.py runs
 * it. It drives every entry point of b2f_oracle.h over mixed rounds (0, 1, 4, 12, 13), a padded
 * tail, single-cell corruptions of advice and fixed cells, a tampered fill, the Fp export in both
 * forms and both fields' Montgomery pins. Exit 0 = every call returned and every expected verdict
 * held; any sanitizer finding aborts with its report. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "b2f_oracle.h"

static uint64_t sm_state = 0x9E3779B97F4A7C15ull;
static uint64_t splitmix(void) {
  uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

#define CHECK(c)                                               \
  do {                                                         \
    if (!(c)) {                                                \
      fprintf(stderr, "asan_check: %s failed (line %d)\n", #c, __LINE__); \
      return 1;                                                \
    }                                                          \
  } while (0)

int main(void) {
  const uint32_t rounds_of[] = {0, 1, 4, 12, 13, 1, 12};
  const size_t n = sizeof rounds_of / sizeof rounds_of[0];
  orc_input in[sizeof rounds_of / sizeof rounds_of[0]];
  for (size_t i = 0; i < n; i++) {
    for (int k = 0; k < 8; k++) in[i].h[k] = splitmix();
    for (int k = 0; k < 16; k++) in[i].m[k] = splitmix();
    in[i].t[0] = splitmix();
    in[i].t[1] = splitmix();
    in[i].rounds = rounds_of[i];
    in[i].f = (uint32_t)(splitmix() & 1u);
  }
  uint64_t off[sizeof rounds_of / sizeof rounds_of[0] + 1];
  orc_offsets(in, n, off);
  const uint64_t total = off[n] + 64;  /* a padded tail of zero rows */
  uint32_t* adv = calloc(10 * total, 4);
  uint32_t* fixed = calloc(total, 4);
  uint32_t* fx2 = calloc(total, 4);
  uint64_t* hout = calloc(8 * n, 8);
  CHECK(adv && fixed && fx2 && hout);
  CHECK(orc_fill(in, n, off, total, adv, fixed, hout, 2) == 0);
  for (size_t i = 0; i < n; i++) {  /* h' equals the compression function */
    uint64_t ref[8];
    orc_compress(in[i].rounds, in[i].h, in[i].m, in[i].t, in[i].f, ref);
    CHECK(memcmp(ref, hout + 8 * i, sizeof ref) == 0);
  }
  CHECK(orc_fixed(off, n, total, fx2) == 0);
  CHECK(memcmp(fixed, fx2, 4 * total) == 0);
  orc_report rep;
  CHECK(orc_eval(adv, fixed, off, n, total, &rep, 2) == 0);
  CHECK(rep.first_failure == UINT64_MAX && rep.copy_failures == 0 && rep.lookup_failures == 0);
  int flagged = 0;
  for (int t = 0; t < 200; t++) {  /* single-cell corruptions */
    const uint64_t row = splitmix() % off[n];
    const int col = (int)(splitmix() % 11);
    uint32_t* cell = col < 10 ? adv + (uint64_t)col * total + row : fixed + row;
    const uint32_t mask = 1u << (splitmix() % 20);
    *cell ^= mask;
    CHECK(orc_eval(adv, fixed, off, n, total, &rep, 2) == 0);
    flagged += rep.first_failure != UINT64_MAX;
    *cell ^= mask;
  }
  CHECK(flagged > 200 / 3);  /* unused (zero) cells are unconstrained */
  /* a trace consistent with an altered fixed column: only the structure check sees it */
  CHECK(orc_fill_tampered(in, n, off, total, adv, fixed, hout, 3, 1, 164 + 52, 1) == 0);
  CHECK(orc_eval(adv, fixed, off, n, total, &rep, 2) == 0);
  CHECK(rep.fixed_failures > 0);
  size_t cap = 1u << 16;
  uint32_t* cp = malloc(4 * 4 * cap);
  CHECK(cp);
  for (uint32_t r = 0; r < 14; r++) CHECK(orc_copies(r, cp, cap) > 0);
  uint64_t* fp = malloc(8 * 4 * 10 * 256);
  CHECK(fp);
  orc_export_fp(adv, total, off[2], 256, 0, fp, 256);
  orc_export_fp(adv, total, off[2], 256, 1, fp, 256);
  uint64_t mont[4];
  orc_fp_mont(0, 12345u, mont);
  orc_fp_mont(1, 12345u, mont);
  CHECK(orc_max_threads() >= 1);
  free(fp);
  free(cp);
  free(hout);
  free(fx2);
  free(fixed);
  free(adv);
  printf("asan_check ok: %zu instances, %llu rows, %d of 200 corruptions flagged\n", n,
         (unsigned long long)off[n], flagged);
  return 0;
}

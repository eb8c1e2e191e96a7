#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "b2f_safegcd.h"
// Host check of b2f_safegcd.h (tests/test_safegcd.py builds it with g++): reads lines
// "p_hex x_hex", prints x^-1 mod p as hex (0 for x = 0), or "nonconverged" when inverse()
// reports that the divsteps did not end at g = 0 (the test asserts it never does for x < p).
static void parse(const char* s, uint32_t (&w)[8]) {
  memset(w, 0, sizeof w);
  int n = strlen(s);
  for (int i = 0; i < n; i++) {
    char c = s[n - 1 - i];
    int d = c <= '9' ? c - '0' : (c | 32) - 'a' + 10;
    w[i / 8] |= (uint32_t)d << (4 * (i % 8));
  }
}
int main() {
  char a[80], b[80];
  while (scanf("%79s %79s", a, b) == 2) {
    uint32_t p[8], x[8], o[8];
    parse(a, p); parse(b, x);
    if (!b2f::sgcd::inverse(x, p, o)) {
      printf("nonconverged\n");
      continue;
    }
    for (int i = 7; i >= 0; i--) printf("%08x", o[i]);
    printf("\n");
  }
}

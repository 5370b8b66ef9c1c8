/* TEST INFRASTRUCTURE (tests/test_crmath_host.py): the exhaustive part of the
 * one-step Markstein division proof (sdf3d_amd/csrc/cr_math.h div_refined).
 *
 * The proof covers every divisor whose mantissa field is <= 2^23 - 8 by a
 * margin argument; this program checks the rest -- with a margin, the N
 * largest mantissa fields (default 64) -- against every numerator mantissa in
 * two binades (the quotient's binade relative to the divisor's: the result
 * scales exactly by powers of two away from underflow and overflow):
 *
 *   y = RN(1/b), q = RN(a y), r = fma(b, q, -a), q1 = fma(-r, y, q)
 *   must equal a / b (IEEE, round to nearest even)
 *
 * Also a random sample over general normal a, b.  fmaf is the C library's
 * correctly rounded fused multiply-add.  Prints one JSON line; exit 1 on a
 * mismatch.
 *
 *     gcc -O2 -o markstein_window markstein_window.c -lm && ./markstein_window [N] [SAMPLES]
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float u2f(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static uint32_t f2u(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
static int one_step_ok(float a, float b, float y) {
  const float q = a * y;
  const float r = fmaf(b, q, -a);
  const float q1 = fmaf(-r, y, q);
  volatile float ex = a / b;
  return f2u(q1) == f2u(ex);
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 64u;
  const long samples = argc > 2 ? atol(argv[2]) : 20000000L;
  long checked = 0, bad = 0;
  for (uint32_t mf = (1u << 23) - n; mf < (1u << 23); mf++) {
    const float b = u2f((127u << 23) | mf);
    volatile float yv = 1.0f / b;
    const float y = yv;
    for (uint32_t e = 126; e <= 127; e++)
      for (uint32_t m = 0; m < (1u << 23); m++) {
        const float a = u2f((e << 23) | m);
        checked++;
        if (!one_step_ok(a, b, y)) {
          if (bad < 4) fprintf(stderr, "window: a=%a b=%a\n", a, b);
          bad++;
        }
      }
  }
  uint64_t s = 0x9E3779B97F4A7C15ull;
  long sbad = 0;
  for (long i = 0; i < samples; i++) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const float b = u2f((uint32_t)((97 + (s & 63)) << 23) | (uint32_t)((s >> 8) & 0x7FFFFF));
    const float a = u2f((uint32_t)((97 + ((s >> 32) & 63)) << 23) | (uint32_t)((s >> 40) & 0x7FFFFF));
    volatile float yv = 1.0f / b;
    if (!one_step_ok(a, b, yv)) {
      if (sbad < 4) fprintf(stderr, "sample: a=%a b=%a\n", a, b);
      sbad++;
    }
  }
  printf("{\"window_mantissas\": %u, \"window_checked\": %ld, \"window_bad\": %ld, "
         "\"samples\": %ld, \"sample_bad\": %ld}\n", n, checked, bad, samples, sbad);
  return bad || sbad ? 1 : 0;
}

/* TEST INFRASTRUCTURE (tests/test_crmath_host.py): random check of the exact
 * shadow march's first skip bound (sdf3d_amd/csrc/render_kernel.inc
 * SDF_EXACT_SHSKIP1).  Wherever the kernel's test
 *     hn <= RN(1.5 h_prev)  and  RN(k66 hn - RN(RN(s t)(1 + 2^-20))) > 2^-100
 * holds (k66 = RN(0.66 k)), the oracle's step term RN(k dest / den) must be
 * >= s, so that its min keeps s: the oracle's operation sequence below
 * (voxel_fragment.frag's improved soft shadow, fp32, no contraction).
 * Prints one JSON line; exit 1 on a violation.
 *
 *     gcc -O2 -ffp-contract=off -o shadow_skip_bound shadow_skip_bound.c -lm && ./shadow_skip_bound [N]
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint64_t st = 0x2545F4914F6CDD1Dull;
static double rnd(void) {
  st ^= st << 13; st ^= st >> 7; st ^= st << 17;
  return (double)(st >> 11) * (1.0 / 9007199254740992.0);
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 20000000L;
  long pass = 0, bad = 0;
  for (long i = 0; i < n; i++) {
    /* k in [0, 20), h_prev log-uniform over [2^-12, 2^3), hn / h_prev in
     * [0, 1.6), t in [0, 5), s in [0, 1]; every 4th sample puts s t next to
     * the bound's edge */
    const float k = (float)(rnd() * 20.0);
    const float hp = (float)exp2(rnd() * 15.0 - 12.0);
    const float hn = hp * (float)(rnd() * 1.6);
    float t = (float)(rnd() * 5.0);
    float s = (float)rnd();
    if ((i & 3) == 0 && s > 0.0f) t = (float)(0.66 * k * hn / s * (1.0 - rnd() * 1e-5));
    const float k66 = k * 0.66f;
    const float w0 = s * t;
    const float w = fmaf(w0, 0x1p-20f, w0);
    const float lhs = fmaf(k66, hn, -w);
    if (!(hn <= 1.5f * hp && lhs > 0x1p-100f)) continue;
    pass++;
    const float hh = hn * hn;
    const float inter = hh / (2.0f * hp);
    const float dest = sqrtf(hh - inter * inter);
    const float num = k * dest;
    const float d0 = t - inter;
    const float den = 0.0f < d0 ? d0 : 0.0f;          /* GLSL max(0, .) */
    const float term = num / den;
    const float r = term < s ? term : s;               /* GLSL min(s, term) */
    if (r != s) {
      if (bad < 4) fprintf(stderr, "k=%a hp=%a hn=%a t=%a s=%a term=%a\n", k, hp, hn, t, s, term);
      bad++;
    }
  }
  printf("{\"samples\": %ld, \"bound_held\": %ld, \"violations\": %ld}\n", n, pass, bad);
  return bad ? 1 : 0;
}

// cr_math.h -- correctly rounded fp32 building blocks for the EXACT-precision
// kernel (render_exact.hip), cheaper on gfx950 than the compiler's generic
// sequences yet bit-identical to what the oracle computes (IEEE sqrtf, a / b,
// and log evaluated in fp64 and rounded once: oracle/sdf_oracle.c cr_logf).
//
//   cr_sqrt(x)           == sqrtf(x) for every x (every x but +INF with
//                           SDF_CRM_SQRT_GUARD 1).  Fast path on [2^-100,
//                           2^100) (on [2^-100, FLT_MAX] with guard 1): v_rsq,
//                           then one Newton/Markstein correction (rsq, 2 mul,
//                           2 fma) instead of the generic v_sqrt + denormal
//                           scaling + 2-candidate residual test + class
//                           fix-up (17 instructions).
//   div_prepared(a,b,yb) == a / b, given yb = RN(1/b) prepared on the host,
//                           by one Markstein step (proof at div_refined:
//                           fma(r, yb, q) = RN(a/b)) wherever a/b, q and r
//                           neither overflow nor underflow (3 instructions
//                           instead of 11).  div_scaled applies it to the
//                           smooth-min's h = n / k (render_kernel.inc smin)
//                           after an exact power-of-two scaling that puts
//                           every positive k in its domain.
//   cr_log(x)            == (float)log((double)x) for every x.  Fast path:
//                           m in [sqrt(1/2), sqrt(2)), f = (m-1)/(m+1) with a
//                           refined v_rcp_f64, 2 f (1 + s/3 + ... + s^8/17)
//                           with s = f^2, plus e ln2, in fp64 (error below
//                           2^-49 relative); when that value lies too close to
//                           a float rounding boundary to round it safely, or x
//                           is not a positive normal float, the lane takes the
//                           fp64 library log the oracle's reading is.
//
// Every fast path is taken by a lane only where it is proven or checked
// bit-identical; the fall-backs run in a branch the wave skips when no lane
// needs it.  tests/crmath/crmath_check.hip runs cr_sqrt and cr_log
// EXHAUSTIVELY on the GPU (all 2^32 inputs) and rcp_fast on every float of its
// domain, against the generic sequences (tests/test_gpu_crmath.py).
// div_scaled's domain, the (k, n) pairs of the smooth-min, has ~2^64 points:
// it is SAMPLED (2^32 pairs, k log-uniform over every positive float, plus
// denormal k, k near FLT_MAX and n whose scaled value underflows); its
// bit-identity rests on the one-step proof at div_refined, not on the sample.
#pragma once

#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif

namespace sdf {
namespace crm {

// a wave-uniform "does any lane need the slow path" (no divergent branch)
__device__ __forceinline__ bool any_lane(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }
// Placed in a slow-path block: an instruction with side effects keeps LLVM
// from if-converting the block into selects, i.e. from computing the slow
// path on every lane of every wave.
#define SDF_CRM_COLD() asm volatile("" ::: "memory")

// x in [2^-100, 2^100) (positive, normal, far from both ends of the range):
// the fast path's x * y, s * s and residual neither underflow nor overflow
// (the domain rcp_fast is checked on, tests/crmath/crmath_check.hip)
__device__ __forceinline__ bool sqrt_fast_ok(float x) {
  return (__float_as_uint(x) - 0x0D800000u) < (0x71800000u - 0x0D800000u);
}

// The guard cr_sqrt takes the fast path behind (SDF_CRM_SQRT_GUARD):
//   0  the integer range test above (2 VALU): cr_sqrt(x) == sqrtf(x) for
//      EVERY x.
//   1  ONE float compare, x >= 2^-100 (catches 0, denormals, tiny x,
//      negatives and NaN): the fast path is exact on all of [2^-100,
//      FLT_MAX] (tests/crmath "sqrtwide", every positive normal), so
//      cr_sqrt(x) == sqrtf(x) for every x but +INF (where it gives NaN).
//      For callers whose arguments are finite by their domain:
//      render_kernel.inc sets it for the CSG units, where sdf_validate's
//      working range bounds every squared length far below FLT_MAX; the
//      Mandelbulb unit keeps 0 (its orbit may overflow).
// (A guard on the fast path's own product x RN(1/sqrt x) >= 2^-50 -- also
// one compare -- fails: v_rsq flushes denormal inputs to +-INF, and x * INF
// passes it.  tests/crmath "sqrt" caught that.)
#ifndef SDF_CRM_SQRT_GUARD
#define SDF_CRM_SQRT_GUARD 0
#endif

__device__ __forceinline__ float sqrt_fast(float x) {
  const float y = __builtin_amdgcn_rsqf(x);   // 1/sqrt(x), ~1 ulp
  const float s = x * y;                      // sqrt(x), within ~2 ulp
  const float h = 0.5f * y;                   // 1/(2 sqrt(x)), exact halving
  const float r = __builtin_fmaf(-s, s, x);   // x - s^2, exact
  return __builtin_fmaf(h, r, s);
}
template <int G>
__device__ __forceinline__ bool sqrt_guard_g(float x) {
  if constexpr (G == 1) return x >= 0x1p-100f;
  else return sqrt_fast_ok(x);
}
__device__ __forceinline__ bool sqrt_guard(float x) { return sqrt_guard_g<SDF_CRM_SQRT_GUARD>(x); }

template <int G>
__device__ __forceinline__ float cr_sqrt_g(float x) {
  float s = sqrt_fast(x);
  const bool ok = sqrt_guard_g<G>(x);
  if (any_lane(!ok)) {
    SDF_CRM_COLD();
    s = ok ? s : __builtin_sqrtf(x);
  }
  return s;
}
__device__ __forceinline__ float cr_sqrt(float x) { return cr_sqrt_g<SDF_CRM_SQRT_GUARD>(x); }

// N square roots behind ONE guard (independent chains stay in one basic
// block, render_kernel.inc mandelbulb_n): each s[i] == cr_sqrt(x[i])
template <int N>
__device__ __forceinline__ void cr_sqrt_n(const float (&x)[N], float (&s)[N]) {
  bool ok = true;
#pragma unroll
  for (int i = 0; i < N; i++) {
    s[i] = sqrt_fast(x[i]);
    ok = ok & sqrt_guard(x[i]);
  }
  if (any_lane(!ok)) {
    SDF_CRM_COLD();
#pragma unroll
    for (int i = 0; i < N; i++) s[i] = sqrt_guard(x[i]) ? s[i] : __builtin_sqrtf(x[i]);
  }
}

// 1/x for x in [2^-100, 2^100) (the caller's domain; no guard): v_rcp and
// one Newton step with an exact fma residual, checked equal to IEEE 1.0f / x
// on every float of that range
__device__ __forceinline__ float rcp_fast(float x) {
  const float y = __builtin_amdgcn_rcpf(x);
  const float e = __builtin_fmaf(-x, y, 1.0f);
  return __builtin_fmaf(e, y, y);
}

// a / b = RN(a/b) from yb = RN(1/b) (one Markstein step, proven below at
// div_refined): valid where no intermediate underflows or overflows -- the
// caller's domain argument.
__device__ __forceinline__ float div_prepared(float a, float b, float yb) {
  const float q = a * yb;
  const float r = __builtin_fmaf(-b, q, a);
  return __builtin_fmaf(r, yb, q);
}

// a / l from y = RN(1/l) (the host's, or rcp_fast) by ONE Markstein step:
// q0 = RN(a y), r = RN(l q0 - a), q1 = RN(q0 - r y) == RN(a/l) wherever
// nothing underflows or overflows.  Proof (round 6; rounds 1-5 took a second
// step because q0 need not be faithful):
//   Let Q = a/l = mu 2^j (mu in [1,2)), u = ulp(Q), l = ml 2^e (ml in [1,2);
//   a power-of-two l makes everything exact).  |y - 1/l| <= ulp(1/l)/2 gives
//   |a y - Q| <= E u with E = mu (ml/2) / 2 < ml/2.
//   * q0 faithful: Markstein's theorem (y within 1/2 ulp of 1/l, q0 within
//     1 ulp of Q; r is then exact) gives q1 = RN(Q).
//   * q0 not faithful: rounding past the float adjacent to Q needs |a y - Q|
//     > u/2 + (distance from Q to that float), so Q lies within (E - 1/2) u
//     of a float and at least (1 - E) u from every rounding midpoint.  With
//     r = (l q0 - a)(1 + rho), |rho| <= 2^-24, and l y = 1 + delta, |delta| <
//     2^-24, q0 - r y = Q + (Q - q0)(1 - (1 + delta)(1 + rho)) = Q + eps,
//     |Q - q0| < 2u, |eps| < 2^-22 u (1 + 2^-24).  So q1 = RN(Q + eps) = RN(Q)
//     unless (1 - E) u <= |eps|, i.e. E > 1 - 2^-22 (1 + 2^-24): impossible
//     for ml <= 2 - 2^-20 (E < ml/2 <= 1 - 2^-21), i.e. for every divisor
//     mantissa field <= 2^23 - 8.
//   * the 8 largest mantissa fields (with a margin: the 64 largest) against
//     every numerator mantissa, two binades: checked exhaustively
//     (tests/crmath/markstein_window.c, tests/test_crmath_host.py) -- none
//     differs from a / l.
// The residual's sign convention keeps a signed zero numerator's sign (q0 =
// +-0, r = +0, q1 = -0 + q0 = q0).  Domain: l in [2^-30, 2^30), every a zero
// or |a| >= 2^-60 (quotients and residuals stay normal); other lanes of the
// wave take the IEEE division.
// SDF_CRM_DIV_STEPS 2: rounds 1-5's second step (A/B only; same results)
#ifndef SDF_CRM_DIV_STEPS
#define SDF_CRM_DIV_STEPS 1
#endif
__device__ __forceinline__ float div_refined(float a, float l, float y) {
  float q = a * y;
#if SDF_CRM_DIV_STEPS == 2
  q = __builtin_fmaf(-__builtin_fmaf(l, q, -a), y, q);
#endif
  const float r = __builtin_fmaf(l, q, -a);
  return __builtin_fmaf(-r, y, q);
}
// the divisor's magnitude in [2^-30, 2^30) (either sign)
__device__ __forceinline__ bool divisor_ok(float l) {
  return ((__float_as_uint(l) << 1) - (0x30800000u << 1)) < ((0x4E800000u - 0x30800000u) << 1);
}
// every numerator zero or of magnitude >= 2^-60 (|a| bits shifted out of the
// sign; a zero wraps to the top when 1 is subtracted).  The callers' own
// domains bound |a| above: |a| <= l (normalize), the working range (the
// Mandelbulb's p - c).
__device__ __forceinline__ bool numerators_ok(float a0, float a1, float a2) {
  const uint32_t m = min(min((__float_as_uint(a0) << 1) - 1u, (__float_as_uint(a1) << 1) - 1u),
                         (__float_as_uint(a2) << 1) - 1u);
  return m >= (0x21800000u << 1) - 1u;
}
__device__ __forceinline__ bool div3_ok(float a0, float a1, float a2, float l) {
  // `&`, not `&&`: no short-circuit branch (which made the compiler carry the
  // mask across blocks and rebuild it with v_cndmask + v_cmp)
  const bool d = divisor_ok(l), n = numerators_ok(a0, a1, a2);
  return d & n;
}
// (a0, a1, a2) / l from the host's y = RN(1/l), l's range checked by the
// caller (wave-uniform): the Mandelbulb's (p - c) / scale
// SDF_CRM_DIV3_MIN3 1 (round 6): the wave's fast test is ONE v_min3_f32 of
// the numerators' magnitudes against 2^-60 (2 VALU instead of 5); a wave
// where it fails (a zero numerator: the Mandelbulb's p - c is rarely exactly
// zero) takes the exact numerators_ok test in the cold block.  Same
// quotients: a lane passing the min3 test passes numerators_ok.
#ifndef SDF_CRM_DIV3_MIN3
#define SDF_CRM_DIV3_MIN3 1
#endif
__device__ __forceinline__ void div3_prepared(float& a0, float& a1, float& a2, float l, float y) {
#if SDF_CRM_DIV3_MIN3
  const bool fast = __builtin_fminf(__builtin_fminf(__builtin_fabsf(a0), __builtin_fabsf(a1)),
                                    __builtin_fabsf(a2)) >= 0x1p-60f;
#else
  const bool fast = numerators_ok(a0, a1, a2);
#endif
  float q0 = div_refined(a0, l, y), q1 = div_refined(a1, l, y), q2 = div_refined(a2, l, y);
  if (any_lane(!fast)) {
    SDF_CRM_COLD();
    if (!numerators_ok(a0, a1, a2)) {
      q0 = a0 / l;
      q1 = a1 / l;
      q2 = a2 / l;
    }
  }
  a0 = q0;
  a1 = q1;
  a2 = q2;
}
// a / b for one division (the DE's, the shadow march's): computed as
// (sign(b) a) / |b| -- the same correctly rounded quotient (round to nearest
// is symmetric), and with a positive divisor the two steps keep a zero
// numerator's sign (with a negative one +0 / b would come out +0, not -0) --
// y = RN(1/|b|) by rcp_fast, one Markstein step; |b| in [2^-30, 2^30) and a
// zero or |a| in [2^-60, 2^60) (guarded; the IEEE division elsewhere)
__device__ __forceinline__ float div_one(float a, float b) {
  const uint32_t ua = (__float_as_uint(a) << 1) - 1u;
  const bool ok = divisor_ok(b) && ua >= (0x21800000u << 1) - 1u &&
                  (ua < (0x5D800000u << 1) - 1u || ua == 0xFFFFFFFFu);
  const float mb = __builtin_fabsf(b);
  float q = div_refined(__builtin_copysignf(1.0f, b) * a, mb, rcp_fast(mb));
  if (any_lane(!ok)) {
    SDF_CRM_COLD();
    if (!ok) q = a / b;
  }
  return q;
}
__device__ __forceinline__ void div3(float& a0, float& a1, float& a2, float l) {
  const float y = rcp_fast(l);
  const bool ok = div3_ok(a0, a1, a2, l);
  float q0 = div_refined(a0, l, y), q1 = div_refined(a1, l, y), q2 = div_refined(a2, l, y);
  if (any_lane(!ok)) {
    SDF_CRM_COLD();
    if (!ok) {
      q0 = a0 / l;
      q1 = a1 / l;
      q2 = a2 / l;
    }
  }
  a0 = q0;
  a1 = q1;
  a2 = q2;
}

// n / k for the smooth-min (n in [0, k], any positive finite k), from the
// host-prepared sc = 2^s with k sc in [2^-22, 1) (s <= 127) and ys =
// RN(1/(k sc)): n/k = (n sc)/(k sc) exactly, k sc is exact, n sc is exact
// unless it underflows (then h < 2^-104), and Markstein's conditions hold
// for n sc >= 2^-100.  Below that h < 2^-77 on both paths, so h*h -- all the
// smooth-min uses -- is +0 on both: the smooth-min's result is bit-identical.
__device__ __forceinline__ float div_scaled(float n, float k, float sc, float ys) {
  return div_prepared(n * sc, k * sc, ys);
}

// The smooth-min's whole h = max(k - |e|, 0) / k (e = RN(a - b)) from the
// same preparation, ksc = k sc (exact), in 4 instructions instead of 6
// (round 6, tools/block_counts.py: the smooth-min was 12 VALU, ~400 per
// wave on C4):
//   n' = clamp(RN(ksc - |e| sc), 0, 1): ONE FMA whose product |e| sc is exact,
//        with the clamp bit for the max (n' <= ksc < 1, so the clamp's upper
//        end never binds; no operand is NaN in the working range);
//   h  = div_prepared(n', ksc, ys).
// Against div_scaled(max(RN(k - |e|), 0), k, sc, ys): RN((k - |e|) sc) =
// RN(k - |e|) sc exactly whenever both lie in the normal range (scaling by a
// power of two commutes with rounding there); a difference k - |e| below
// 2^-126 is exact already (a difference of floats that small is
// representable), so both round the same exact product; otherwise the scaled
// value is below 2^-126 < 2^-100 on both paths, where h*h is +0 on both (see
// div_scaled).  A non-positive k - |e| gives +0 on both (an exact zero sum is
// +0 in round-to-nearest).  Checked on the GPU (tests/crmath "sminh":
// sampled k over every positive float, |e| around k, tiny, huge).
__device__ __forceinline__ float smin_h(float e, float sc, float ksc, float ys) {
  const float n =
      __builtin_amdgcn_fmed3f(__builtin_fmaf(-__builtin_fabsf(e), sc, ksc), 0.0f, 1.0f);
  return div_prepared(n, ksc, ys);
}

// ---- natural log ----------------------------------------------------------
// log(2) as a double (the rounding error, 2^-54 relative, times |e| <= 126
// stays far below the fast path's error bound)
#define SDF_CRM_LN2 0.693147180559945309417232121458
// relative error bound of log_fast's double result.  Round 6
// (SDF_CRM_LOG_SHORT 1): the series to s^7/15 and ONE Newton step for the
// reciprocal -- truncation s^8/17 <= 2^-44.8 relative at |f| <= 0.1716, the
// reciprocal 2^-46 (v_rcp_f64's 2^-23, squared), ~17 fp64 roundings each
// <= 2^-52: a generous 2^-42 (a lane whose value lies that close to a float
// rounding boundary, ~2^-17 of them, takes the library log; the exhaustive
// check of all 2^32 inputs is the proof that the bound holds); three fp64 operations fewer per log
// (tools/block_counts.py: cr_log was 9 % of C5 exact's VALU issue).  0: the
// round-5 evaluation (s^8/17, two Newton steps, 2^-47)
#ifndef SDF_CRM_LOG_SHORT
#define SDF_CRM_LOG_SHORT 1
#endif
#if SDF_CRM_LOG_SHORT
#define SDF_CRM_LOG_EPS 2.2737367544323206e-13
#else
#define SDF_CRM_LOG_EPS 7.105427357601002e-15
#endif

// p s + c as a three-address v_fma_f64 with the coefficient c in an SGPR
// pair (SDF_CRM_FMA64 1).  With the builtin the compiler keeps the Horner
// coefficients in VGPR pairs and picks the two-address v_fmac_f64, so every
// step first copies its coefficient (v_mov_b64): 6 extra VALU per log and 14
// VGPRs held.  Same operation, same rounding; C5 exact 2.0-2.5 % faster
// (72 -> 68 VGPRs, profiles/r05_ab_log_fma64_C5.json).
#ifndef SDF_CRM_FMA64
#define SDF_CRM_FMA64 1
#endif
__device__ __forceinline__ double fma64(double p, double s, double c) {
#if SDF_CRM_FMA64
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(p), "v"(s), "s"(c));
  return r;
#else
  return __builtin_fma(p, s, c);
#endif
}

// The library fp64 log (the oracle's reading), out of line: only the rare
// lanes near a rounding boundary call it, and its constants stay out of the
// callers' loops (shade.h library_pow)
#if !defined(SDF_CRM_LOG_CALL) || SDF_CRM_LOG_CALL
inline __device__ __attribute__((noinline)) float library_log(float x) {
  return (float)log((double)x);
}
#else
__device__ __forceinline__ float library_log(float x) { return (float)log((double)x); }
#endif

__device__ __forceinline__ double log_fast(float x) {
  // x = 2^e m, m in [sqrt(1/2), sqrt(2))
  float mf = __builtin_amdgcn_frexp_mantf(x);            // [0.5, 1)
  int e = __builtin_amdgcn_frexp_expf(x);
  if (mf < 0.70710678f) {
    mf = mf * 2.0f;                                      // exact
    e = e - 1;
  }
  const double m = (double)mf;
  const double d = m + 1.0;                              // exact
  double y = __builtin_amdgcn_rcp(d);                    // ~2^-23 relative
  y = __builtin_fma(__builtin_fma(-d, y, 1.0), y, y);    // ~2^-46
#if !SDF_CRM_LOG_SHORT
  y = __builtin_fma(__builtin_fma(-d, y, 1.0), y, y);    // ~2^-52
#endif
  const double f = (m - 1.0) * y;                        // m - 1 exact
  const double s = f * f;
#if SDF_CRM_LOG_SHORT
  double p = 1.0 / 15.0;
#else
  double p = 1.0 / 17.0;
  p = fma64(p, s, 1.0 / 15.0);
#endif
  p = fma64(p, s, 1.0 / 13.0);
  p = fma64(p, s, 1.0 / 11.0);
  p = fma64(p, s, 1.0 / 9.0);
  p = fma64(p, s, 1.0 / 7.0);
  p = fma64(p, s, 1.0 / 5.0);
  p = fma64(p, s, 1.0 / 3.0);
  const double lm = 2.0 * f + (2.0 * f) * (s * p);      // 2 atanh(f) = log(m)
  return __builtin_fma((double)e, SDF_CRM_LN2, lm);
}

// Rounding v to float is safe when v's error interval [v - tol, v + tol],
// tol = SDF_CRM_LOG_EPS |v|, holds no fp32 rounding midpoint (x a positive
// normal float).  SDF_CRM_LOG_BITCHECK 1 (round 6) tests that on v's bits:
// an fp32 midpoint is a double whose low 29 mantissa bits are 2^28, and tol
// is below 2^11 of v's ulps (2^-42 |v| with |v| < 2 2^ev, ulp 2^(ev-52)), so
// v is safe when its low 29 bits differ from 2^28 by more than 2^11 -- two
// integer VALU on the low dword instead of an fp64 multiply, two fp64 adds
// and two conversions (at a power of two the interval may reach the next
// binade, whose midpoints lie 2^-25 relative away: no midpoint either).  The
// exhaustive GPU check of all 2^32 inputs (tests/crmath "log") covers both.
#ifndef SDF_CRM_LOG_BITCHECK
#define SDF_CRM_LOG_BITCHECK 1
#endif
__device__ __forceinline__ bool log_round_ok(float x, double v, float r) {
  const bool normal = (__float_as_uint(x) - 0x00800000u) < (0x7F800000u - 0x00800000u);
#if SDF_CRM_LOG_BITCHECK
  static_assert(SDF_CRM_LOG_EPS <= 0x1p-42, "tol must stay below 2^11 ulps of v");
  (void)r;
  const uint32_t lo = (uint32_t)__builtin_bit_cast(unsigned long long, v);
  return normal & (((lo & 0x1FFFFFFFu) - (0x10000000u - 0x800u)) >= 0x1000u);
#else
  const double tol = SDF_CRM_LOG_EPS * __builtin_fabs(v);
  return normal & ((float)(v - tol) == r) & ((float)(v + tol) == r);
#endif
}

__device__ __forceinline__ float cr_log(float x) {
  const double v = log_fast(x);
  const float r = (float)v;
  const bool ok = log_round_ok(x, v, r);
  float out = r;
  if (any_lane(!ok)) {
    SDF_CRM_COLD();
    out = ok ? r : library_log(x);
  }
  return out;
}

// N logs behind ONE guard (as cr_sqrt_n): each out[i] == cr_log(x[i])
template <int N>
__device__ __forceinline__ void cr_log_n(const float (&x)[N], float (&out)[N]) {
  bool ok = true;
#pragma unroll
  for (int i = 0; i < N; i++) {
    const double v = log_fast(x[i]);
    out[i] = (float)v;
    ok = ok & log_round_ok(x[i], v, out[i]);
  }
  if (any_lane(!ok)) {
    SDF_CRM_COLD();
#pragma unroll
    for (int i = 0; i < N; i++) {
      const double v = log_fast(x[i]);
      if (!log_round_ok(x[i], v, out[i])) out[i] = library_log(x[i]);
    }
  }
}

}  // namespace crm
}  // namespace sdf

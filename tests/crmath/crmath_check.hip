// crmath_check.hip -- TEST INFRASTRUCTURE: exhaustive GPU check of the
// exact-precision kernel's correctly rounded building blocks
// (sdf3d_amd/csrc/cr_math.h) against the generic sequences they replace:
//   sqrt : cr_sqrt(x) vs IEEE sqrtf(x) on all 2^32 bit patterns
//   sqrtbounded : cr_sqrt with the one-compare guard (SDF_CRM_SQRT_GUARD 1)
//          vs sqrtf on all 2^32 bit patterns: "effective" counts mismatches
//          other than x = +INF (the one input it does not cover)
//   sqrtwide : the unguarded sqrt_fast(x) vs sqrtf(x) on EVERY positive normal
//          x (v_cmp_class's "positive normal"): "mismatch" counts them all,
//          "effective" those below 2^-100 (the range a class-only guard would
//          add at the bottom; the top, 2^100 .. FLT_MAX, is the rest)
//   rcp  : rcp_fast(x) vs IEEE 1.0f / x on its domain [2^-100, 2^100)
//   log  : cr_log(x) vs (float)log((double)x) on all 2^32 bit patterns
//   smin : div_scaled(n, k, sc, ys) vs n / k over the smooth-min domain
//          (every positive finite k, n in [0, k]): bits, and h*h*k*0.25
//          (what the smooth-min uses) -- 2^32 (k, n) pairs, k uniform in
//          bits, n spread over [0, k] including tiny and denormal n
//   sminedge : the same comparison on 2^32 pairs from four edge families
//          (ADVICE r03): denormal k; k within 2^20 ulps of FLT_MAX; k >= 2^64
//          with n so small that n * sc underflows; tiny normal k (2^-126 ..
//          2^-100)
//   sminh / sminhedge : the smooth-min's whole h by smin_h (round 6: one
//          clamped FMA + div_prepared) vs IEEE max(k - |e|, 0) / k, 2^32
//          sampled (k, e) pairs each (k over every positive float / from the
//          edge families; e of either sign, near k, tiny, denormal, huge);
//          "effective" compares what the smooth-min subtracts: h h (k/4)
//          (the kernel's form, k >= 2^-64) against ((h h) k) 0.25
//   minmax : v_min_f32 / v_max_f32 vs the GLSL select on the operand pairs
//          the exact kernel relies on (hw_min / hw_max)
//   rcpneg : rcp_fast on the negative half of its domain
//   div  : the Markstein divisions (div_one / div_refined) vs IEEE a / b on
//          2^32 sampled pairs (edge families included)
//   pow  : shade.h spec_pow<exact>(x, n) (repeated squaring in fp64, the
//          library pow on lanes near a rounding boundary) vs the library
//          (float)pow((double)x, (double)n), for EVERY float x in [0, 1.0001]
//          (spec_x = max(N.H, 0)) and every integer shininess n in [0, 64]
// Prints one JSON line.  Built by sdf3d_amd/build.py (build_crmath_check);
// run by tests/test_gpu_crmath.py.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

#include "../../sdf3d_amd/csrc/cr_math.h"
#include "../../sdf3d_amd/csrc/shade.h"

struct Counts {
  unsigned long long mismatch, fast, effective;
  unsigned first[8];
  unsigned nfirst;
};

__device__ __forceinline__ bool same_bits(float a, float b) {
  return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}

__device__ void tally(Counts* c, bool bad, bool fast, bool eff, unsigned tag) {
  const unsigned long long mb = __builtin_amdgcn_ballot_w64(bad);
  const unsigned long long fb = __builtin_amdgcn_ballot_w64(fast);
  const unsigned long long eb = __builtin_amdgcn_ballot_w64(eff);
  const unsigned lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if (lane == 0) {
    if (mb) atomicAdd(&c->mismatch, (unsigned long long)__builtin_popcountll(mb));
    if (fb) atomicAdd(&c->fast, (unsigned long long)__builtin_popcountll(fb));
    if (eb) atomicAdd(&c->effective, (unsigned long long)__builtin_popcountll(eb));
  }
  if (bad) {
    const unsigned slot = atomicAdd(&c->nfirst, 1u);
    if (slot < 8) c->first[slot] = tag;
  }
}

__global__ void check_sqrt(unsigned base, Counts* c) {
  const unsigned u = base + blockIdx.x * blockDim.x + threadIdx.x;
  const float x = __uint_as_float(u);
  const float a = sdf::crm::cr_sqrt(x), b = __builtin_sqrtf(x);
  const bool bad = !same_bits(a, b);
  tally(c, bad, sdf::crm::sqrt_guard_g<0>(x), bad, u);
}

// the one-compare guard (SDF_CRM_SQRT_GUARD 1): every x but +INF
__global__ void check_sqrt_bounded(unsigned base, Counts* c) {
  const unsigned u = base + blockIdx.x * blockDim.x + threadIdx.x;
  const float x = __uint_as_float(u);
  const float a = sdf::crm::cr_sqrt_g<1>(x), b = __builtin_sqrtf(x);
  const bool bad = !same_bits(a, b);
  tally(c, bad, sdf::crm::sqrt_guard_g<1>(x), bad && u != 0x7F800000u, u);
}

__global__ void check_sqrt_wide(unsigned base, Counts* c) {
  const unsigned u = base + blockIdx.x * blockDim.x + threadIdx.x;
  const float x = __uint_as_float(u);
  const bool in = (u - 0x00800000u) < (0x7F800000u - 0x00800000u);   // positive normal
  const bool bad = in && !same_bits(sdf::crm::sqrt_fast(x), __builtin_sqrtf(x));
  tally(c, bad, in, bad && u < 0x0D800000u, u);
}

__global__ void check_rcp(unsigned base, Counts* c) {
  const unsigned u = base + blockIdx.x * blockDim.x + threadIdx.x;
  const float x = __uint_as_float(u);
  const bool in = sdf::crm::sqrt_fast_ok(x);   // its domain: [2^-100, 2^100)
  const float a = sdf::crm::rcp_fast(x), b = 1.0f / x;
  const bool bad = in && !same_bits(a, b);
  tally(c, bad, in, bad, u);
}

__global__ void check_log(unsigned base, Counts* c) {
  const unsigned u = base + blockIdx.x * blockDim.x + threadIdx.x;
  const float x = __uint_as_float(u);
  const float a = sdf::crm::cr_log(x), b = (float)log((double)x);
  const bool bad = !same_bits(a, b);
  // "fast": lanes whose fast value was safe to round (recomputed here)
  const double v = sdf::crm::log_fast(x);
  const double tol = SDF_CRM_LOG_EPS * __builtin_fabs(v);
  const bool ok = ((float)(v - tol) == (float)v) & ((float)(v + tol) == (float)v) &
                  ((u - 0x00800000u) < (0x7F800000u - 0x00800000u));
  tally(c, bad, ok, bad, u);
}

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

__global__ void check_smin(unsigned base, Counts* c) {
  const unsigned i = base + blockIdx.x * blockDim.x + threadIdx.x;
  // k: 2^20 values, uniform in bits over every positive finite float
  // (denormals included: the host's scaling must cover them); n: 4096 per k
  const unsigned ki = i >> 12, ni = i & 4095u;
  const unsigned kbits = 1u + (unsigned)(((unsigned long long)hash32(ki) * 0x7F7FFFFFull) >> 32);
  const float k = __uint_as_float(kbits);
  // the host's preparation (sdf_abi.cpp prepare_prims): sc = 2^min(-e, 127)
  // with k = m 2^e, m in [0.5, 1); ys = RN(1/(k sc))
  const int e = __builtin_amdgcn_frexp_expf(k);
  const float sc = __builtin_ldexpf(1.0f, -e < 127 ? -e : 127);
  const float ys = 1.0f / (k * sc);
  float n;
  const unsigned h = hash32(i * 2654435761u + 12345u);
  if (ni < 2048) n = k * (__uint_as_float(0x3F800000u | (h >> 9)) - 1.0f);  // [0, k)
  else if (ni < 3072) n = __uint_as_float(h % kbits);                      // any float below k
  else if (ni < 3584) n = __uint_as_float(h & 0x007FFFFFu) < k
                              ? __uint_as_float(h & 0x007FFFFFu) : 0.0f;   // denormal
  else n = __uint_as_float(kbits - (h & 0xFFFu) < kbits ? kbits - (h & 0xFFFu) : 0u);
  if (!(n <= k)) n = k;
  const float a = sdf::crm::div_scaled(n, k, sc, ys), b = n / k;
  const bool bad = !same_bits(a, b);
  const bool eff = !same_bits(a * a * k * 0.25f, b * b * k * 0.25f);
  tally(c, bad, true, eff, i);
}

// the smooth-min's host preparation and comparison (check_smin)
__device__ __forceinline__ void smin_case(float k, float n, unsigned tag, Counts* c) {
  const int e = __builtin_amdgcn_frexp_expf(k);
  const float sc = __builtin_ldexpf(1.0f, -e < 127 ? -e : 127);
  const float ys = 1.0f / (k * sc);
  if (!(n <= k)) n = k;
  const float a = sdf::crm::div_scaled(n, k, sc, ys), b = n / k;
  const bool bad = !same_bits(a, b);
  const bool eff = !same_bits(a * a * k * 0.25f, b * b * k * 0.25f);
  tally(c, bad, true, eff, tag);
}

__global__ void check_smin_edges(unsigned base, Counts* c) {
  const unsigned i = base + blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned fam = i >> 30, ki = (i >> 12) & 0x3FFFFu, ni = i & 4095u;
  const unsigned hk = hash32(ki * 0x9E3779B9u + fam), h = hash32(i * 2654435761u + 777u);
  unsigned kbits;
  switch (fam) {
    case 0: kbits = 1u + hk % 0x007FFFFEu; break;                    // denormal k
    case 1: kbits = 0x7F7FFFFFu - (hk & 0xFFFFFu); break;            // near FLT_MAX
    case 2: kbits = 0x5F800000u + hk % (0x7F7FFFFFu - 0x5F800000u); break;   // k >= 2^64
    default: kbits = 0x00800000u + hk % (0x0D800000u - 0x00800000u); break;  // 2^-126..2^-100
  }
  const float k = __uint_as_float(kbits);
  float n;
  if (fam == 2) {
    // n * sc underflows: sc <= 2^-63, so any n below 2^-63 (denormal or tiny)
    n = ni < 2048 ? __uint_as_float(h & 0x007FFFFFu)                  // denormal
                  : __uint_as_float(0x00800000u + h % (0x20000000u - 0x00800000u));
  } else if (ni < 2048) {
    n = k * (__uint_as_float(0x3F800000u | (h >> 9)) - 1.0f);           // [0, k)
  } else if (ni < 3584) {
    n = __uint_as_float(h % kbits);                                     // any float below k
  } else {
    n = __uint_as_float(kbits - (h & 0xFFFu) < kbits ? kbits - (h & 0xFFFu) : 0u);   // near k
  }
  smin_case(k, n, i, c);
}

// The smooth-min's whole h (cr_math.h smin_h, round 6: the subtraction from
// k, the max and the scaling as one clamped FMA, then div_prepared) vs the
// IEEE max(k - |e|, 0) / k the oracle computes, for e = RN(a - b) of either
// sign: bits, and ("effective") h*h*k*0.25, what the smooth-min uses.  k as in
// check_smin (every positive finite float, uniform in bits) or, with `edge`,
// from check_smin_edges' families; |e| spread over [0, 2k] (most of it below
// k), within 4096 ulps of k on both sides, tiny and denormal, and far above k.
__device__ __forceinline__ void sminh_case(float k, float e, unsigned tag, Counts* c) {
  const int ex = __builtin_amdgcn_frexp_expf(k);
  const float sc = __builtin_ldexpf(1.0f, -ex < 127 ? -ex : 127);
  const float ksc = k * sc;
  const float ys = 1.0f / ksc;
  const float a = sdf::crm::smin_h(e, sc, ksc, ys);
  const float n = k - __builtin_fabsf(e);
  const float b = (n > 0.0f ? n : 0.0f) / k;
  const bool bad = !same_bits(a, b);
  // what the kernel forms: h h (k/4) for the k sdf_validate admits (>= 2^-64),
  // against the oracle's ((h h) k) 0.25; below, the unfolded product
  const bool eff = k >= 0x1p-64f ? !same_bits(a * a * (k * 0.25f), b * b * k * 0.25f)
                                 : !same_bits(a * a * k * 0.25f, b * b * k * 0.25f);
  tally(c, bad, true, eff, tag);
}
__device__ __forceinline__ float sminh_e(float k, unsigned kbits, unsigned ni, unsigned h) {
  float e;
  if (ni < 1536) e = k * 2.0f * (__uint_as_float(0x3F800000u | (h >> 9)) - 1.0f);   // [0, 2k)
  else if (ni < 2560) e = __uint_as_float(h % kbits);                                // below k
  else if (ni < 3072) e = __uint_as_float(h & 0x007FFFFFu);                          // denormal
  else if (ni < 3840) {                                                              // near k
    const unsigned d = h & 0xFFFu;
    e = __uint_as_float((h & 0x1000u) ? (kbits + d < 0x7F800000u ? kbits + d : kbits)
                                      : (kbits > d ? kbits - d : 0u));
  } else e = __uint_as_float(kbits + (h % (0x7F7FFFFFu - kbits + 1u)));              // above k
  return (h & 0x80000000u) ? -e : e;
}
__global__ void check_sminh(unsigned base, Counts* c) {
  const unsigned i = base + blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned ki = i >> 12, ni = i & 4095u;
  const unsigned kbits = 1u + (unsigned)(((unsigned long long)hash32(ki * 31u + 7u) * 0x7F7FFFFFull) >> 32);
  const unsigned h = hash32(i * 2654435761u + 99991u);
  sminh_case(__uint_as_float(kbits), sminh_e(__uint_as_float(kbits), kbits, ni, h), i, c);
}
__global__ void check_sminh_edges(unsigned base, Counts* c) {
  const unsigned i = base + blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned fam = i >> 30, ki = (i >> 12) & 0x3FFFFu, ni = i & 4095u;
  const unsigned hk = hash32(ki * 0x9E3779B9u + fam + 17u), h = hash32(i * 2654435761u + 4242u);
  unsigned kbits;
  switch (fam) {
    case 0: kbits = 1u + hk % 0x007FFFFEu; break;                    // denormal k
    case 1: kbits = 0x7F7FFFFFu - (hk & 0xFFFFFu); break;            // near FLT_MAX
    case 2: kbits = 0x3D800000u + hk % (0x3F800000u - 0x3D800000u); break;   // k in [2^-4, 1)
    default: kbits = 0x00800000u + hk % (0x0D800000u - 0x00800000u); break;  // 2^-126..2^-100
  }
  sminh_case(__uint_as_float(kbits), sminh_e(__uint_as_float(kbits), kbits, ni, h), i, c);
}

// The hardware v_min_f32 / v_max_f32 against the GLSL select gmin/gmax on
// the operand pairs where the exact kernel uses the former (render_kernel.inc
// hw_min / hw_max): the select returns its first operand unless the second
// is strictly smaller (larger), so the two differ only for a NaN first
// operand or a (+0, -0) / (-0, +0) pair.  Lane i takes pair i of the table.
__device__ __forceinline__ float hwmin(float x, float y) {
  float r;
  asm volatile("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
__device__ __forceinline__ float hwmax(float x, float y) {
  float r;
  asm volatile("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
  return r;
}
__global__ void check_minmax(unsigned base, Counts* c) {
  const unsigned i = base + blockIdx.x * blockDim.x + threadIdx.x;
  const float nan = __uint_as_float(0x7FC00000u), inf = __builtin_inff();
  const float z = 0.0f, nz = __uint_as_float(0x80000000u);
  // min(x, y): (accumulator or shadow value, primitive value or quotient)
  const float mins[][2] = {{nz, z}, {z, 1.0f}, {1.0f, z}, {-1.0f, 2.0f}, {2.0f, -1.0f},
                           {1.0f, nan}, {-inf, nan}, {z, nan}, {nz, nan}, {inf, 3.0f},
                           {nz, 1.0f}, {z, inf}, {-3.0f, -3.0f}};
  // max(x, +0) / max(+0, y): the smooth-min's h, the shadow's denominator
  const float maxs[][2] = {{z, z}, {1.0f, z}, {-1.0f, z}, {-inf, z}, {inf, z},
                           {z, nan}, {z, -1.0f}, {z, 2.0f}, {z, -inf}};
  constexpr unsigned nmin = sizeof(mins) / sizeof(mins[0]), nmax = sizeof(maxs) / sizeof(maxs[0]);
  bool bad = false;
  if (i < nmin) {
    const float x = mins[i][0], y = mins[i][1];
    bad = !same_bits(hwmin(x, y), y < x ? y : x);
  } else if (i < nmin + nmax) {
    const float x = maxs[i - nmin][0], y = maxs[i - nmin][1];
    bad = !same_bits(hwmax(x, y), x < y ? y : x);
  }
  if (i < nmin + nmax) tally(c, bad, true, bad, i);
}

// x = index (bits) in [0, 0x3F800347) i.e. [0, 1.0001]; every n in [0, 64]
constexpr unsigned kPowXEnd = 0x3F800347u;
__global__ void check_pow(unsigned base, Counts* c) {
  const unsigned u = base + blockIdx.x * blockDim.x + threadIdx.x;
  // past the end: only the high lanes of the last wave (tally counts from
  // lane 0, which is inside) and whole waves after it
  if (u >= kPowXEnd) return;
  const float x = __uint_as_float(u);
  unsigned long long bad_n = 0ull;
  for (int n = 0; n <= 64; n++) {
    const float a = sdf::spec_pow<true>(x, (float)n);
    const float b = (float)pow((double)x, (double)n);
    if (!same_bits(a, b)) bad_n |= 1ull << (n & 63);
  }
  tally(c, bad_n != 0ull, true, bad_n != 0ull, u);
}

// rcp_fast on the negative half of its domain: -[2^-100, 2^100) (the
// shadow march's divisor 2 h_prev may be negative)
__global__ void check_rcp_neg(unsigned base, Counts* c) {
  const unsigned u = base + blockIdx.x * blockDim.x + threadIdx.x;
  const float x = -__uint_as_float(u);
  const bool in = sdf::crm::sqrt_fast_ok(-x);
  const float a = sdf::crm::rcp_fast(x), b = 1.0f / x;
  const bool bad = in && !same_bits(a, b);
  tally(c, bad, in, bad, u);
}

// Markstein divisions (cr_math.h div_refined / div_one; render_kernel.inc
// normalize, the Mandelbulb's (p - c) / scale, its DE, the shadow march):
// 2^32 sampled (a, b) pairs, b of magnitude log-uniform over [2^-30, 2^30)
// (either sign) plus out-of-range b, a from four families: |a| <= |b|
// (normalize), any magnitude in [2^-60, 2^60), quotients within a few ulps of
// a power of two or of 1 (hard rounding cases), and zeros, denormals, tiny
// and huge a (the guard's edges).  "mismatch": div_one (guard included) vs
// IEEE a / b on every pair; "effective": the unguarded two-step quotient vs
// IEEE on the pairs inside the guard ("fast_path" counts those).
__global__ void check_div(unsigned base, Counts* c) {
  const unsigned i = base + blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned fam = i >> 30;
  const unsigned h1 = hash32(i * 2654435761u + 99u), h2 = hash32(h1 ^ 0x5bd1e995u),
                 h3 = hash32(h2 + i);
  // b: exponent in [-30, 29] (1 in 64: [-40, 40], partly outside), random sign
  const int eb = (h1 & 63u) == 0u ? (int)(h1 >> 6) % 81 - 40 : (int)((h1 >> 6) % 60u) - 30;
  float b = __builtin_ldexpf(__uint_as_float(0x3F800000u | (h2 & 0x7FFFFFu)), eb);
  if (h2 & 0x80000000u) b = -b;
  float a;
  switch (fam) {
    case 0:   // |a| <= |b| (normalize's components)
      a = b * (2.0f * __uint_as_float(0x3F800000u | (h3 >> 9)) - 3.0f);
      break;
    case 1: {  // any magnitude 2^-60 .. 2^60
      const int ea = (int)(h3 % 120u) - 60;
      a = __builtin_ldexpf(__uint_as_float(0x3F800000u | (hash32(h3) & 0x7FFFFFu)), ea);
      if (h3 & 1u) a = -a;
      break;
    }
    case 2: {  // a = b * (2^k +- a few ulps): quotients near powers of two
      const int k = (int)(h3 % 41u) - 20;
      const float t = __builtin_ldexpf(1.0f, k);
      const int d = (int)(hash32(h3) % 9u) - 4;
      a = b * __uint_as_float(__float_as_uint(t) + (unsigned)d);
      break;
    }
    default: {  // edges: +-0, denormals, tiny, huge, just inside / outside the guard
      const unsigned sel = h3 % 8u;
      const unsigned r = hash32(h3);
      a = sel == 0 ? 0.0f : sel == 1 ? -0.0f : sel == 2 ? __uint_as_float(r & 0x007FFFFFu)
        : sel == 3 ? __builtin_ldexpf(1.0f + (r >> 9) * 0x1p-23f, -61 + (int)(r % 4u))
        : sel == 4 ? __builtin_ldexpf(1.0f + (r >> 9) * 0x1p-23f, 58 + (int)(r % 4u))
        : sel == 5 ? __uint_as_float(0x3F800000u | (r >> 9)) * 1e30f
        : sel == 6 ? __builtin_ldexpf(1.0f, -60) : -__builtin_ldexpf(1.0f, 60) * 0.999f;
      break;
    }
  }
  const float ieee = a / b;
  const bool bad = !same_bits(sdf::crm::div_one(a, b), ieee);
  const uint32_t ua = (__float_as_uint(a) << 1) - 1u;
  const bool in = sdf::crm::divisor_ok(b) && ua >= (0x21800000u << 1) - 1u &&
                  (ua < (0x5D800000u << 1) - 1u || ua == 0xFFFFFFFFu);
  const float mb = __builtin_fabsf(b);
  const bool eff = in && !same_bits(sdf::crm::div_refined(__builtin_copysignf(1.0f, b) * a, mb,
                                                          sdf::crm::rcp_fast(mb)),
                                    ieee);
  tally(c, bad, in, eff, i);
}

static int run(const char* name, void (*kern)(unsigned, Counts*), Counts* d, char* out,
               size_t cap, unsigned long long end = 1ull << 32) {
  (void)hipMemset(d, 0, sizeof(Counts));
  const unsigned threads = 256, chunk = 1u << 28;
  for (unsigned long long base = 0; base < end; base += chunk) {
    hipLaunchKernelGGL(kern, dim3(chunk / threads), dim3(threads), 0, 0, (unsigned)base, d);
    if (hipDeviceSynchronize() != hipSuccess) return -1;
  }
  Counts h;
  (void)hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost);
  char firsts[200] = "";
  for (unsigned j = 0; j < (h.nfirst < 8 ? h.nfirst : 8); j++) {
    char tmp[24];
    snprintf(tmp, sizeof tmp, "%s%u", j ? "," : "", h.first[j]);
    strncat(firsts, tmp, sizeof firsts - strlen(firsts) - 1);
  }
  return snprintf(out, cap, "\"%s\": {\"inputs\": %llu, \"mismatch\": %llu, \"effective\": %llu, "
                  "\"fast_path\": %llu, \"first\": [%s]}", name, end, h.mismatch,
                  h.effective, h.fast, firsts);
}

int main(int argc, char** argv) {
  Counts* d;
  if (hipMalloc(&d, sizeof(Counts)) != hipSuccess) return 2;
  const bool all = argc < 2;
  struct Check {
    const char* name;
    void (*kern)(unsigned, Counts*);
    unsigned long long end;
    char out[400];
  } checks[] = {{"rcp", check_rcp, 1ull << 32, ""},   {"sqrt", check_sqrt, 1ull << 32, ""},
                {"log", check_log, 1ull << 32, ""},   {"smin", check_smin, 1ull << 32, ""},
                {"sminedge", check_smin_edges, 1ull << 32, ""},
                {"sminh", check_sminh, 1ull << 32, ""},
                {"sminhedge", check_sminh_edges, 1ull << 32, ""},
                {"pow", check_pow, kPowXEnd, ""}, {"minmax", check_minmax, 256, ""},
                {"rcpneg", check_rcp_neg, 1ull << 32, ""}, {"div", check_div, 1ull << 32, ""},
                {"sqrtwide", check_sqrt_wide, 1ull << 32, ""},
                {"sqrtbounded", check_sqrt_bounded, 1ull << 32, ""}};
  // an argument selects checks by name (e.g. "sqrt,log"; "smin" matches only
  // itself)
  auto wanted = [&](const char* name) {
    if (all) return true;
    for (const char* p = argv[1]; (p = strstr(p, name)) != nullptr; p += strlen(name)) {
      const char after = p[strlen(name)];
      const bool start = p == argv[1] || p[-1] == ',';
      if (start && (after == 0 || after == ',')) return true;
    }
    return false;
  };
  bool first = true;
  printf("{");
  for (Check& k : checks) {
    if (!wanted(k.name)) continue;
    if (run(k.name, k.kern, d, k.out, sizeof k.out, k.end) < 0) return 3;
    printf("%s%s", first ? "" : ", ", k.out);
    first = false;
  }
  printf("}\n");
  (void)hipFree(d);
  return 0;
}

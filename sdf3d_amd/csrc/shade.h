// shade.h -- a pixel's colour from its three shading terms, shared by the
// render kernels and the TILES decoder (tiles.hip) so that a frame assembled
// from TILES streams is bit-identical to one rendered in place.
//
// voxel_fragment.frag:204-210 (+ the AO extension, DESIGN.md Scene spec):
//   spec = pow(max(N.H, 0), shininess)            x = max(N.H, 0)
//   dif  = clamp(N.L, 0, 1) * shadow
//   c    = la * amb * ao + dif * mat_dif + spec * mat_ref,  alpha 1
// (ao = 1 without AO: la * amb * 1 is la * amb bit for bit).  The TILES wire
// carries (ao, dif, x) instead of the colour: the terms are smooth where the
// colour mixes them, and x^12 spreads x's residuals over 3.6 more bits, so
// the 4K C4 stream is 29 % smaller (TILES).
//
// The operation sequence is pinned here, not left to the translation unit's
// contraction mode: exact precision is the oracle's unfused fp32 sequence and
// fp64 pow rounded once (oracle/oracle_core.h shade_pixel), fast precision the
// FMA chain below.  Units that include this header are built with
// -ffp-contract=off or =fast-honor-pragmas (sdf3d_amd/build.py), both of
// which honour the pragma (=fast would fuse across it).
#pragma once

namespace sdf {

// The frame's shading constants as the kernel uses them (lam = light ambient
// x material ambient, rounded to fp32 once); TILES stream header words 4..13.
struct ShadeK {
  float lam[3], dif[3], ref[3], shin;
};

// TILES stream header word 2: what the three channels hold
enum TilesShade : uint32_t {
  kTilesRaw = 0,         // the channel values themselves (RGB)
  kTilesShadeFast = 1,   // shading terms of a fast-precision render
  kTilesShadeExact = 2   // shading terms of an exact-precision render
};

// Exact precision: pow in fp64, rounded to fp32 once (the oracle's cr_powf).
// For an integer exponent n in [0, 64] (the shininess, a uniform; 12 by
// default) x^n by repeated squaring in fp64 instead of the library pow (~130
// fp64 instructions).  Binary powering is one parenthesisation of the product
// of n factors x: expanded as a product tree (a squared node's rounding error
// counts once per use) it has n - 1 multiplications, so with u = 2^-53 the
// value v satisfies |v / x^n - 1| <= (n - 1) u / (1 - (n - 1) u) < 2^-46 for
// n <= 64 (no intermediate underflows where x^n is near a float: x <= 1 keeps
// every partial product >= x^n, x > 1 keeps it >= 1).  The exhaustive GPU
// comparison with the library pow for every n in [0, 64] and every x in
// [0, 1.0001] (tests/crmath "pow", tests/test_gpu_crmath.py) checks it.  Where both ends of a 2^-44 interval around it round to the same
// float, that float is the correct rounding of x^n -- and of the library's
// fp64 pow, which lies in the same interval; other lanes (rounding
// boundaries, NaN) take the library pow.  SDF_SHADE_LIBRARY_POW 1: the
// library pow alone -- the same floats (the TILES decoder used it until
// round 5 to keep its tile loop rolled at 8 waves/SIMD; on exact-precision
// streams it cost 0.084 ms of decode per 4K frame, tiles.hip).
// The library fp64 pow, out of line (SDF_SHADE_POW_CALL 1): inlined, its
// ~30 fp64 constants were hoisted out of the persistent frames kernel's tile
// loop (render_kernel.inc render_frames) and spilled to scratch; as a call
// they exist only on the rare lanes that need it.
#if !defined(SDF_SHADE_POW_CALL) || SDF_SHADE_POW_CALL
inline __device__ __attribute__((noinline)) float library_pow(float x, float y) {
  return (float)pow((double)x, (double)y);
}
#else
__device__ __forceinline__ float library_pow(float x, float y) {
  return (float)pow((double)x, (double)y);
}
#endif

template <bool EXACT>
__device__ __forceinline__ float spec_pow(float x, float shin) {
#pragma clang fp contract(off)
  if constexpr (EXACT) {
#if !defined(SDF_SHADE_LIBRARY_POW) || !SDF_SHADE_LIBRARY_POW
    const int n = (int)shin;
    if ((float)n == shin && n >= 0 && n <= 64) {
      double b = (double)x, v = 1.0;
      // n is uniform: each step's multiplies sit behind real (scalar)
      // branches -- an empty volatile asm keeps LLVM from if-converting them
      // into two fp64 multiplies and four v_cndmask per step (the TILES
      // decoder's exact shading: ~24 VALU per pixel for n = 12, 5 now)
      for (int e = n; e != 0; e >>= 1) {
        if (e & 1) {
#if !defined(SDF_SHADE_POW_BRANCH) || SDF_SHADE_POW_BRANCH
          asm volatile("");
#endif
          v = v * b;
        }
        if (e > 1) {
#if !defined(SDF_SHADE_POW_BRANCH) || SDF_SHADE_POW_BRANCH
          asm volatile("");
#endif
          b = b * b;
        }
      }
      const float r = (float)v;
#if !defined(SDF_SHADE_POW_BITCHECK) || SDF_SHADE_POW_BITCHECK
      // The same test on v's bits (as cr_math.h log_round_ok): for a normal
      // float r, an fp32 rounding midpoint is a double with low 29 mantissa
      // bits 2^28, and the tolerance is below 2^9 of v's ulps; v < 2^-151
      // rounds to +0 from anywhere in its interval.  Lanes with a subnormal
      // r (x^n in [2^-151, 2^-126): x^12 for x in ~[1.6e-4, 6.9e-4]) take
      // the interval test below, the library pow only where that fails.
      const uint32_t lo = (uint32_t)__builtin_bit_cast(unsigned long long, v);
      const bool ok = ((((lo & 0x1FFFFFFFu) - (0x10000000u - 0x200u)) >= 0x400u) &
                       (r >= 0x1p-126f)) | (v < 0x1p-151);
#else
      const double tol0 = 0x1p-44 * __builtin_fabs(v);
      const bool ok = ((float)(v - tol0) == r) & ((float)(v + tol0) == r);
#endif
      float out = r;
      if (__builtin_amdgcn_ballot_w64(!ok) != 0) {
        asm volatile("" ::: "memory");   // keep the library pow out of the fast path
        const double tol = 0x1p-44 * __builtin_fabs(v);
        const bool ok2 = ok | (((float)(v - tol) == r) & ((float)(v + tol) == r));
        out = ok2 ? r : library_pow(x, shin);
      }
      return out;
    }
#endif
    return library_pow(x, shin);
  } else {
    return __builtin_amdgcn_exp2f(shin * __builtin_amdgcn_logf(x));
  }
}

template <bool EXACT>
__device__ __forceinline__ float shade_channel(float lam, float md, float mr, float ao, float dif,
                                               float spec) {
#pragma clang fp contract(off)
  const float a = lam * ao;
  if constexpr (EXACT) {
    return (a + dif * md) + spec * mr;
  } else {
    return __builtin_fmaf(spec, mr, __builtin_fmaf(dif, md, a));
  }
}

template <bool EXACT>
__device__ __forceinline__ float4 shade_colour(const ShadeK& K, float ao, float dif, float x) {
  const float spec = spec_pow<EXACT>(x, K.shin);
  return make_float4(shade_channel<EXACT>(K.lam[0], K.dif[0], K.ref[0], ao, dif, spec),
                     shade_channel<EXACT>(K.lam[1], K.dif[1], K.ref[1], ao, dif, spec),
                     shade_channel<EXACT>(K.lam[2], K.dif[2], K.ref[2], ao, dif, spec), 1.0f);
}

}  // namespace sdf

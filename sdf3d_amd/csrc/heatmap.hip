// heatmap.hip -- step-count debug view.
//
// The reference ships a Turbo colormap (Code/kernel/utilities.cl:7-284: a
// 256-entry LUT indexed by round(255 * intensity), clamped to [0, 255]) that
// nothing calls.  Here it colours the per-pixel iteration counts that
// sdf_render can emit, to show where sphere tracing spends its steps.  The
// colour of entry i is the published polynomial approximation of Turbo
// evaluated at x = i / 255 (not the reference's table: parity with its LUT
// is unpinned, the view is diagnostic).  One lane per pixel; HBM-bound
// (8 B in, <= 16 B out per pixel).
#include <hip/hip_runtime.h>

#include "kernel_args.h"

namespace sdf {

__device__ __forceinline__ float3 turbo(float x) {
  const float x2 = x * x, x3 = x2 * x, x4 = x2 * x2, x5 = x3 * x2;
  float r = 0.13572138f + 4.61539260f * x - 42.66032258f * x2 + 132.13108234f * x3 -
            152.94239396f * x4 + 59.28637943f * x5;
  float g = 0.09140261f + 2.19418839f * x + 4.84296658f * x2 - 14.18503333f * x3 +
            4.27729857f * x4 + 2.82956604f * x5;
  float b = 0.10667330f + 12.64194608f * x - 60.58204836f * x2 + 110.36276771f * x3 -
            89.90310912f * x4 + 27.34824973f * x5;
  return make_float3(fminf(fmaxf(r, 0.f), 1.f), fminf(fmaxf(g, 0.f), 1.f),
                     fminf(fmaxf(b, 0.f), 1.f));
}

__device__ __forceinline__ unsigned unorm8(float c) {
  return (unsigned)__fadd_rn(__fmul_rn(fminf(fmaxf(c, 0.f), 1.f), 255.0f), 0.5f);
}

__global__ __launch_bounds__(256) void heatmap_kernel(const int2* __restrict__ steps, int count,
                                                      int which, float inv_max, int format,
                                                      void* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int2 s = steps[i];
  const int n = which == 0 ? s.x : (which == 1 ? s.y : s.x + s.y);
  // utilities.cl: i = round(255 * intensity), clamped to [0, 255]
  int idx = (int)rintf(255.0f * ((float)n * inv_max));
  idx = idx < 0 ? 0 : (idx > 255 ? 255 : idx);
  const float3 c = turbo((float)idx / 255.0f);
  if (format == SDF_FORMAT_RGBA8) {
    reinterpret_cast<unsigned*>(out)[i] =
        unorm8(c.x) | (unorm8(c.y) << 8) | (unorm8(c.z) << 16) | (255u << 24);
  } else if (format == SDF_FORMAT_RGB32F) {
    float* q = reinterpret_cast<float*>(out) + 3 * (size_t)i;
    q[0] = c.x;
    q[1] = c.y;
    q[2] = c.z;
  } else if (format == SDF_FORMAT_RGBA16F) {
    const _Float16 h[4] = {(_Float16)c.x, (_Float16)c.y, (_Float16)c.z, (_Float16)1.0f};
    uint2 u;
    __builtin_memcpy(&u, h, 8);
    reinterpret_cast<uint2*>(out)[i] = u;
  } else {
    reinterpret_cast<float4*>(out)[i] = make_float4(c.x, c.y, c.z, 1.0f);
  }
}

int launch_heatmap(const int32_t* steps, int count, int which, int max_steps, int format,
                   void* out, void* stream) {
  if (count == 0) return 0;
  const float inv_max = max_steps > 0 ? 1.0f / (float)max_steps : 0.0f;
  hipLaunchKernelGGL(heatmap_kernel, dim3((count + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, reinterpret_cast<const int2*>(steps), count, which,
                     inv_max, format, out);
  return (int)hipGetLastError();
}

}  // namespace sdf

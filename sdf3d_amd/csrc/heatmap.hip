// heatmap.hip -- step-count debug view.
//
// The reference ships a Turbo colormap that nothing calls
// (Code/kernel/utilities.cl:7-284): a 256-entry RGB table (:12-267) indexed by
// i = round(255 * intensity), clamped to [0, 255] (:269-281).  Here it colours
// the per-pixel iteration counts sdf_render can emit, with intensity =
// count / max_steps, to show where sphere tracing spends its steps.  The table
// is the reference's own, carried as fp32 bit patterns (turbo_lut.inc,
// generated from the fixture tests/golden/turbo_lut.json), and OpenCL round()
// rounds half away from zero (roundf, not rintf).  One lane per pixel;
// HBM-bound (8 B in, <= 16 B out per pixel).
#include <hip/hip_runtime.h>

#include "kernel_args.h"

namespace sdf {

#include "turbo_lut.inc"

__device__ __forceinline__ float3 turbo(int i) {
  return make_float3(__uint_as_float(kTurboBits[3 * i]), __uint_as_float(kTurboBits[3 * i + 1]),
                     __uint_as_float(kTurboBits[3 * i + 2]));
}

__device__ __forceinline__ unsigned unorm8(float c) {
  return (unsigned)__fadd_rn(__fmul_rn(fminf(fmaxf(c, 0.f), 1.f), 255.0f), 0.5f);
}

__global__ __launch_bounds__(256) void heatmap_kernel(const int2* __restrict__ steps, int count,
                                                      int which, float max_steps, int format,
                                                      void* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int2 s = steps[i];
  const int n = which == 0 ? s.x : (which == 1 ? s.y : s.x + s.y);
  // utilities.cl:269-281: i = round(255 * intensity), clamped to [0, 255]
  const float intensity = max_steps > 0.0f ? __fdiv_rn((float)n, max_steps) : 0.0f;
  const float r = roundf(__fmul_rn(255.0f, intensity));
  const int idx = r > 255.0f ? 255 : (r > 0.0f ? (int)r : 0);
  const float3 c = turbo(idx);
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
  (void)hipGetLastError();  // a stale error of an earlier call is not this launch's
  hipLaunchKernelGGL(heatmap_kernel, dim3((count + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, reinterpret_cast<const int2*>(steps), count, which,
                     (float)max_steps, format, out);
  return (int)hipGetLastError();
}

}  // namespace sdf

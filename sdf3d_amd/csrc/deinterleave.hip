// deinterleave.hip -- root-side scatter of gathered row blocks into a frame.
//
// With an N-device interleaved tiling (sdf_tiling {B, r, N}), device r renders
// frame rows of blocks r, r+N, r+2N, ... densely ("packed").  After the gather
// the root holds the N packed parts back to back; this kernel moves every row
// to its place in the frame.  Pure HBM copy: 2 x 16 B per pixel; float4 per
// lane, one workgroup per frame row (rows are >= 512 float4 at the configs'
// widths, so each workgroup streams whole 2 KB+ rows).  New functionality:
// the reference renders into a single GL context (main.cpp:48,53).
#include <hip/hip_runtime.h>

#include "kernel_args.h"

namespace sdf {

// Rows are moved as 16-byte vectors when a row is a multiple of 16 bytes
// (every config: 3840 px x 4, 8 or 16 B), otherwise as 4-byte words.
template <class T>
__global__ __launch_bounds__(256) void deinterleave_rows(const T* __restrict__ parts,
                                                         int nparts, int part_stride_rows,
                                                         int row_elems, int block_rows,
                                                         T* __restrict__ frame) {
  const int y = blockIdx.x;
  const int b = y / block_rows;
  const int r = b % nparts;
  const int pr = (b / nparts) * block_rows + (y - b * block_rows);
  const T* src = parts + ((size_t)r * part_stride_rows + pr) * row_elems;
  T* dst = frame + (size_t)y * row_elems;
  for (int x = threadIdx.x; x < row_elems; x += blockDim.x) dst[x] = src[x];
}

int launch_deinterleave(const void* parts, int nparts, int part_stride_rows, int row_bytes,
                        int height, int block_rows, void* frame, void* stream) {
  if (height == 0 || row_bytes == 0) return 0;
  (void)hipGetLastError();  // a stale error of an earlier call is not this launch's
  hipStream_t s = (hipStream_t)stream;
  if (row_bytes % 16 == 0) {
    hipLaunchKernelGGL(deinterleave_rows<uint4>, dim3(height), dim3(256), 0, s,
                       reinterpret_cast<const uint4*>(parts), nparts, part_stride_rows,
                       row_bytes / 16, block_rows, reinterpret_cast<uint4*>(frame));
  } else {
    hipLaunchKernelGGL(deinterleave_rows<unsigned>, dim3(height), dim3(256), 0, s,
                       reinterpret_cast<const unsigned*>(parts), nparts, part_stride_rows,
                       row_bytes / 4, block_rows, reinterpret_cast<unsigned*>(frame));
  }
  return (int)hipGetLastError();
}

// RGB32F parts (12 B/pixel, the lossless wire format) -> RGBA32F frame with
// alpha = 1 (the shader's constant alpha, voxel_fragment.frag:210).
__global__ __launch_bounds__(256) void deinterleave_rgb_rows(const float* __restrict__ parts,
                                                             int nparts, int part_stride_rows,
                                                             int width, int block_rows,
                                                             float4* __restrict__ frame) {
  const int y = blockIdx.x;
  const int b = y / block_rows;
  const int r = b % nparts;
  const int pr = (b / nparts) * block_rows + (y - b * block_rows);
  const float* src = parts + ((size_t)r * part_stride_rows + pr) * width * 3;
  float4* dst = frame + (size_t)y * width;
  for (int x = threadIdx.x; x < width; x += blockDim.x)
    dst[x] = make_float4(src[3 * x], src[3 * x + 1], src[3 * x + 2], 1.0f);
}

int launch_deinterleave_rgb(const void* parts, int nparts, int part_stride_rows, int width,
                            int height, int block_rows, void* frame, void* stream) {
  if (height == 0 || width == 0) return 0;
  (void)hipGetLastError();  // a stale error of an earlier call is not this launch's
  hipLaunchKernelGGL(deinterleave_rgb_rows, dim3(height), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const float*>(parts), nparts, part_stride_rows, width,
                     block_rows, reinterpret_cast<float4*>(frame));
  return (int)hipGetLastError();
}

}  // namespace sdf

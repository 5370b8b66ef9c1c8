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

__global__ __launch_bounds__(256) void deinterleave_rows(const float4* __restrict__ parts,
                                                         int nparts, int part_stride_rows,
                                                         int width, int block_rows,
                                                         float4* __restrict__ frame) {
  const int y = blockIdx.x;
  const int b = y / block_rows;
  const int r = b % nparts;
  const int pr = (b / nparts) * block_rows + (y - b * block_rows);
  const float4* src = parts + ((size_t)r * part_stride_rows + pr) * width;
  float4* dst = frame + (size_t)y * width;
  for (int x = threadIdx.x; x < width; x += blockDim.x) dst[x] = src[x];
}

int launch_deinterleave(const float* parts, int nparts, int part_stride_rows, int width,
                        int height, int block_rows, float* frame, void* stream) {
  if (height == 0 || width == 0) return 0;
  hipLaunchKernelGGL(deinterleave_rows, dim3(height), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const float4*>(parts), nparts, part_stride_rows, width,
                     block_rows, reinterpret_cast<float4*>(frame));
  return (int)hipGetLastError();
}

}  // namespace sdf

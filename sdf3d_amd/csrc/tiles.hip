// tiles.hip -- the TILES wire format (sdf_abi.h SDF_FORMAT_TILES) around the
// render kernel's encoder (render_kernel.inc store_tiles):
//
//   compaction  the encoder leaves each tile's record in a fixed worst-case
//               slot and its size in sizes[]; one workgroup scans the sizes
//               into the offset table and `used`, then one wave per tile
//               copies its record into the contiguous stream (kernel_args.h
//               TilesLayout).
//   decode      fused with the multi-device de-interleave: rank r's stream
//               holds the packed rows of tiling {block_rows, r, nparts};
//               every record is expanded to RGBA32F (alpha 1) straight into
//               its rows of the assembled frame.  One wave = one tile of one
//               part (lane j = pixel 8 * row + column): the planes arrive by
//               one vector load, each is broadcast with v_readlane, lanes
//               gather their residual's bits, un-zigzag, and the tile's 2-D
//               inclusive prefix sum (rows by 8-lane shuffles, then columns)
//               inverts the gradient predictor exactly in uint32 arithmetic.
//
// All three are HBM-bound at a few bytes per pixel (16 out for the decode).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernel_args.h"

namespace sdf {
namespace {

// Transpose of the 64 x 64 bit matrix whose row r is lane r's word: on
// return lane c holds column c (bit r = bit c of lane r's input).  Six
// butterfly stages swap the off-diagonal j x j blocks of every 2j x 2j block
// between lanes r and r ^ j (a 64-bit shuffle, shifts, masks).
__device__ __forceinline__ uint64_t transpose64(uint64_t a, int lane) {
  const uint64_t masks[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull, 0x00FF00FF00FF00FFull,
                             0x0F0F0F0F0F0F0F0Full, 0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
  for (int st = 0; st < 6; st++) {
    const int j = 32 >> st;
    const uint64_t m = masks[st];
    const uint32_t plo = (uint32_t)__shfl_xor((int)(uint32_t)a, j);
    const uint32_t phi = (uint32_t)__shfl_xor((int)(uint32_t)(a >> 32), j);
    const uint64_t p = (uint64_t)phi << 32 | plo;
    if (lane & j) {
      const uint64_t t = ((p >> j) ^ a) & m;        // the partner's block to take
      a ^= t;
    } else {
      const uint64_t t = ((a >> j) ^ p) & m;
      a ^= t << j;
    }
  }
  return a;
}

__device__ __forceinline__ uint32_t unordered_bits(uint32_t u) {
  return (u & 0x80000000u) ? (u ^ 0x7fffffffu) : u;
}

// rows of tiling {block_rows, part, nparts} in a frame of `height` rows
__device__ __forceinline__ int part_rows(int height, int block_rows, int part, int nparts) {
  const int nblocks = (height + block_rows - 1) / block_rows;
  if (part >= nblocks) return 0;
  const int mine = (nblocks - 1 - part) / nparts + 1;
  int rows = mine * block_rows;
  if ((nblocks - 1) % nparts == part) rows -= nblocks * block_rows - height;   // short last block
  return rows;
}

constexpr int kDecodeTiles = 8;   // tiles per wave of the decoder

// one tile: planes (pa: planes 0..63, pb: 64..95) -> RGBA32F frame rows
__device__ __forceinline__ void decode_tile(uint2 pa, uint2 pb, uint32_t widths, uint32_t f0,
                                            uint32_t f1, uint32_t f2, int tile, int lane,
                                            int part, int nparts, int rows, int width,
                                            int block_rows, float4* __restrict__ frame) {
  const int nplanes = (widths & 255) + ((widths >> 8) & 255) + ((widths >> 16) & 255);
  // transposed, lane j holds bit k of its residuals' concatenation (channel
  // c at bits [k_c, k_c + w_c))
  const uint64_t ta = transpose64((uint64_t)pa.y << 32 | pa.x, lane);
  const uint64_t tb = nplanes > 64 ? transpose64((uint64_t)pb.y << 32 | pb.x, lane) : 0ull;
  const uint32_t first[3] = {f0, f1, f2};
  const int col = lane & 7;
  float v[3];
  int k = 0;
#pragma unroll
  for (int ch = 0; ch < 3; ch++) {
    const int w = (widths >> (8 * ch)) & 255;
    const uint64_t lo64 = k < 64 ? (ta >> k) | (k ? tb << (64 - k) : 0ull) : tb >> (k - 64);
    uint32_t z = w ? (uint32_t)lo64 & (uint32_t)(0xFFFFFFFFull >> (32 - w)) : 0u;
    k += w;
    uint32_t r = (z >> 1) ^ (0u - (z & 1u));            // un-zigzag
    if (lane == 0) r = first[ch];                       // pixel 0 travels raw
    // 2-D inclusive prefix sum over the 8x8 tile (mod 2^32)
#pragma unroll
    for (int s = 1; s < 8; s <<= 1) {
      const uint32_t t = (uint32_t)__shfl_up((int)r, s, 8);
      if (col >= s) r += t;
    }
#pragma unroll
    for (int s = 8; s < 64; s <<= 1) {
      const uint32_t t = (uint32_t)__shfl_up((int)r, s, 64);
      if (lane >= s) r += t;
    }
    v[ch] = __uint_as_float(unordered_bits(r));
  }
  const int tiles_x = (width + 7) >> 3;
  const int ty = tile / tiles_x;
  const int x = (tile - ty * tiles_x) * 8 + col;
  const int pr = ty * 8 + (lane >> 3);
  if (x >= width || pr >= rows) return;
  const int blk = pr / block_rows;
  const int y = (part + blk * nparts) * block_rows + (pr - blk * block_rows);
  frame[(size_t)y * width + x] = make_float4(v[0], v[1], v[2], 1.0f);
}

// One wave = kDecodeTiles consecutive tiles of one part.  Their offsets and
// heads arrive by one vector load each (lane i: tile i); each tile's planes
// are loaded one tile ahead, so the load overlaps the previous tile's
// transpose and prefix sums.
__global__ __launch_bounds__(256) void decode_tiles(const uint8_t* __restrict__ parts,
                                                    int nparts, long long part_stride,
                                                    int width, int height, int block_rows,
                                                    int waves_per_part, float4* __restrict__ frame) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int part = gw / waves_per_part;
  if (part >= nparts) return;
  const int tbase = (gw - part * waves_per_part) * kDecodeTiles;
  const int rows = part_rows(height, block_rows, part, nparts);
  const int ntiles = ((width + 7) >> 3) * ((rows + 7) >> 3);
  if (tbase >= ntiles) return;
  const uint8_t* base = parts + (long long)part * part_stride;
  if (reinterpret_cast<const uint32_t*>(base)[1] == 0) return;   // no stream: rows rendered in place
  const TilesLayout Lt(ntiles);
  const int nt = min(kDecodeTiles, ntiles - tbase);
  const uint32_t offv = lane < nt ? reinterpret_cast<const uint32_t*>(base + Lt.table)[tbase + lane] : 0u;
  const uint4 hdv = lane < nt ? reinterpret_cast<const uint4*>(base + Lt.head)[tbase + lane]
                              : make_uint4(0u, 0u, 0u, 0u);
  const uint2* data = reinterpret_cast<const uint2*>(base + Lt.data);
  auto planes_of = [&](int k, int np, int from) -> uint2 {
    const uint32_t off = __builtin_amdgcn_readlane((int)offv, k);
    return lane + from < np ? data[off / 8 + from + lane] : make_uint2(0u, 0u);
  };
  auto nplanes_of = [&](uint32_t w) {
    return (int)((w & 255) + ((w >> 8) & 255) + ((w >> 16) & 255));
  };
  uint32_t wn = __builtin_amdgcn_readlane((int)hdv.x, 0);
  uint2 next = planes_of(0, nplanes_of(wn), 0);
#pragma unroll
  for (int k = 0; k < kDecodeTiles; k++) {
    if (k >= nt) break;
    const uint32_t widths = wn;
    const uint2 pa = next;
    const int np = nplanes_of(widths);
    const uint2 pb = np > 64 ? planes_of(k, np, 64) : make_uint2(0u, 0u);
    if (k + 1 < nt) {                     // prefetch the next tile's planes
      wn = __builtin_amdgcn_readlane((int)hdv.x, k + 1);
      next = planes_of(k + 1, nplanes_of(wn), 0);
    }
    decode_tile(pa, pb, widths, __builtin_amdgcn_readlane((int)hdv.y, k),
                __builtin_amdgcn_readlane((int)hdv.z, k), __builtin_amdgcn_readlane((int)hdv.w, k),
                tbase + k, lane, part, nparts, rows, width, block_rows, frame);
  }
}

// Offsets of the plane blocks in tile order: exclusive scan of 8 * (w0 + w1
// + w2) over the heads.  tiles_scan: 256 threads x 8 consecutive tiles per
// block of kScanTiles -> block-local offsets + the block's total.
// tiles_move: one wave per tile adds its block's prefix (the sum of earlier
// block totals, a wave reduction), writes the final offset, and copies its
// planes from the slot into the stream; the last tile writes `used`.
__device__ __forceinline__ uint32_t plane_bytes(uint32_t widths) {
  return 8u * ((widths & 255u) + ((widths >> 8) & 255u) + ((widths >> 16) & 255u));
}

__global__ __launch_bounds__(256) void tiles_scan(uint8_t* buf, int ntiles) {
  const TilesLayout L(ntiles);
  const uint4* head = reinterpret_cast<const uint4*>(buf + L.head);
  uint32_t* table = reinterpret_cast<uint32_t*>(buf + L.table);
  __shared__ uint32_t wsum[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int t0 = blockIdx.x * kScanTiles + tid * 8;
  uint32_t sz[8], sum = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    sz[i] = t0 + i < ntiles ? plane_bytes(head[t0 + i].x) : 0u;
    sum += sz[i];
  }
  // block exclusive scan of the thread sums: wave scan, then wave totals
  uint32_t inc = sum;
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const uint32_t v = (uint32_t)__shfl_up((int)inc, s, 64);
    if (lane >= s) inc += v;
  }
  if (lane == 63) wsum[wv] = inc;
  __syncthreads();
  uint32_t off = inc - sum;
  for (int i = 0; i < wv; i++) off += wsum[i];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    if (t0 + i < ntiles) table[t0 + i] = off;
    off += sz[i];
  }
  if (tid == 255)
    reinterpret_cast<uint32_t*>(buf + L.bsums)[blockIdx.x] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

__global__ __launch_bounds__(256) void tiles_move(uint8_t* buf, int ntiles) {
  const TilesLayout L(ntiles);
  const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tile >= ntiles) return;
  const int lane = threadIdx.x & 63;
  const int blk = tile / kScanTiles;
  const uint32_t* bsums = reinterpret_cast<const uint32_t*>(buf + L.bsums);
  uint32_t pre = 0;
  for (int i = lane; i < blk; i += 64) pre += bsums[i];
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) pre += (uint32_t)__shfl_xor((int)pre, s);
  uint32_t* table = reinterpret_cast<uint32_t*>(buf + L.table);
  const uint32_t off = table[tile] + pre;
  const uint32_t bytes = plane_bytes(reinterpret_cast<const uint4*>(buf + L.head)[tile].x);
  const uint2* src = reinterpret_cast<const uint2*>(buf + L.slots + (size_t)tile * kTilePlaneBytes);
  uint2* dst = reinterpret_cast<uint2*>(buf + L.data + off);
  for (uint32_t i = lane; i < bytes / 8; i += 64) dst[i] = src[i];
  if (lane == 0) {
    table[tile] = off;
    if (tile == ntiles - 1) {
      reinterpret_cast<uint32_t*>(buf)[0] = off + bytes;
      reinterpret_cast<uint32_t*>(buf)[1] = (uint32_t)ntiles;
    }
  }
}

}  // namespace

int launch_tiles_compact(void* stream_buf, int ntiles, void* stream) {
  if (ntiles <= 0) return 0;
  uint8_t* buf = reinterpret_cast<uint8_t*>(stream_buf);
  hipLaunchKernelGGL(tiles_scan, dim3((ntiles + kScanTiles - 1) / kScanTiles), dim3(256), 0,
                     (hipStream_t)stream, buf, ntiles);
  hipLaunchKernelGGL(tiles_move, dim3((ntiles + 3) / 4), dim3(256), 0, (hipStream_t)stream, buf,
                     ntiles);
  return (int)hipGetLastError();
}

int launch_tiles_decode(const void* parts, int nparts, long long part_stride, int width,
                        int height, int block_rows, void* frame, void* stream) {
  const int tiles_x = (width + 7) >> 3;
  // part 0 owns the most rows of an interleaved tiling
  const int nblocks = (height + block_rows - 1) / block_rows;
  const int rows0 = ((nblocks - 1) / nparts + 1) * block_rows;
  const int tiles_per_part = tiles_x * ((rows0 + 7) >> 3);
  const int waves_per_part = (tiles_per_part + kDecodeTiles - 1) / kDecodeTiles;
  const long long waves = (long long)waves_per_part * nparts;
  if (waves == 0) return 0;
  hipLaunchKernelGGL(decode_tiles, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, reinterpret_cast<const uint8_t*>(parts), nparts,
                     part_stride, width, height, block_rows, waves_per_part,
                     reinterpret_cast<float4*>(frame));
  return (int)hipGetLastError();
}

}  // namespace sdf

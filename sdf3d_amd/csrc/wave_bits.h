// wave_bits.h -- wave64 bit-matrix transpose shared by the TILES encoder
// (render_kernel.inc store_tiles) and decoder (tiles.hip decode_tiles).
//
// Transpose of the 64 x 64 bit matrix whose row r is lane r's word (lo =
// bits 0..31, hi = 32..63): on return lane c holds column c (bit r = bit c
// of lane r's input).  Six butterfly stages exchange the off-diagonal j x j
// blocks of every 2j x 2j block between lanes r and r ^ j:
//   j = 32     one v_permlane32_swap (lanes 32..63 of lo <-> lanes 0..31 of hi);
//   j <= 16    inside each 32-bit half: the partner's word (DPP quad_perm for
//              j = 1, 2, ds_swizzle for 4, 8, 16) rotated by j toward this
//              lane's blocks (v_alignbit, per-lane amount) and merged into
//              them (v_bfi, per-lane mask).
// A lane with bit j clear keeps its low blocks (mask m_j) and takes the
// partner's low blocks shifted up by j; a lane with bit j set keeps its high
// blocks and takes the partner's high blocks shifted down by j.
//
// Decoder: lane i holds bit plane i of a tile (bit j = bit i of pixel j's
// residual) -> lane j holds the concatenation of its residuals' bits.
// Encoder: lane j holds its residual z_j (hi = 0) -> lane b holds plane b.
#pragma once

namespace sdf {

struct TransposeLanes {
  uint32_t keep[5], rot[5];   // stages j = 16, 8, 4, 2, 1
  __device__ __forceinline__ explicit TransposeLanes(int lane) {
    const uint32_t m[5] = {0x0000FFFFu, 0x00FF00FFu, 0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const int j = 16 >> i;
      const bool upper = lane & j;
      keep[i] = upper ? ~m[i] : m[i];
      rot[i] = upper ? (uint32_t)j : (uint32_t)(32 - j);   // rotate right (rotl j = rotr 32 - j)
    }
  }
};

template <int J>
__device__ __forceinline__ uint32_t xor_partner(uint32_t v) {
  if constexpr (J == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  else if constexpr (J == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  else return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (J << 10));
}

// (a & mask) | (b & ~mask) in one v_bfi_b32 (the compiler splits it in two
// when the mask's complement is live)
__device__ __forceinline__ uint32_t bitfield_merge(uint32_t mask, uint32_t a, uint32_t b) {
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(mask), "v"(a), "v"(b));
  return r;
}

template <int I>
__device__ __forceinline__ void transpose_stage(uint32_t& lo, uint32_t& hi, const TransposeLanes& T) {
  constexpr int J = 16 >> I;
  const uint32_t plo = xor_partner<J>(lo), phi = xor_partner<J>(hi);
  const uint32_t qlo = __builtin_amdgcn_alignbit(plo, plo, T.rot[I]);
  const uint32_t qhi = __builtin_amdgcn_alignbit(phi, phi, T.rot[I]);
  lo = bitfield_merge(T.keep[I], lo, qlo);
  hi = bitfield_merge(T.keep[I], hi, qhi);
}

__device__ __forceinline__ void transpose64(uint32_t& lo, uint32_t& hi, const TransposeLanes& T) {
  const auto sw = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
  lo = sw[0];
  hi = sw[1];
  transpose_stage<0>(lo, hi, T);
  transpose_stage<1>(lo, hi, T);
  transpose_stage<2>(lo, hi, T);
  transpose_stage<3>(lo, hi, T);
  transpose_stage<4>(lo, hi, T);
}

}  // namespace sdf

// tiles.hip -- the TILES wire format (sdf_abi.h SDF_FORMAT_TILES) around the
// render kernel's encoder (render_kernel.inc store_tiles):
//
//   compaction  the encoder leaves each tile's words in a fixed worst-case
//               slot and its head (base widths, raw first pixel) in place;
//               tiles_scan turns the widths into block-local offsets and
//               per-block totals, tiles_move adds the block prefix and copies
//               each tile's words into the contiguous stream (kernel_args.h
//               TilesLayout).
//   decode      fused with the multi-device de-interleave: rank r's stream
//               holds the packed rows of its tiling (the interleave
//               {block_rows, r, nparts}, or any sdf_tiling per part);
//               every tile is expanded to RGBA32F (alpha 1) straight into its
//               rows of the assembled frame; a rendered stream's channels
//               are the pixels' shading terms, made into the colour here
//               exactly as the render kernel does (shade.h).  Lane j = pixel (j / 8, j % 8):
//               each lane loads its own base bits of each channel (stored
//               pixel by pixel, ABI 10), adds its escaped high bits, then
//               un-zigzag and the tile's 2-D inclusive prefix sum (DPP along
//               rows, ds_bpermute along columns) invert the gradient
//               predictor in uint32 arithmetic.
//
// All three move a few bytes per pixel; the decode writes 16 per pixel
// (RGBA32F); the decode is VALU-issue bound (TILES).
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "kernel_args.h"
// Exact-precision streams' specular term: 1 = the library fp64 pow alone
// (through round 4), 0 = shade.h's repeated squaring with the library pow
// only on lanes near a rounding boundary -- the same floats
#ifndef SDF_SHADE_LIBRARY_POW
#define SDF_SHADE_LIBRARY_POW 0
#endif
#include "shade.h"

namespace sdf {
namespace {

// Inclusive 2-D prefix sum (mod 2^32) over the 8 x 8 tile, lane = 8 row +
// col.  Rows: DPP row_shr by 1, 2, 4 inside the 16-lane DPP rows, the
// sources that would cross into the next 8-lane group zeroed first (shift 4
// masks whole banks instead).  Columns: ds_bpermute from lane - 8, - 16,
// - 32 (addresses `up`), the wrapped-around source rows zeroed first.
struct ScanLanes {
  uint32_t up8, up16, up32;
  bool c6, c5, r6, r5, r3;   // col <= 6, col <= 5, row <= 6, row <= 5, row <= 3
  __device__ __forceinline__ explicit ScanLanes(int lane)
      : up8(((lane - 8) & 63) << 2), up16(((lane - 16) & 63) << 2), up32(((lane - 32) & 63) << 2),
        c6((lane & 7) <= 6), c5((lane & 7) <= 5), r6((lane >> 3) <= 6), r5((lane >> 3) <= 5),
        r3((lane >> 3) <= 3) {}
};

__device__ __forceinline__ uint32_t scan_tile(uint32_t r, const ScanLanes& L) {
  r += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(L.c6 ? r : 0u), 0x111, 0xF, 0xF, true);
  r += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(L.c5 ? r : 0u), 0x112, 0xF, 0xF, true);
  r += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)r, 0x114, 0xF, 0xA, false);
  r += (uint32_t)__builtin_amdgcn_ds_bpermute((int)L.up8, (int)(L.r6 ? r : 0u));
  r += (uint32_t)__builtin_amdgcn_ds_bpermute((int)L.up16, (int)(L.r5 ? r : 0u));
  r += (uint32_t)__builtin_amdgcn_ds_bpermute((int)L.up32, (int)(L.r3 ? r : 0u));
  return r;
}

__device__ __forceinline__ uint32_t unordered_bits(uint32_t u) {
  return (u & 0x80000000u) ? (u ^ 0x7fffffffu) : u;
}

// tiles per wave of the decoder: 4 (0.051 ms for the root's 7/8 of a 4K
// frame) beats 2 (0.055); forcing 8 waves / SIMD spills and gains nothing.
// Round 4 (rank 0's 49/51 of the 4K C4 frame, profiles/r04_decode_ab.json):
// non-temporal frame stores 0.0445 against 0.0466 ms; one-wave workgroups
// 0.0470 (four kept); the column scan and the 16- and 8-bit transpose stages
// on the VALU (v_permlane16/32_swap, v_perm_b32, DPP row_ror) instead of
// ds_bpermute / ds_swizzle 0.0506 (not kept: the LDS round trips were not
// what bounds it, the extra VALU work and hazard waits are).
#ifndef SDF_DECODE_TILES
#define SDF_DECODE_TILES 4
#endif
#ifndef SDF_DECODE_WG_WAVES
#define SDF_DECODE_WG_WAVES 4   // waves per decoder workgroup
#endif
#ifndef SDF_DECODE_NT
#define SDF_DECODE_NT 1         // the frame's pixels by non-temporal stores
#endif
#ifndef SDF_DECODE_ESC_VMEM
#define SDF_DECODE_ESC_VMEM 0   // 1: a pixel's escape window by its own loads, not ds_bpermute
#endif
#ifndef SDF_DECODE_SKIP
#define SDF_DECODE_SKIP 0   // timing probes only (wrong pixels): 2 escapes, 4 scan, 8 shade
#endif
// The macros above are experiment knobs (tools/flag_variant.py, which
// defines SDF_EXPERIMENT); SKIP builds decode wrong pixels on purpose, and
// none of them enters sdf_kernel_id, so a library built with any of them
// away from its default must not pass for a product build.
#if !defined(SDF_EXPERIMENT) && (SDF_DECODE_SKIP != 0 || SDF_DECODE_ESC_VMEM != 0 || \
                                 SDF_DECODE_TILES != 4 || SDF_DECODE_WG_WAVES != 4 || \
                                 SDF_DECODE_NT != 1)
#error "decoder probe / layout knobs build only as experiments (tools/flag_variant.py)"
#endif
constexpr int kDecodeTiles = SDF_DECODE_TILES;
constexpr int kDecodeWgWaves = SDF_DECODE_WG_WAVES;

// One wave = TPW consecutive tiles of one part, lane j = pixel (j / 8, j % 8)
// of each.  The memory traffic is issued up front in two dependent rounds:
// the part header with the tiles' offsets and heads (one vector load each,
// lane i: tile i), then every tile's first 64 words (lane i: word i; the
// escapes' masks and bitstream are read from them).  Per tile: each lane's
// base bits (its own loads), escaped fields, un-zigzag, 2-D prefix sum,
// RGBA32F store into the tile's frame rows.
template <int TPW>
__device__ __forceinline__ void decode_body(const DecodeParts& D, const uint8_t* __restrict__ parts,
                                            int waves_per_part, float4* __restrict__ frame) {
  const int lane = threadIdx.x & 63;
  // the wave index as a scalar: from threadIdx.x the compiler cannot tell it
  // is wave-uniform and would run all tile / part arithmetic (divisions
  // included) on the VALU
  const int gw = blockIdx.x * kDecodeWgWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int part = gw / waves_per_part;
  if (part >= D.nparts) return;
  const int tbase = (gw - part * waves_per_part) * TPW;
  const int rows = D.rows[part], width = D.width;
  const int tiles_x = (width + 7) >> 3;
  const int ntiles = tiles_x * ((rows + 7) >> 3);
  if (tbase >= ntiles) return;
  const uint8_t* base = D.part_ptr[part] ? reinterpret_cast<const uint8_t*>(D.part_ptr[part])
                                         : parts + (long long)part * D.part_stride;
  const TilesLayout Lt(ntiles);
  const int nt = min(TPW, ntiles - tbase);
  // the header words are loaded with the tables (a part with ntiles = 0 holds
  // no tables, but they lie inside its pitch and are discarded)
  const uint32_t hused = reinterpret_cast<const uint32_t*>(base)[0];
  const uint32_t present = reinterpret_cast<const uint32_t*>(base)[1];
  const uint32_t offv = lane < nt ? reinterpret_cast<const uint32_t*>(base + Lt.table)[tbase + lane] : 0u;
  const uint4 hdv = lane < nt ? reinterpret_cast<const uint4*>(base + Lt.head)[tbase + lane]
                              : make_uint4(0u, 0u, 0u, 0u);
  const long long want = D.used[part];
  // a malformed part is reported and skipped: lane 0 stores 1 into the
  // cause's own byte of the part's word (a vector byte store), so the causes
  // found by different waves of one part combine without atomics
  auto report = [&](uint32_t code) {
    if (D.status && lane == 0)
      reinterpret_cast<uint8_t*>(D.status + part)[__builtin_ctz(code) >> 3] = 1;
  };
  if (present == 0) {   // no stream: rows rendered in place -- unless one was sent
    if (want >= 0) report(kTilesBadHeader);
    return;
  }
  // the stream's data bytes: what the ranks agreed on, within the part's
  // worst case (ntiles comes from the host's tiling, not from the stream)
  const uint32_t cap = (uint32_t)ntiles * (uint32_t)kTilePlaneBytes;
  if (present != (uint32_t)ntiles || hused > cap || (want >= 0 && (long long)hused != want)) {
    report(kTilesBadHeader);
    return;
  }
  // what the channels hold, and the frame's shading constants (header words
  // 2, 4..13: scalar loads)
  const uint32_t* const hw = reinterpret_cast<const uint32_t*>(base);
  const uint32_t shade = hw[2];
  ShadeK K;
#pragma unroll
  for (int c = 0; c < 3; c++) {
    K.lam[c] = __uint_as_float(hw[4 + c]);
    K.dif[c] = __uint_as_float(hw[7 + c]);
    K.ref[c] = __uint_as_float(hw[10 + c]);
  }
  K.shin = __uint_as_float(hw[13]);
  const uint2* data = reinterpret_cast<const uint2*>(base + Lt.data);
  uint2 pa[TPW];   // lane i: qword i of each tile's data (up to 64)
  // tile k's words lie in the stream's data, [off, off + 8 nq) within
  // [0, hused), and hold its base words and escape masks (B + P qwords) and,
  // when it escapes, the bitstream's first qword; each base width is at most
  // 32 (scalar checks; bit k of `good`).  Every later read of the tile
  // stays inside its nq qwords (the escape window is checked per lane).
  uint32_t good = 0u;
#pragma unroll
  for (int k = 0; k < TPW; k++) {
    const uint32_t head = (uint32_t)__builtin_amdgcn_readlane((int)hdv.x, k);
    const uint32_t off = __builtin_amdgcn_readlane((int)offv, k);
    const uint32_t nqk = tile_qwords(head);
    const uint32_t b0 = head & 63u, b1 = (head >> 6) & 63u, b2 = (head >> 12) & 63u;
    const uint32_t P = (uint32_t)__builtin_popcount((head >> 26) & 7u);
    const bool ok = k < nt && (off & 7u) == 0u && off <= hused && 8u * nqk <= hused - off &&
                    max(b0, max(b1, b2)) <= 32u && b0 + b1 + b2 + P + (P ? 1u : 0u) <= nqk;
    good |= (uint32_t)ok << k;
    const int nq = ok ? (int)nqk : 0;
    pa[k] = lane < nq ? data[off / 8 + lane] : make_uint2(0u, 0u);
  }
  if (good != (nt >= 32 ? ~0u : (1u << nt) - 1u)) report(kTilesBadTile);
  const ScanLanes SL(lane);
  const int col = lane & 7, prow = lane >> 3;
  // tile position, stepped per tile without divisions: tile column tx, tile
  // row ty, and the period `blk` of the part's tiling holding packed row
  // 8 ty at row `within` of its run of blocks (sdf_tiling)
  const int chunk = D.chunk_rows[part];
  const int first_blk = D.first_block[part], period = D.block_stride[part], brows = D.block_rows[part];
  const int gap = D.run_gap_rows[part];
  int ty = tbase / tiles_x, tx = tbase - ty * tiles_x;
  int blk = (8 * ty) / chunk, within = 8 * ty - blk * chunk;
  // spaced runs (gap > 0, block_rows % 8 == 0): the tile's block of its run
  // is jb, and its row in that block wb, stepped with `within`
  int jb = gap ? within / brows : 0, wb = within - jb * brows;
#pragma unroll
  for (int k = 0; k < TPW; k++) {
    if (k >= nt) continue;
    // (a malformed tile is skipped below, after the position step)
    if (k > 0 && ++tx == tiles_x) {
      tx = 0;
      ++ty;
      within += 8;
      wb += 8;
      if (wb >= brows) {
        wb -= brows;
        ++jb;
      }
      while (within >= chunk) {
        within -= chunk;
        ++blk;
        jb = 0;
        wb = within;
      }
    }
    if (!((good >> k) & 1u)) continue;
    const uint32_t head = __builtin_amdgcn_readlane((int)hdv.x, k);
    const int bw[3] = {(int)(head & 63), (int)((head >> 6) & 63), (int)((head >> 12) & 63)};
    const int nq = (int)tile_qwords(head);
    const uint32_t escaped = (head >> 26) & 7;
    const int B = bw[0] + bw[1] + bw[2];
    const uint2* tdata = data + __builtin_amdgcn_readlane((int)offv, k) / 8;
    // this pixel's base bits of each channel (lane-major: bw[c] words per
    // channel, pixel j's at bit j bw[c]): the two dwords holding them, by the
    // lane's own loads (no transpose; 0.0383 against 0.0407 ms with the bit
    // planes' 64 x 64 transpose, profiles/r04_decode_ab.json)
    uint32_t xb[3];
    {
      const uint32_t* t32 = reinterpret_cast<const uint32_t*>(tdata);
      uint32_t kb = 0u;
#pragma unroll
      for (int ch = 0; ch < 3; ch++) {
        const uint32_t w = (uint32_t)bw[ch];
        const uint32_t lbit = 64u * kb + (uint32_t)lane * w;
        // the second dword only where the bits reach it (never past the
        // channel's words: a stream may end there)
        const uint32_t d0 = lbit >> 5, d1 = (lbit & 31u) + w > 32u ? d0 + 1 : d0;
        xb[ch] = w ? __builtin_amdgcn_alignbit(t32[d1], t32[d0], lbit & 31u) & (0xFFFFFFFFu >> (32u - w))
                   : 0u;
        kb += w;
      }
    }
    const uint32_t first[3] = {(uint32_t)__builtin_amdgcn_readlane((int)hdv.y, k),
                               (uint32_t)__builtin_amdgcn_readlane((int)hdv.z, k),
                               (uint32_t)__builtin_amdgcn_readlane((int)hdv.w, k)};
    // the escapes: masks at qwords B.., then the field-width bytes and the
    // pixel-major fields, a bitstream from qword B + P (P escaped channels):
    // this pixel's fields (all its escaped channels) are one window of <= 36
    // bits at bit 8 P + sum_c d_c * (outliers of c below this pixel).  dl[c]:
    // this pixel's field bits in channel c (d_c for an outlier, else 0, by
    // one v_cndmask on the mask itself), so the fields are cut out of the
    // window by v_bfe at the running offset, without 64-bit shifts
    const int P = __builtin_popcount(escaped);
    uint32_t dl[3] = {0u, 0u, 0u}, f_lo = 0u, f_hi = 0u;
    if (!(SDF_DECODE_SKIP & 2) && escaped) {
      const int bs = 2 * (B + P);                       // bitstream's first dword
      const uint32_t deltas = bs < 128 ? (uint32_t)__builtin_amdgcn_readlane(
                                             (int)((bs & 1) ? pa[k].y : pa[k].x), bs >> 1)
                                       : reinterpret_cast<const uint32_t*>(tdata)[bs];
      uint32_t o = 8u * (uint32_t)P;
      int j = 0;
#pragma unroll
      for (int ch = 0; ch < 3; ch++) {
        if (!((escaped >> ch) & 1)) continue;
        const int mq = B + j;
        uint32_t mlo, mhi;
        if (mq < 64) {
          mlo = (uint32_t)__builtin_amdgcn_readlane((int)pa[k].x, mq);
          mhi = (uint32_t)__builtin_amdgcn_readlane((int)pa[k].y, mq);
        } else {
          const uint2 mm = tdata[mq];
          mlo = __builtin_amdgcn_readfirstlane(mm.x);
          mhi = __builtin_amdgcn_readfirstlane(mm.y);
        }
        const uint32_t d = (deltas >> (8 * j++)) & 255u;
        o += d * __builtin_amdgcn_mbcnt_hi(mhi, __builtin_amdgcn_mbcnt_lo(mlo, 0u));
        dl[ch] = __builtin_amdgcn_inverse_ballot_w64((uint64_t)mhi << 32 | mlo) ? d : 0u;
      }
      const uint32_t dw = (uint32_t)bs + (o >> 5);
      // this pixel's fields are bits [o, o + nb) of the bitstream: dwords dw
      // .. dw + (endbit - 1) / 32, which must lie in the tile's words
      // (malformed masks or widths could point past them: such a lane loads
      // nothing, the part is reported); a load is made only for a dword the
      // fields reach (the last tile's words may end the stream's buffer)
      const uint32_t nb = dl[0] + dl[1] + dl[2];
      const uint32_t endbit = (o & 31u) + nb;
      const bool inside = nb == 0u || dw + ((endbit - 1u) >> 5) < 2u * (uint32_t)nq;
      if (__builtin_amdgcn_ballot_w64(!inside)) report(kTilesBadField);
#if SDF_DECODE_ESC_VMEM
      // dwords dw .. dw + 2 of the tile's data, loaded by the lanes with fields
      uint32_t d0 = 0u, d1 = 0u, d2 = 0u;
      if (nb && inside) {
        const uint32_t* t32 = reinterpret_cast<const uint32_t*>(tdata);
        d0 = t32[dw];
        d1 = endbit > 32u ? t32[dw + 1] : 0u;
        d2 = endbit > 64u ? t32[dw + 2] : 0u;
      }
#else
      // dwords dw .. dw + 2 of the tile's data: qwords dw / 2 and dw / 2 + 1
      // from the lanes holding them
      const int a = (int)((dw >> 1) << 2);
      const uint32_t s0 = __builtin_amdgcn_ds_bpermute(a, (int)pa[k].x);
      const uint32_t s1 = __builtin_amdgcn_ds_bpermute(a, (int)pa[k].y);
      const uint32_t t0 = __builtin_amdgcn_ds_bpermute(a + 4, (int)pa[k].x);
      const uint32_t t1 = __builtin_amdgcn_ds_bpermute(a + 4, (int)pa[k].y);
      uint32_t d0 = (dw & 1) ? s1 : s0, d1 = (dw & 1) ? t0 : s1, d2 = (dw & 1) ? t1 : t0;
      if (nb && dw + 2 >= 128 && inside) {   // beyond the loaded qwords: rare
        const uint32_t* t32 = reinterpret_cast<const uint32_t*>(tdata);
        d0 = t32[dw];
        d1 = endbit > 32u ? t32[dw + 1] : 0u;
        d2 = endbit > 64u ? t32[dw + 2] : 0u;
      }
#endif
      f_lo = __builtin_amdgcn_alignbit(d1, d0, o & 31);
      f_hi = __builtin_amdgcn_alignbit(d2, d1, o & 31);
    }
    float v[3];
    uint32_t sh = 0u;   // this pixel's fields consumed so far (<= 24 bits)
#pragma unroll
    for (int ch = 0; ch < 3; ch++) {
      const int w = bw[ch];
      uint32_t z = xb[ch];
      if ((escaped >> ch) & 1) {   // this pixel's field (dl[ch] bits, 0 if none): bits w.. of z
        const uint32_t f = __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbit(f_hi, f_lo, sh), 0u, dl[ch]);
        z |= f << w;
        sh += dl[ch];
      }
      uint32_t r = (z >> 1) ^ (0u - (z & 1u));            // un-zigzag
      if (lane == 0) r = first[ch];                       // pixel 0 travels raw
      if constexpr (SDF_DECODE_SKIP & 4) v[ch] = __uint_as_float(r);
      else v[ch] = __uint_as_float(unordered_bits(scan_tile(r, SL)));
    }
    const int x = tx * 8 + col;
    if (x < width && ty * 8 + prow < rows) {
      // this lane's row: `prow` rows past (blk, within); a tile spans
      // several periods only when the run's rows are not a multiple of 8
      int b = blk, w = within + prow;
      while (w >= chunk) {
        w -= chunk;
        ++b;
      }
      const int y = (first_blk + b * period) * brows + w + jb * gap;
      float4 px = make_float4(v[0], v[1], v[2], 1.0f);
      if (SDF_DECODE_SKIP & 8) px = make_float4(v[0], v[1], v[2], 1.0f);
      else if (shade == kTilesShadeFast) px = shade_colour<false>(K, v[0], v[1], v[2]);
      else if (shade == kTilesShadeExact) px = shade_colour<true>(K, v[0], v[1], v[2]);
      if constexpr (SDF_DECODE_NT) {
        typedef float v4f __attribute__((ext_vector_type(4)));
        const v4f pv = {px.x, px.y, px.z, px.w};
        __builtin_nontemporal_store(pv, reinterpret_cast<v4f*>(frame + (size_t)y * width + x));
      } else {
        frame[(size_t)y * width + x] = px;
      }
    }
    (void)nq;
  }
}

__global__ __launch_bounds__(64 * kDecodeWgWaves) void decode_tiles(const DecodeParts D,
                                                    const uint8_t* __restrict__ parts,
                                                    int waves_per_part, float4* __restrict__ frame) {
  decode_body<kDecodeTiles>(D, parts, waves_per_part, frame);
}

// Offsets of the tiles' word blocks in tile order: exclusive scan of 8 * (w0 + w1
// + w2) over the heads.  tiles_scan: one wave x 32 consecutive tiles per lane
// per block of kScanTiles -> block-local offsets + the block's total.
// tiles_move: one wave per 8 consecutive tiles (in one scan block) adds the
// block's prefix (the sum of earlier block totals, a wave reduction), writes
// the final offsets and copies the tiles' words from their slots into the
// stream, the 8 tiles' loads in flight together (one wave per tile took
// 30.7 us on a whole 4K frame); the last tile writes `used`.  Both launch
// one-wave workgroups (round 4): they run beside the next frames' render
// kernels, whose one-wave workgroups fill the CUs, and a wave finds a free
// slot long before four waves on one CU do.
__device__ __forceinline__ uint32_t plane_bytes(uint32_t head) { return 8u * tile_qwords(head); }

constexpr int kScanLaneTiles = kScanTiles / 64;   // consecutive tiles per lane

__global__ __launch_bounds__(64) void tiles_scan(uint8_t* buf, int ntiles) {
  const TilesLayout L(ntiles);
  const uint4* head = reinterpret_cast<const uint4*>(buf + L.head);
  uint32_t* table = reinterpret_cast<uint32_t*>(buf + L.table);
  const int lane = threadIdx.x;
  const int t0 = blockIdx.x * kScanTiles + lane * kScanLaneTiles;
  uint32_t sz[kScanLaneTiles], sum = 0;
#pragma unroll
  for (int i = 0; i < kScanLaneTiles; i++) {
    sz[i] = t0 + i < ntiles ? plane_bytes(head[t0 + i].x) : 0u;
    sum += sz[i];
  }
  // exclusive scan of the lane sums
  uint32_t inc = sum;
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const uint32_t v = (uint32_t)__shfl_up((int)inc, s, 64);
    if (lane >= s) inc += v;
  }
  uint32_t off = inc - sum;
#pragma unroll
  for (int i = 0; i < kScanLaneTiles; i++) {
    if (t0 + i < ntiles) table[t0 + i] = off;
    off += sz[i];
  }
  if (lane == 63) reinterpret_cast<uint32_t*>(buf + L.bsums)[blockIdx.x] = inc;
}

constexpr int kMoveTiles = 8;   // tiles per wave of tiles_move (divides kScanTiles)

__global__ __launch_bounds__(64) void tiles_move(uint8_t* buf, int ntiles, uint32_t* used_out) {
  const TilesLayout L(ntiles);
  const int t0 = blockIdx.x * kMoveTiles;
  if (t0 >= ntiles) return;
  const int lane = threadIdx.x & 63;
  const int nt = min(kMoveTiles, ntiles - t0);
  const int blk = t0 / kScanTiles;   // all nt tiles lie in this scan block
  const uint32_t* bsums = reinterpret_cast<const uint32_t*>(buf + L.bsums);
  uint32_t pre = 0;
  for (int i = lane; i < blk; i += 64) pre += bsums[i];
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) pre += (uint32_t)__shfl_xor((int)pre, s);
  uint32_t* table = reinterpret_cast<uint32_t*>(buf + L.table);
  // lane k < nt: tile t0 + k's block-local offset and data bytes
  const uint32_t loc = lane < nt ? table[t0 + lane] : 0u;
  const uint32_t byt =
      lane < nt ? plane_bytes(reinterpret_cast<const uint4*>(buf + L.head)[t0 + lane].x) : 0u;
  const uint2* slots = reinterpret_cast<const uint2*>(buf + L.slots);
  uint2* data = reinterpret_cast<uint2*>(buf + L.data);
  constexpr int kQ = kTilePlaneBytes / 8;   // planes per slot
  // every tile's first 64 planes in flight at once (lane i: plane i)
  uint2 v[kMoveTiles];
#pragma unroll
  for (int k = 0; k < kMoveTiles; k++) {
    const int nq = (int)((uint32_t)__builtin_amdgcn_readlane((int)byt, k) >> 3);
    v[k] = lane < nq ? slots[(size_t)(t0 + k) * kQ + lane] : make_uint2(0u, 0u);
  }
#pragma unroll
  for (int k = 0; k < kMoveTiles; k++) {
    if (k >= nt) break;
    const int nq = (int)((uint32_t)__builtin_amdgcn_readlane((int)byt, k) >> 3);
    const uint32_t off = (uint32_t)__builtin_amdgcn_readlane((int)loc, k) + pre;
    if (lane < nq) data[off / 8 + lane] = v[k];
    if (nq > 64 && lane + 64 < nq)   // planes 64..95 (residuals over 21 bits on average): rare
      data[off / 8 + 64 + lane] = slots[(size_t)(t0 + k) * kQ + 64 + lane];
    if (lane == 0) {
      table[t0 + k] = off;
      if (t0 + k == ntiles - 1) {
        reinterpret_cast<uint32_t*>(buf)[0] = off + (uint32_t)nq * 8u;
        reinterpret_cast<uint32_t*>(buf)[1] = (uint32_t)ntiles;
        if (used_out) *used_out = off + (uint32_t)nq * 8u;
      }
    }
  }
}

}  // namespace

int launch_tiles_compact(void* stream_buf, int ntiles, void* stream, uint32_t* used_out) {
  if (ntiles <= 0) return 0;
  (void)hipGetLastError();  // a stale error of an earlier call is not this launch's
  uint8_t* buf = reinterpret_cast<uint8_t*>(stream_buf);
  hipLaunchKernelGGL(tiles_scan, dim3((ntiles + kScanTiles - 1) / kScanTiles), dim3(64), 0,
                     (hipStream_t)stream, buf, ntiles);
  const int waves = (ntiles + kMoveTiles - 1) / kMoveTiles;
  hipLaunchKernelGGL(tiles_move, dim3(waves), dim3(64), 0, (hipStream_t)stream, buf, ntiles,
                     used_out);
  return (int)hipGetLastError();
}

int launch_tiles_decode(const DecodeParts& d, void* frame, const void* parts, void* stream) {
  const int tiles_x = (d.width + 7) >> 3;
  int max_rows = 0;
  for (int r = 0; r < d.nparts; ++r) max_rows = max_rows > d.rows[r] ? max_rows : d.rows[r];
  const int tiles_per_part = tiles_x * ((max_rows + 7) >> 3);
  const int waves_per_part = (tiles_per_part + kDecodeTiles - 1) / kDecodeTiles;
  const long long waves = (long long)waves_per_part * d.nparts;
  if (waves == 0) return 0;
  (void)hipGetLastError();  // a stale error of an earlier call is not this launch's
  hipLaunchKernelGGL(decode_tiles, dim3((unsigned)((waves + kDecodeWgWaves - 1) / kDecodeWgWaves)),
                     dim3(64 * kDecodeWgWaves), 0,
                     (hipStream_t)stream, d, reinterpret_cast<const uint8_t*>(parts),
                     waves_per_part, reinterpret_cast<float4*>(frame));
  return (int)hipGetLastError();
}

}  // namespace sdf

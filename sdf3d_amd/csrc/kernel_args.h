// kernel_args.h -- uniform block handed from the C-ABI host code to the HIP
// render kernels.  Everything here is per-frame constant: the host hoists the
// shader's uniform-only work (inverse(V_mat) twice per pixel, camera.pos, the
// focal term -2/tan(fov*PI/360); voxel_fragment.frag:180, :191-192) so each
// lane only does per-pixel arithmetic.  Passed by value as the kernel argument
// so the fields are read with scalar loads (SGPRs), never per lane.
#pragma once

#ifndef __HIPCC_RTC__
#include <stddef.h>
#include <stdint.h>
#else
typedef __hip_internal::uint8_t uint8_t;
typedef __hip_internal::uint16_t uint16_t;
typedef __hip_internal::uint32_t uint32_t;
typedef __hip_internal::uint64_t uint64_t;
#endif

#include "../../include/sdf_abi.h"

namespace sdf {

constexpr int kMaxAoTaps = 64;

struct KernelArgs {
  // camera (hoisted uniforms)
  float inv_view[16];   // inverse(V_mat), column-major
  float cam[3];         // (inverse(V_mat) * vec4(camera.pos, 1)).xyz
  float focal;          // -2 / tan(fov * PI / 360)
  float aspect;         // AR
  // light + material (voxel_fragment.frag:182-189)
  float light_pos[3];
  float light_amb;
  float mat_amb[3];
  float mat_dif[3];
  float mat_ref[3];
  float shininess;
  // march parameters
  int32_t width, height;
  int32_t max_steps;
  float max_dist, eps, shadow_k, normal_eps, shadow_offset;
  int32_t flags, normal_mode, format;
  int32_t ao_taps;
  float ao_step, ao_base, ao_falloff, ao_strength;
  float ao_h[kMaxAoTaps];  // tap heights base + step * i / (taps - 1), host fp32
  float ao_path[kMaxAoTaps];  // path length P -> tap 0 -> .. -> tap i (fp64, rounded up)
  float inv_width, inv_height;  // fast precision quad mapping
  // tiling
  int32_t block_rows, first_block, block_stride, rows;
  int32_t chunk_rows;   // block_rows * run: rows of one period's run of blocks
  int32_t run_gap_rows; // (run_step - 1) * block_rows: rows skipped between a run's blocks
  int32_t frame_rows;   // SDF_TILING_FRAME_ROWS: output row = frame row y
  // scene
  int32_t scene_kind, prim_count;
  float bulb_center[3], bulb_scale, bulb_inv_scale, bulb_bail2;
  int32_t bulb_iterations;
  // prepared primitives (sdf_abi.cpp prepare_prims): kind, op, k,
  // reserved = 1/k, p = per-kind parameter block (see render_kernel.inc)
  sdf_primitive prims[SDF_MAX_PRIMS];
  // culling bounds (fixed-scene kernels): per primitive {centre.xyz, K} with
  // K = k + R + margin, R the radius of a sphere containing the primitive;
  // and the same for the cluster of primitives [cluster_first, count)
  alignas(16) float bound[SDF_MAX_PRIMS][4];   // 16-B aligned: read as float4 vector loads
  alignas(16) float cluster[4];
  int32_t cluster_first;
  // outputs
  void* rgba;           // rows * width pixels of `format`, packed rows
  int32_t* steps;       // rows * width int2 or null
};

// ---- dispatch order of a frame's 8-row blocks (sdf_render_scheduled) -------
// The render grid's row of workgroups blockIdx.y renders packed 8-row block
// order[blockIdx.y] (n > 0; launch order otherwise): a schedule puts the
// blocks that cost most in earlier frames first, so the frame's longest tiles
// do not run alone at its end.  The table rides in the kernel-argument
// segment (never a buffer another frame may be rewriting): any permutation
// renders every block exactly once.  `cost` (may be null): each wave adds the
// shader-clock cycles it took to its block's word.
constexpr int kMaxOrderBlocks = 512;   // 4096 packed rows
struct RowOrder {
  unsigned long long* cost;
  int32_t n;
  int32_t reserved;
  uint16_t order[kMaxOrderBlocks];
};
struct RenderArgs {
  KernelArgs a;   // first: the kernels read it at the start of the segment
  RowOrder o;
};

// Waves (8x8 tiles side by side) per render workgroup (render_kernel.inc
// render / render_tiles; the built-in and the run-time specialised launchers).
// Round 4: one wave per workgroup -- each wave is placed on its own, so the
// frame's last, longest tiles pack onto the CUs better than in 4-wave groups
// that need four slots of one CU: C4 fast 0-1.6 % faster, C5 fast up to 4 %,
// C4/C5 exact 0.2-1.8 % (profiles/r04_ab_workgroup.json; 2 waves lie between,
// 8 are 3-5 % slower).  Overridable for experiments (SDF_WG_WAVES).
#ifndef SDF_WG_WAVES
#define SDF_WG_WAVES 1
#endif
constexpr int kWgWaves = SDF_WG_WAVES;

// ---- frame sequences (sdf_render_frames) ----------------------------------
// Up to kFramesPerLaunch whole frames of one scene in one launch of a
// persistent kernel: its waves take 8x8 tiles of all the launch's frames from
// one work counter, frame after frame, so a frame's slowest tiles overlap the
// next frame's first ones instead of ending a launch.  The per-frame uniforms
// ride in the kernel-argument segment beside the shared KernelArgs (whose own
// camera and output fields are unused): sizeof(KernelArgs) + 16 x 104 bytes,
// checked below against the 4 KiB explicit kernel-argument limit.
constexpr int kFramesPerLaunch = 16;
struct FrameCam {
  float inv_view[16];   // inverse(V_mat) of this frame's camera
  float cam[3];
  float focal, aspect;
  void* rgba;           // width * height pixels of the params' format
  int32_t* steps;       // width * height int2 or null
};
struct FramesArgs {
  KernelArgs a;
  FrameCam frame[kFramesPerLaunch];
  int32_t nframes;          // 1 .. kFramesPerLaunch
  int32_t tiles_x;          // ceil(width / 8)
  int32_t tiles_per_frame;  // tiles_x * ceil(height / 8)
  int32_t queues;           // work queues (1 .. kFrameQueues, <= workgroups)
  int32_t schedule;         // 0 work queues, 1 static (tools/frames_probe.py)
  int32_t chunk;            // tiles per queue request (kChunkTiles)
  uint32_t* counter;        // queue q's counter at counter[q * kQueueStride], zero at launch
};
// the by-value kernel argument must fit the 4 KiB kernarg limit:
// raising kMaxAoTaps, SDF_MAX_PRIMS or kFramesPerLaunch fails here, not at launch
static_assert(sizeof(FramesArgs) <= 4096, "FramesArgs exceeds the 4 KiB kernel-argument limit");
static_assert(sizeof(KernelArgs) <= 4096, "KernelArgs exceeds the 4 KiB kernel-argument limit");
static_assert(sizeof(RenderArgs) <= 4096, "RenderArgs exceeds the 4 KiB kernel-argument limit");
// Tiles a wave takes per queue request, queues per launch (workgroup b uses
// queue b % queues, i.e. one per XCD), and the queues' spacing in uint32s:
// requests on one address serialise at the memory-side atomic unit, so the
// launch spreads them over several addresses.  One tile per request since
// round 6: the same rate on 16-frame launches (r02 sweep: 0.3665 against
// 0.3663 ms per frame with 2), and a ONE-frame launch 0.384 -> 0.237 ms on
// C3 exact, where larger requests leave waves without tiles (a 1080p frame
// has ~4 tiles per wave; profiles/r06_frames1_env.jsonl).
constexpr int kChunkTiles = 1;
constexpr int kFrameQueues = 32;   // at most; kDefaultQueues by default
constexpr int kDefaultQueues = 8;
constexpr int kQueueStride = 64;

// Kernel launchers, one per precision translation unit (render_exact.hip /
// render_fast.hip); `variant` selects a compile-time scene specialisation
// (see render_kernel.inc).  Return a hipError_t as int.
int launch_render_exact(const RenderArgs& a, int variant, void* stream);
int launch_render_fast(const RenderArgs& a, int variant, void* stream);
// the persistent frame-sequence kernel on `nblocks` 256-thread workgroups
int launch_frames_exact(const FramesArgs& a, int variant, int nblocks, void* stream);
int launch_frames_fast(const FramesArgs& a, int variant, int nblocks, void* stream);
// the Mandelbulb scene's kernels live in units of their own
// (render_{fast,exact}_bulb.hip, scheduled for ILP: sdf3d_amd/build.py); the
// launchers above forward kVariantBulb to these
int launch_render_exact_bulb(const RenderArgs& a, void* stream);
int launch_render_fast_bulb(const RenderArgs& a, void* stream);
int launch_frames_exact_bulb(const FramesArgs& a, int nblocks, void* stream);
int launch_frames_fast_bulb(const FramesArgs& a, int nblocks, void* stream);
int launch_deinterleave(const void* parts, int nparts, int part_stride_rows, int row_bytes,
                        int height, int block_rows, void* frame, void* stream);
int launch_heatmap(const int32_t* steps, int count, int which, int max_steps, int format,
                   void* out, void* stream);
int launch_deinterleave_rgb(const void* parts, int nparts, int part_stride_rows, int width,
                            int height, int block_rows, void* frame, void* stream);
// TILES decode of parts with their own tilings (sdf_tiles_decode_tilings)
struct DecodeParts {
  int nparts, width, height;
  long long part_stride;
  int rows[SDF_MAX_DECODE_PARTS], first_block[SDF_MAX_DECODE_PARTS],
      block_stride[SDF_MAX_DECODE_PARTS], block_rows[SDF_MAX_DECODE_PARTS],
      chunk_rows[SDF_MAX_DECODE_PARTS], run_gap_rows[SDF_MAX_DECODE_PARTS];
  // part r's stream at part_ptr[r] when non-null (another device's memory,
  // peer-mapped: sdf_render_multi), else at parts + r * part_stride
  const void* part_ptr[SDF_MAX_DECODE_PARTS];
  // A stream is untrusted input (it crossed RCCL): the decoder reads nothing
  // outside the part's worst-case stream.  used[r] >= 0: the data bytes part
  // r must hold (the length the ranks agreed on; its header word 0 must say
  // the same); -1: the header's word 0, at most the part's capacity.
  long long used[SDF_MAX_DECODE_PARTS];
  // device-writable, nparts words (may be null): word r is set to a nonzero
  // kTilesBad* code when part r is malformed (the decoder then skips the
  // part, or the tiles that are out of bounds, and writes nothing for them)
  uint32_t* status;
  // everything zero, no expected lengths (used = -1), no status words
  __host__ DecodeParts() {
    __builtin_memset(this, 0, sizeof(*this));
    for (int r = 0; r < SDF_MAX_DECODE_PARTS; ++r) used[r] = -1;
  }
};
// (sdf_abi.h SDF_TILES_BAD_*)
constexpr uint32_t kTilesBadHeader = SDF_TILES_BAD_HEADER;   // length / tile count disagree
constexpr uint32_t kTilesBadTile = SDF_TILES_BAD_TILE;       // a tile's offset, size or widths
constexpr uint32_t kTilesBadField = SDF_TILES_BAD_FIELD;     // an escape field past its tile
int launch_tiles_decode(const DecodeParts& d, void* frame, const void* parts, void* stream);

// ---- TILES stream buffer (sdf_abi.h SDF_FORMAT_TILES) ----------------------
// The buffer handed to sdf_render holds the stream (header, offset table,
// per-tile heads, worst-case plane data) followed by the encoder's scratch:
// per-block plane-byte totals of the offset scan and fixed worst-case plane
// slots.  sdf_tiles_bytes() = end.
constexpr int kTilePlaneBytes = 8 * 96;   // 3 channels x 32 planes
constexpr int kScanTiles = 2048;          // tiles per block of the offset scan
constexpr int kTilesHeaderBytes = 64;     // used, ntiles, shade mode, 0, ShadeK, 0, 0
struct TilesLayout {
  size_t table, head, data, stream_end, bsums, slots, end;
  __host__ __device__ explicit TilesLayout(long long ntiles) {
    const size_t n = (size_t)ntiles;
    const size_t nb = (n + kScanTiles - 1) / kScanTiles;
    table = kTilesHeaderBytes;
    head = (kTilesHeaderBytes + 4 * n + 15) & ~(size_t)15;
    data = head + 16 * n;
    stream_end = data + n * kTilePlaneBytes;
    bsums = (stream_end + 15) & ~(size_t)15;
    slots = (bsums + 4 * nb + 15) & ~(size_t)15;
    end = slots + n * kTilePlaneBytes;
  }
};
// `used_out` (may be null): a device word that also receives the stream's
// length (header word 0), e.g. one slot of the frame driver's lengths array
// whose slots of consecutive frames are all-gathered in one call.
int launch_tiles_compact(void* stream_buf, int ntiles, void* stream, uint32_t* used_out = nullptr);
// A tile's head word 0 (sdf_abi.h SDF_FORMAT_TILES): base widths b0 | b1 << 6
// | b2 << 12, the tile's data in qwords << 18, escaped channels << 26.
__host__ __device__ inline uint32_t tile_qwords(uint32_t head) { return (head >> 18) & 255u; }
constexpr int kEscapeWindow = 12;   // base widths tried below the widest residual
constexpr int kEscapeDwords = 72;   // bitstream bound: 3 width bytes + 3 x 12 x 63 bits
// run-time specialised kernel for a scene signature (jit.cpp); -1 = none
int launch_render_jit(const RenderArgs& a, const int* sig, int n, bool exact, void* stream);
int jit_compiled_count();

// ---- compile-time scene variants ------------------------------------------
// A variant fixes the (kind, op) sequence of the primitive list at compile
// time; parameter values stay runtime uniforms.  The host picks the variant
// whose signature equals the scene's (select_variant, sdf_abi.cpp); anything
// else runs the generic kernel, which reads kinds and ops at run time.

// Internal primitive kind: a PLANE whose normal is exactly (0,1,0), evaluated
// as p.y + h -- the reference's planeSDF (voxel_fragment.frag:68) when h = 0.
constexpr int kPrimPlaneY = 7;
#define SDF_KO(kind, op) ((kind) * 8 + (op))

// X(variant id, signature...)
#define SDF_FIXED_VARIANTS(X)                                                        \
  /* reference scene: min(min(INF, plane), sphere), voxel_fragment.frag:73-81 */   \
  X(1, SDF_KO(kPrimPlaneY, SDF_OP_UNION), SDF_KO(SDF_PRIM_SPHERE, SDF_OP_UNION))    \
  /* C1: single sphere */                                                          \
  X(2, SDF_KO(SDF_PRIM_SPHERE, SDF_OP_UNION))                                      \
  /* C3/C4: 8-primitive smooth-min CSG (sdf3d_amd/scenes.py set_csg8) */           \
  X(3, SDF_KO(kPrimPlaneY, SDF_OP_UNION), SDF_KO(SDF_PRIM_SPHERE, SDF_OP_SMOOTH_UNION), \
    SDF_KO(SDF_PRIM_BOX, SDF_OP_SMOOTH_UNION), SDF_KO(SDF_PRIM_TORUS, SDF_OP_SMOOTH_UNION), \
    SDF_KO(SDF_PRIM_CAPSULE, SDF_OP_SMOOTH_UNION),                                 \
    SDF_KO(SDF_PRIM_CYLINDER, SDF_OP_SMOOTH_UNION),                                \
    SDF_KO(SDF_PRIM_ROUND_BOX, SDF_OP_SMOOTH_UNION),                               \
    SDF_KO(SDF_PRIM_SPHERE, SDF_OP_SMOOTH_UNION))

// ---- exact bounding-volume culling -----------------------------------------
// For op UNION, min(d, s) == d whenever s >= d; for SMOOTH_UNION,
// smin(d, s, k) == d bit for bit whenever s >= d + k (h = 0).  Every SDF here
// is exact, so s >= |p - c| - R for a sphere (c, R) containing the primitive.
// A primitive can therefore be skipped -- without changing any output bit --
// at points where |p - c| * (1 - kCullRel) >= d + k + R + kCullAbs; the
// margins cover fp32 rounding of s and of the bound.  A plane is unbounded;
// a hard-union sphere costs no more than its own bound.
constexpr float kCullAbs = 1e-4f;
constexpr float kCullRel = 1e-5f;
constexpr float kCullScale = 1.0f / (1.0f - kCullRel);
// path lengths used by cached bounds are scaled up by this factor so that
// unit directions normalised in fp32 (|dir| <= 1 + 2^-22) stay conservative
constexpr float kPathScale = 1.000002f;
constexpr bool cullable(int kind, int op) {
  return kind != SDF_PRIM_PLANE && kind != kPrimPlaneY &&
         (op == SDF_OP_SMOOTH_UNION || (op == SDF_OP_UNION && kind != SDF_PRIM_SPHERE));
}

enum SceneVariant : int {
  kVariantGeneric = 0,
  kVariantBulb = 100,
};

// Variant for a validated scene (kVariantGeneric when no fixed one matches).
int select_variant(const sdf_scene& scene);
int scene_signature(const sdf_scene& scene, int* sig);

}  // namespace sdf

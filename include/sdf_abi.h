/*
 * sdf_abi.h -- C-ABI of the MI355X-native SDF sphere-tracing renderer.
 *
 * This is the drop-in boundary that replaces the reference's device programs
 * (ezorzin/SDF3D `Code/shader/voxel_fragment.frag`, `voxel_geometry.geom`,
 * `voxel_vertex.vert` and the never-enqueued `Code/kernel/thekernel_1.cl`).
 * Plain C: POD structs, plain pointers and sizes, integer status codes.  No
 * torch / C++ types cross this boundary.
 *
 * Reference interface each entry point replaces (paths relative to the
 * reference root):
 *
 *   sdf_defaults()   the hard-coded constants and scene of the fragment shader:
 *                    voxel_fragment.frag:15-23 (PI, MAX_STEPS, MAX_DISTANCE,
 *                    EPSILON), :54-81 (sphere + plane, hard union), :178-189
 *                    (camera, light, material), :205 (shadow k = 10); and the
 *                    host's default window / view (main.cpp:4-11: 800x600,
 *                    orbit and pan at 0 -> V_mat = identity).
 *   sdf_render()     one frame of `gl->plot(sh, proj_mode)` (main.cpp:95), i.e.
 *                    the fragment stage `main()` (voxel_fragment.frag:160-211)
 *                    run once per pixel, with the pixel -> `quad` mapping of
 *                    voxel_geometry.geom:26-52 folded into the index math, and
 *                    with the uniforms `V_mat`, `AR` (voxel_fragment.frag:5-7)
 *                    passed explicitly in sdf_camera.  The output is the
 *                    shader's `fragment_color` (:12, :210) as float RGBA.
 *   sdf_deinterleave() gathers per-device row blocks into one frame (new: the
 *                    reference has a single GL context, main.cpp:48,53).
 *   sdf_driver_*()   the multi-device frame loop: the reference's per-frame
 *                    `gl->plot` loop (main.cpp:87-98) run across the GPUs of
 *                    one node, every rank rendering its row blocks and rank 0
 *                    assembling the frame over RCCL (new: the reference has a
 *                    single GL context, main.cpp:48,53).
 *   sdf_strerror()   error text (the reference has none: main.cpp:109).
 *
 * Conventions
 *   - Framebuffer: width x height pixels, 4 floats (R,G,B,A) per pixel,
 *     row-major, row 0 = BOTTOM row (GL window origin), pixel (x, y) at
 *     rgba[(y * width + x) * 4].
 *   - Matrices: 16 floats, column-major, exactly like a GLSL mat4 uniform.
 *   - All device pointers are HIP device pointers on the current device; the
 *     call is asynchronous on `stream` (a hipStream_t, NULL = null stream).
 *   - Functions return SDF_OK (0) or a negative SDF_E* code; they never throw.
 */
#ifndef SDF_ABI_H
#define SDF_ABI_H

#ifndef __HIPCC_RTC__
#include <stdint.h>
#else
/* compiled at run time by hipRTC (the library's kernel specialiser) */
typedef __hip_internal::int32_t int32_t;
typedef __hip_internal::int64_t int64_t;
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define SDF_ABI_VERSION 11  /* 7: sdf_comm_create timeout, sdf_render_multi;
                                8: sdf_render_frames;
                                9: TILES carries shading terms (64-byte
                                   stream header), SDF_FORMAT_SHADE32F;
                                10: sdf_driver_config.batch (frames per
                                   ship); TILES base bits pixel by pixel
                                   (lane-major) instead of bit planes;
                                11: sdf_schedule_*, sdf_render_scheduled,
                                   sdf_tiles_decode_checked (SDF_TILES_BAD_*
                                   one byte each), sdf_validate bounds every
                                   length to 1e15 */

/* ---- status codes ------------------------------------------------------ */
#define SDF_OK               0
#define SDF_E_INVALID_ARG   -1  /* null pointer, bad size, bad enum value      */
#define SDF_E_UNSUPPORTED   -2  /* valid request this build cannot serve       */
#define SDF_E_HIP           -3  /* a HIP runtime call failed                   */
#define SDF_E_NO_DEVICE     -4  /* no gfx950 device visible                    */
#define SDF_E_COMM          -5  /* RCCL could not be loaded or a collective failed */
#define SDF_E_TIMEOUT       -6  /* the frame driver waited longer than its limit */

/* ---- scene description -------------------------------------------------- */
#define SDF_MAX_PRIMS 16

/* Primitive kinds.  Parameter layout in sdf_primitive.p[]:
 *   SPHERE     c.xyz, radius                       (voxel_fragment.frag:54-64)
 *   PLANE      n.xyz, h        sdf = dot(p, n) + h   (voxel_fragment.frag:66-71
 *                              is n = (0,1,0), h = 0: sdf = p.y)
 *   BOX        c.xyz, half.xyz                     (extension, parity unpinned)
 *   ROUND_BOX  c.xyz, half.xyz, r                  (extension)
 *   TORUS      c.xyz, R, r     ring in the xz plane (extension)
 *   CAPSULE    a.xyz, b.xyz, r                     (extension)
 *   CYLINDER   c.xyz, r, half_height, y-axis, capped (extension)            */
typedef enum {
  SDF_PRIM_SPHERE = 0,
  SDF_PRIM_PLANE = 1,
  SDF_PRIM_BOX = 2,
  SDF_PRIM_ROUND_BOX = 3,
  SDF_PRIM_TORUS = 4,
  SDF_PRIM_CAPSULE = 5,
  SDF_PRIM_CYLINDER = 6,
  SDF_PRIM_KIND_COUNT = 7
} sdf_prim_kind;

/* How primitive i combines with the running scene distance d (d starts at
 * +INF, voxel_fragment.frag:75).  UNION is GLSL `min(d, s)` exactly as
 * voxel_fragment.frag:77-78; the smooth forms use the polynomial smooth-min
 * with blend radius `k` (extension, see DESIGN.md "Scene spec").            */
typedef enum {
  SDF_OP_UNION = 0,
  SDF_OP_SMOOTH_UNION = 1,
  SDF_OP_SUBTRACT = 2,         /* max(d, -s)                                  */
  SDF_OP_INTERSECT = 3,        /* max(d, s)                                   */
  SDF_OP_SMOOTH_SUBTRACT = 4,
  SDF_OP_SMOOTH_INTERSECT = 5,
  SDF_OP_COUNT = 6
} sdf_csg_op;

typedef struct {
  int32_t kind;   /* sdf_prim_kind */
  int32_t op;     /* sdf_csg_op    */
  float k;        /* smooth blend radius (> 0 for SMOOTH_* ops)               */
  float reserved;
  float p[12];    /* kind-specific parameters, see above                      */
} sdf_primitive;  /* 64 bytes */

typedef enum {
  SDF_SCENE_PRIMITIVES = 0,    /* CSG list of prims[0..count)                 */
  SDF_SCENE_MANDELBULB = 1     /* power-8 Mandelbulb distance estimator        */
} sdf_scene_kind;

typedef struct {
  int32_t kind;                /* sdf_scene_kind                               */
  int32_t count;               /* number of primitives used (PRIMITIVES)       */
  sdf_primitive prims[SDF_MAX_PRIMS];
  /* MANDELBULB: world p -> local q = (p - center) / scale, DE(q) * scale.   */
  float bulb_center[3];
  float bulb_scale;
  int32_t bulb_iterations;     /* default 12                                   */
  float bulb_bailout;          /* default 2; (0, 2^32]                         */
  int32_t reserved[2];
} sdf_scene;

/* Camera: voxel_fragment.frag:26-30, :178-180, :191-192.                    */
typedef struct {
  float view[16];              /* V_mat uniform, column-major                  */
  float eye[3];                /* camera.pos before inverse(V_mat): (0,0.2,2)  */
  float fov_deg;               /* camera.fov = 60                              */
  float aspect;                /* AR uniform; <= 0 means width / height        */
  float pi;                    /* the shader's PI literal 3.1415925359f (a1)   */
} sdf_camera;

/* Light: voxel_fragment.frag:32-40, :182-184.                               */
typedef struct {
  float pos[3];                /* (5, 5, 0)                                    */
  float ambient;               /* light.amb = 0.1                              */
  float color[3];              /* light.col = 0.7: declared, never used (:183) */
  float reserved;
} sdf_light;

/* Material: voxel_fragment.frag:42-49, :186-189.                            */
typedef struct {
  float amb[3];                /* (0, 0.2, 0.8)                                */
  float dif[3];                /* (0, 0.2, 0.8)                                */
  float ref[3];                /* (0.5, 0.5, 0.5)                              */
  float shininess;             /* 12                                           */
} sdf_material;

/* Render flags */
#define SDF_FLAG_SHADOW     0x1  /* soft shadow march (voxel_fragment.frag:205) */
#define SDF_FLAG_AO         0x2  /* ambient occlusion (extension)               */

typedef enum {
  SDF_NORMAL_CENTRAL = 0,      /* 6-tap central differences (:134-155)         */
  SDF_NORMAL_TETRA = 1         /* 4-tap tetrahedral differences (extension)    */
} sdf_normal_mode;

typedef enum {
  SDF_PRECISION_EXACT = 0,     /* IEEE div/sqrt, no FMA contraction: bit-level
                                  restatement of the shader arithmetic         */
  SDF_PRECISION_FAST = 1       /* hardware sqrt/rcp, FMA contraction           */
} sdf_precision;

typedef struct {
  int32_t width, height;       /* framebuffer size (main.cpp:4-5: 800 x 600)   */
  int32_t max_steps;           /* MAX_STEPS = 100 (both marches, :17)          */
  float max_dist;              /* MAX_DISTANCE = 100 (:18)                     */
  float eps;                   /* EPSILON = 0.01 (:19)                         */
  float shadow_k;              /* 10 (:205)                                    */
  float normal_eps;            /* DX/DY/DZ offset = EPSILON (:21-23)           */
  float shadow_offset;         /* P + N*2*EPSILON: 2 (:205)                    */
  int32_t flags;               /* SDF_FLAG_*; reference = SDF_FLAG_SHADOW      */
  int32_t normal_mode;         /* sdf_normal_mode; reference = CENTRAL          */
  int32_t ao_taps;             /* AO samples (5 when SDF_FLAG_AO)              */
  float ao_step;               /* AO: h_i = ao_base + ao_step * i / (taps-1)   */
  float ao_base;
  float ao_falloff;            /* per-tap weight decay                         */
  float ao_strength;           /* ao = clamp(1 - strength * occ, 0, 1)         */
  int32_t precision;           /* sdf_precision                                */
  int32_t dispatch;            /* sdf_dispatch (AUTO: compile-time scene
                                  variant when one matches the scene)         */
  int32_t output_format;       /* sdf_format of the framebuffer written       */
  int32_t reserved[2];
} sdf_params;

/* Framebuffer element formats (4 channels R,G,B,A per pixel).
 *   RGBA32F  the shader's float fragment_color (voxel_fragment.frag:12,210).
 *   RGBA16F  IEEE half, round to nearest even.
 *   RGBA8    what the reference's RGBA8 window shows (main.cpp:95-96):
 *            u8 = trunc(min(max(c, 0), 1) * 255 + 0.5), NaN -> 0, no
 *            multiply-add fusion.
 *   RGB32F   RGBA32F without the alpha channel, which the shader always
 *            writes as 1.0 (voxel_fragment.frag:210): a lossless 12-byte
 *            wire format for multi-device frames; sdf_deinterleave expands
 *            it to an RGBA32F frame with alpha = 1.
 *   SHADE32F the pixel's three shading terms instead of its colour, as
 *            RGBA32F (ao, dif, x, 1): ao the AO factor (1 without AO), dif =
 *            clamp(N.L, 0, 1) * shadow, x = max(N.H, 0); the colour is
 *            la * amb * ao + dif * mat.dif + pow(x, shininess) * mat.ref
 *            (voxel_fragment.frag:204-210) in the precision's fixed operation
 *            sequence (sdf3d_amd/csrc/shade.h).  Diagnostics: what TILES
 *            streams carry.
 *   TILES    the frame losslessly compressed for the multi-device gather
 *            (about 2.3 instead of 12 bytes per pixel on the 4K CSG scene),
 *            decoded bit for bit by sdf_tiles_decode.  A rendered stream
 *            carries the SHADE32F terms in its three channels (smoother than
 *            the colour, which mixes them: 29 % fewer bytes) and the frame's
 *            shading constants in its header; the decoder makes the colour
 *            from them exactly as sdf_render does.  The rendered (packed) rows
 *            are cut into 8x8 tiles, tile t = ty * ceil(width / 8) + tx
 *            covering packed rows 8ty.. and columns 8tx..; pixel j = 8 *
 *            row + column of a tile.  Per tile and channel: the float bits
 *            mapped to ordered integers u (bits ^ 0x7fffffff when the sign
 *            is set, an involution; u = 0 outside the frame), the gradient
 *            residual u - left - up + upleft (neighbours outside the tile
 *            are 0; mod 2^32; its inverse is the tile's 2-D prefix sum),
 *            zigzag-coded to z, with z := 0 for pixel 0 (it travels raw) and
 *            for pixels outside the frame.  Per channel c the tile stores
 *            the low b[c] bits of every z_j, pixel by pixel: b[c] u64 words
 *            whose bits j b[c] .. j b[c] + b[c] - 1 are z_j's (ABI 10; bit
 *            planes before), and, when its widest z has w > b[c] bits, an
 *            escape: a u64 mask of the outlier pixels (z_j >= 2^b[c]), a
 *            width byte d = w - b[c]
 *            and each outlier's bits b[c].. as a d-bit field.  The encoder
 *            picks b[c] among w, w - 1, .., w - 12 by the smallest size
 *            (64 b + 72 + d * outliers bits; ties: larger b).
 *            Stream layout (little-endian; sdf_tiles_bytes() sizes the
 *            buffer, stream plus the encoder's scratch):
 *              u32 used             bytes of tile data
 *              u32 ntiles
 *              u32 shade            0: the channels are RGB (a stream not
 *                                   made by sdf_render); 1 / 2: shading
 *                                   terms of a fast / exact render
 *              u32 0
 *              f32 lam[3]           light.ambient * material.amb[c] (fp32)
 *              f32 dif[3], ref[3]   material.dif, material.ref
 *              f32 shininess
 *              u32 0, 0
 *              u32 offset[ntiles]   (at byte 64) tile t's data at data +
 *                                   offset[t]
 *              head = stream + align16(64 + 4 * ntiles):
 *                u32x4 head[ntiles] {b0 | b1 << 6 | b2 << 12 | q << 18 |
 *                                   e << 26, first[3]}: q the tile's data
 *                                   in u64 words, e bit c set when channel
 *                                   c is escaped (P = popcount(e)),
 *                                   first[c] u of pixel 0
 *              data = head + 16 * ntiles, per tile q u64 words:
 *                                   b0 + b1 + b2 words of base bits,
 *                                   channel by channel; the P masks of the escaped
 *                                   channels; then one bitstream (LSB
 *                                   first, zero-padded to whole words):
 *                                   the P width bytes, then the fields
 *                                   pixel by pixel, each pixel's fields of
 *                                   the channels it is an outlier of in
 *                                   channel order
 *            The meaningful prefix of a stream is data + used bytes; tile
 *            blocks appear in tile order (tests/tiles_ref.py states the
 *            codec in NumPy).                                             */
typedef enum {
  SDF_FORMAT_RGBA32F = 0,
  SDF_FORMAT_RGBA16F = 1,
  SDF_FORMAT_RGBA8 = 2,
  SDF_FORMAT_RGB32F = 3,
  SDF_FORMAT_TILES = 4,
  SDF_FORMAT_SHADE32F = 5
} sdf_format;

typedef enum {
  SDF_DISPATCH_AUTO = 0,       /* specialised kernel: a built-in one when the
                                  scene matches, else one compiled at run time
                                  for the scene's (kind, op) sequence (hipRTC,
                                  ~0.7 s once per sequence and process; off
                                  with SDF3D_JIT=0), else the generic kernel  */
  SDF_DISPATCH_GENERIC = 1,    /* always the generic primitive-list kernel     */
  SDF_DISPATCH_UNCULLED = 2    /* generic kernel evaluating every primitive at
                                  every point (no bounding-volume culling): the
                                  straight restatement, for cross-checks       */
} sdf_dispatch;

/* Which rows of the frame a call renders.  Rows are grouped into blocks of
 * `block_rows` rows; block b (rows [b*block_rows, (b+1)*block_rows)) is
 * rendered iff b >= first_block and, with o = (b - first_block) %
 * block_stride, o % step == 0 and o / step < run: run = max(block_run, 1)
 * blocks per period of `block_stride` blocks, step = max(run_step, 1) blocks
 * apart (step 1: consecutive).  Rendered rows are written densely ("packed")
 * in increasing y order, so {block_rows = 8, first_block = r, block_stride =
 * N} is device r's share of an N-device interleaved tiling and {8, 0, 1} is
 * the whole frame; runs give devices unequal shares (the multi-device frame
 * driver gives rank 0, which also assembles the frame, fewer rows:
 * {8, 0, P, 0, a, 1} for it and {8, a + r - 1, P, 0, b, N - 1} for rank
 * r >= 1, P = a + b (N - 1): the peers' blocks interleave inside the period,
 * so a frame whose block count is not a multiple of P gives its last partial
 * period's blocks to distinct ranks).                                        */
typedef struct {
  int32_t block_rows;
  int32_t first_block;
  int32_t block_stride;
  int32_t flags;      /* sdf_tiling_flags (0: packed rows) */
  int32_t block_run;  /* blocks per period (0 or 1: one) */
  int32_t run_step;   /* blocks between a run's blocks (0 or 1: consecutive);
                         (run - 1) * step < block_stride */
} sdf_tiling;

/* SDF_TILING_FRAME_ROWS: write the owned rows at their frame positions (the
 * buffer holds `height` rows, the others untouched) instead of packed --
 * rank 0 of a multi-device frame renders its share straight into the
 * assembled frame.  Not with SDF_FORMAT_TILES. */
typedef enum { SDF_TILING_FRAME_ROWS = 1 } sdf_tiling_flags;

/* ---- entry points -------------------------------------------------------- */

/* The packed tiling of `rank`'s share of a `world`-device frame: rank 0
 * share_root consecutive blocks and every other rank share_peer blocks,
 * world - 1 apart, per period of share_root + share_peer * (world - 1)
 * 8-row blocks (1:1 = plain interleave; world 1 = the whole frame). */
int sdf_share_tiling(int32_t rank, int32_t world, int32_t share_root, int32_t share_peer,
                     sdf_tiling* tiling);

/* ABI version of the loaded library (== SDF_ABI_VERSION when compatible). */
int sdf_abi_version(void);

/* Fill every non-null struct with the reference defaults (see top comment).
 * `width`/`height` set params->width/height (<= 0: 800 x 600, main.cpp:4-5). */
int sdf_defaults(sdf_scene* scene, sdf_camera* camera, sdf_light* light,
                 sdf_material* material, sdf_params* params,
                 int32_t width, int32_t height);

/* Validate a request without touching the device. */
int sdf_validate(const sdf_scene* scene, const sdf_camera* camera,
                 const sdf_light* light, const sdf_material* material,
                 const sdf_params* params, const sdf_tiling* tiling);

/* Number of rows a tiling owns in a frame of `height` rows (>= 0), or a
 * negative SDF_E* code. */
int sdf_owned_rows(int32_t height, const sdf_tiling* tiling);

/* Bytes per pixel of a sdf_format (16, 8, 4, 12, -, 16), or a negative SDF_E* code
 * (SDF_E_UNSUPPORTED for TILES, whose size is per stream). */
int sdf_format_bytes(int32_t format);

/* Capacity in bytes of a TILES stream of `rows` packed rows of `width`
 * pixels (the worst case: 32-bit residuals), or a negative SDF_E* code
 * (SDF_E_UNSUPPORTED when that worst case would not fit the stream's 32-bit
 * offsets: more than ~5.6M tiles, ~358 Mpixels; sdf_render refuses such a
 * TILES render the same way). */
int64_t sdf_tiles_bytes(int32_t width, int32_t rows);

/* Render the rows owned by `tiling` (NULL = whole frame) into `rgba`
 * (device, owned_rows * width pixels of params->output_format, packed as
 * described above).
 * `steps` (device, may be NULL) receives 2 int32 per pixel: the primary and
 * the shadow march iteration counts (diagnostics / flop accounting).
 * Asynchronous on `stream`. */
int sdf_render(const sdf_scene* scene, const sdf_camera* camera,
               const sdf_light* light, const sdf_material* material,
               const sdf_params* params, const sdf_tiling* tiling,
               void* rgba, int32_t* steps, void* stream);

/* Render schedules.  A frame's cost is uneven: grazing rays near the horizon
 * march long, so a launch whose last waves hold the costliest tiles ends
 * with most of the GPU idle.  sdf_render_scheduled is sdf_render dispatching
 * the rows' 8-row blocks in the order a schedule keeps: the kernel adds
 * every wave's shader-clock cycles to its block's counter, the schedule
 * reads the counters back every `period` launches without waiting (pinned
 * copy behind the launch, event polled at the next call), and later launches
 * take the blocks costliest first.  Any order renders every block exactly
 * once: the output is bit-identical to sdf_render's.  A schedule serves
 * renders of `rows` packed rows (owned rows of the tiling, <= 4096; others
 * render in launch order) and is not thread-safe; one schedule per stream
 * keeps each stream's measurements its own.  Create / destroy synchronise
 * the device. */
typedef struct sdf_schedule sdf_schedule;
int sdf_schedule_create(int32_t rows, int32_t period, sdf_schedule** schedule);
int sdf_schedule_destroy(sdf_schedule* schedule);
/* The schedule's current order (blockIdx.y -> 8-row block) into order[0..n):
 * returns the number of blocks it orders, 0 before its first cost snapshot
 * has landed (launch order). */
int sdf_schedule_order(const sdf_schedule* schedule, int32_t* order, int32_t n);
int sdf_render_scheduled(const sdf_scene* scene, const sdf_camera* camera,
                         const sdf_light* light, const sdf_material* material,
                         const sdf_params* params, const sdf_tiling* tiling,
                         void* rgba, int32_t* steps, sdf_schedule* schedule, void* stream);

/* Scatter `nparts` packed row-block buffers (part r = rank r's output for
 * tiling {block_rows, r, nparts}), laid out back to back in `parts` with a
 * pitch of `part_stride_rows` rows each, into the full frame `frame`
 * (height * width pixels of `format`; RGB32F parts produce an RGBA32F frame
 * with alpha = 1).  Device pointers; asynchronous on `stream`. */
int sdf_deinterleave(const void* parts, int32_t nparts,
                     int32_t part_stride_rows, int32_t width, int32_t height,
                     int32_t block_rows, int32_t format, void* frame, void* stream);

/* Decode `nparts` TILES streams (part r = rank r's output for tiling
 * {block_rows, r, nparts}; nparts = 1 with block_rows = height for a whole
 * frame), laid out back to back in `parts` with a pitch of `part_stride`
 * bytes, into the RGBA32F frame `frame` (height * width, alpha = 1): the
 * de-interleave of sdf_deinterleave fused with the decode.  A part whose
 * header says ntiles = 0 is skipped (its rows rendered into the frame by
 * other means, e.g. SDF_TILING_FRAME_ROWS).  Device pointers; asynchronous
 * on `stream`.
 * sdf_tiles_decode_tilings: part r holds the rows of tilings[r] (a host
 * array of nparts packed tilings, at most SDF_MAX_DECODE_PARTS), e.g. the
 * unequal shares of the frame driver; sdf_tiles_decode is the interleaved
 * case tilings[r] = {block_rows, r, nparts, 0, 1}. */
#define SDF_MAX_DECODE_PARTS 64
int sdf_tiles_decode_tilings(const void* parts, int32_t nparts, int64_t part_stride,
                             const sdf_tiling* tilings, int32_t width, int32_t height,
                             void* frame, void* stream);
int sdf_tiles_decode(const void* parts, int32_t nparts, int64_t part_stride,
                     int32_t width, int32_t height, int32_t block_rows, void* frame,
                     void* stream);

/* Streams are untrusted input (they crossed a wire): every decode reads only
 * inside each part's worst-case stream (sdf_tiles_bytes of its rows), and a
 * malformed part -- header length or tile count that disagrees with the
 * part, a tile whose offset, size or base widths leave the stream's data, an
 * escape field beyond its tile -- is skipped (the whole part, or the tiles
 * concerned: nothing is written for them; every other tile decodes as
 * usual).  sdf_tiles_decode(_tilings) skip silently;
 * sdf_tiles_decode_checked reports:
 *   used    host array of nparts (may be NULL): the data bytes part r must
 *           hold (its header word 0, e.g. the length the ranks agreed on
 *           before the transfer), or -1 for "the header's own, within the
 *           part"; a part expected to carry a stream (used[r] >= 0) whose
 *           header says none is malformed;
 *   status  device-writable array of nparts uint32 (may be NULL), zeroed by
 *           the caller: word r becomes nonzero (SDF_TILES_BAD_* bits) when
 *           part r is malformed -- asynchronous, like the decode.  With
 *           status == NULL the call waits for the decode on `stream` and
 *           returns SDF_E_COMM when some part was malformed. */
/* One byte per cause (ABI 11): each is set by a byte store of its own, so
 * the causes of a part combine without atomics (waves of one part race). */
#define SDF_TILES_BAD_HEADER 0x000001u
#define SDF_TILES_BAD_TILE   0x000100u
#define SDF_TILES_BAD_FIELD  0x010000u
int sdf_tiles_decode_checked(const void* parts, int32_t nparts, int64_t part_stride,
                             const sdf_tiling* tilings, const int64_t* used, int32_t width,
                             int32_t height, void* frame, uint32_t* status, void* stream);

/* Debug view of the `steps` output of sdf_render: `count` int2 entries
 * (primary, shadow) -> colours of `format`, with which = 0 (primary), 1
 * (shadow) or 2 (their sum), intensity = steps / max_steps mapped through the
 * Turbo colormap the reference ships unused (Code/kernel/utilities.cl:7-284:
 * its 256-entry table, index round(255 * intensity) rounded half away from
 * zero and clamped to [0, 255], alpha 1).  Device
 * pointers; asynchronous on `stream`. */
int sdf_heatmap(const int32_t* steps, int32_t count, int32_t which, int32_t max_steps,
                int32_t format, void* out, void* stream);

/* Number of scene signatures compiled at run time in this process (see
 * SDF_DISPATCH_AUTO). */
int sdf_jit_count(void);

/* Build identity of the built-in render kernels of `precision`
 * (SDF_PRECISION_*): 16 hex digits of a SHA-256 over the kernel's sources
 * (its translation unit, render_kernel.inc, kernel_args.h, wave_bits.h, cr_math.h,
 * sdf_abi.h), its compile flags and the compiler's version, fixed when the
 * library is built.  Measurement tools store it beside counters taken from
 * the kernel, so a counter summary is never applied to another build.
 * NULL for an unknown precision. */
const char* sdf_kernel_id(int32_t precision);

/* The culling bounds a primitive scene's fixed-scene kernels read (host
 * only, no device needed; diagnostics and tests): per primitive
 * bounds[4 * i ..] = {centre.xyz, K_i = (k_i + R_i + 1e-4) / (1 - 1e-5)}
 * with R_i the radius of a sphere containing primitive i, the cluster
 * cluster[0..3] = {centre.xyz, K} of the sphere containing primitives
 * [*cluster_first, count) (K with the largest blend radius), and
 * *cluster_first (= count when nothing is culled).  bounds holds
 * 4 * SDF_MAX_PRIMS floats.  SDF_E_UNSUPPORTED for a Mandelbulb scene. */
int sdf_scene_bounds(const sdf_scene* scene, float* bounds, float* cluster,
                     int32_t* cluster_first);

/* ---- multi-device frame driver ----------------------------------------------
 * One process per GPU.  Every rank renders its row blocks of each frame
 * (tiling with shares: rank 0 `share_root` blocks and every other rank
 * `share_peer` blocks per period of share_root + share_peer * (world - 1))
 * as a TILES stream; rank 0 renders its own rows straight into the frame and
 * assembles the rest: an RCCL all-gather of the streams' lengths, RCCL
 * point-to-point transfers of exactly those bytes to rank 0, and
 * sdf_tiles_decode_tilings into the frame -- bit-identical to a one-device
 * render.  Frames rotate over `nbuf` buffer sets, one HIP stream each; frame
 * i is shipped `lag` frames after its render (the host reads its agreed
 * lengths from pinned memory, without stalling the queue when lag >= 2).
 * The RCCL calls go to two communicators, each on a stream of its own (the
 * lengths; the streams), in the same order on every rank.
 *
 * RCCL is loaded at run time from `rccl_path` (the librccl.so this process
 * already uses, e.g. PyTorch's, so one RCCL instance serves both); the
 * caller exchanges each communicator's 128-byte unique id (rank 0 makes it
 * with sdf_comm_unique_id) through its own channel.
 * world == 1 needs no communicator: frames render whole, nothing is shipped. */
#define SDF_COMM_ID_BYTES 128
typedef struct sdf_comm sdf_comm;
typedef struct sdf_driver sdf_driver;

int sdf_comm_unique_id(const char* rccl_path, void* id /* SDF_COMM_ID_BYTES */);
/* Collective over nranks processes (blocks until all have joined, at most
 * timeout_ms, <= 0: 120000; then SDF_E_TIMEOUT); the current HIP device is
 * the communicator's. */
int sdf_comm_create(const char* rccl_path, const void* id, int32_t nranks, int32_t rank,
                    int32_t timeout_ms, sdf_comm** comm);
int sdf_comm_destroy(sdf_comm* comm);

/* SDF_DRIVER_ROOT_AS_PEER: rank 0 ships its rows as a TILES stream to itself
 * like every other rank (probes of one rank's full per-frame cost on one
 * GPU, world == 1 included). */
#define SDF_DRIVER_ROOT_AS_PEER 0x1
typedef struct {
  int32_t rank, world;
  int32_t share_root, share_peer; /* blocks per period (>= 1; 1:1 = plain interleave) */
  int32_t nbuf;                   /* buffer sets, 2 .. 16 (render streams: <= 4)      */
  int32_t lag;                    /* frames from a batch's last render to its gather,
                                     1 .. nbuf - batch                                */
  int32_t flags;                  /* SDF_DRIVER_*                                     */
  int32_t timeout_ms;             /* host waits give up after this (<= 0: 60000)      */
  int32_t batch;                  /* frames per ship (<= 0: 1): one length
                                     all-gather and one send/recv group per `batch`
                                     consecutive frames; nbuf % batch == 0          */
} sdf_driver_config;

/* The frame format is params->output_format (RGBA32F at world > 1: the wire
 * is lossless TILES).  size_comm, data_comm: two distinct communicators
 * over the `world` ranks, used by this driver alone (NULL when world == 1
 * without ROOT_AS_PEER). */
int sdf_driver_create(const sdf_scene* scene, const sdf_camera* camera, const sdf_light* light,
                      const sdf_material* material, const sdf_params* params,
                      const sdf_driver_config* config, sdf_comm* size_comm, sdf_comm* data_comm,
                      sdf_driver** driver);
/* Camera of the frames stepped from now on (the arcball V_mat of main.cpp:93-94). */
int sdf_driver_set_camera(sdf_driver* driver, const sdf_camera* camera);
/* Enqueue the next frame (index returned in *frame_index, may be NULL). */
int sdf_driver_step(sdf_driver* driver, int64_t* frame_index);
/* Ship every rendered frame and wait until all work of this rank is done. */
int sdf_driver_drain(sdf_driver* driver);
/* Rank 0 (or world 1): device pointer of frame `index`'s framebuffer
 * (height * width pixels), one of the last nbuf frames whose buffer set no
 * later frame has taken (after a drain that closed a short batch the next
 * frames may start on other buffer sets): any other index is
 * SDF_E_INVALID_ARG.  With collectives the frame must have been shipped (the
 * last `lag` frames stepped are, after sdf_driver_drain): an index not
 * shipped yet is SDF_E_INVALID_ARG.  A rank-0 decode that finds a peer's
 * stream malformed (sdf_tiles_decode_checked) fails the driver: the next
 * sdf_driver_step or sdf_driver_drain returns SDF_E_COMM. */
int sdf_driver_frame(sdf_driver* driver, int64_t index, void** rgba);
/* Copy frame `index` (as sdf_driver_frame) into the caller's device buffer
 * `dst` of `bytes` (>= the frame's size), asynchronously on `stream` after
 * all work queued for that frame. */
int sdf_driver_read_frame(sdf_driver* driver, int64_t index, void* dst, int64_t bytes,
                          void* stream);
/* Host-time accounting since creation (n >= 3 values): out[0] frames
 * stepped, out[1] seconds spent inside sdf_driver_step / sdf_driver_drain,
 * out[2] the part of out[1] spent waiting for the GPU or a peer; then the
 * seconds spent enqueueing out[3] renders, out[4] length all-gathers (with
 * their copies and events), out[5] RCCL send/recv groups, out[6] decodes. */
int sdf_driver_stats(sdf_driver* driver, double* out, int32_t n);
int sdf_driver_destroy(sdf_driver* driver);

/* ---- single-process multi-device frames -------------------------------------
 * One frame rendered across `ndev` devices of THIS process (the reference's
 * host is one process, main.cpp:34-110): devices[0] is the root and holds
 * `rgba` (width * height RGBA32F pixels, params->output_format must be
 * SDF_FORMAT_RGBA32F); `stream` is a stream of the root device.  Rows are
 * shared as by the driver (sdf_share_tiling with share_root : share_peer
 * blocks, <= 0: the measured defaults): the root renders its rows into
 * `rgba`, every other device its rows as a TILES stream into a buffer of its
 * own, and the root decodes those streams in place through peer-mapped
 * memory (hipDeviceEnablePeerAccess).  Asynchronous: the frame is complete
 * for work enqueued on `stream` after the call.  Successive calls must be
 * ordered (the same `stream`): they share the library's buffers for this
 * device list, two sets alternating so the peers render the next frame while
 * the root decodes this one.  A device may be listed more than once (its
 * shares then render on it in turn).  The current device is left unchanged. */
int sdf_render_multi(const sdf_scene* scene, const sdf_camera* camera, const sdf_light* light,
                     const sdf_material* material, const sdf_params* params, int32_t ndev,
                     const int32_t* devices, int32_t share_root, int32_t share_peer, void* rgba,
                     void* stream);
/* Wait for and free the buffers sdf_render_multi keeps. */
int sdf_render_multi_release(void);

/* ---- frame sequences ----------------------------------------------------------
 * n whole frames of one scene: frame i seen through cameras[i], written to
 * rgba[i] (width * height pixels of params->output_format; TILES is
 * SDF_E_UNSUPPORTED) and, when `steps` is non-null and steps[i] is, its
 * iteration counts to steps[i] (width * height int2).  Equal bit for bit to
 * n sdf_render calls with the same arguments.  This is the reference's frame
 * loop (main.cpp:87-98) for a camera path known in advance: the frames are
 * rendered by a persistent kernel, up to 16 frames per launch, whose waves
 * take 8x8 tiles of all its frames from one work counter, so a frame's
 * slowest tiles overlap the next frame's first ones.  Asynchronous on
 * `stream` (a stream of the current device).  Every camera is validated
 * before anything is enqueued. */
int sdf_render_frames(const sdf_scene* scene, const sdf_camera* cameras, int32_t n,
                      const sdf_light* light, const sdf_material* material,
                      const sdf_params* params, void* const* rgba, int32_t* const* steps,
                      void* stream);

/* Short description of a status code. */
const char* sdf_strerror(int code);

#ifdef __cplusplus
}
#endif

#endif /* SDF_ABI_H */

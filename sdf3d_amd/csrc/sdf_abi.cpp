// sdf_abi.cpp -- host side of the C-ABI declared in include/sdf_abi.h.
//
// Replaces what the reference does around `gl->plot(sh, proj_mode)`
// (/root/reference/Code/src/main.cpp:95): it takes the per-frame uniforms
// (the shader's V_mat and AR, voxel_fragment.frag:5-7) plus the scene, light
// and material that the reference hard-codes in the shader
// (voxel_fragment.frag:178-189), hoists the uniform-only arithmetic the shader
// repeats per pixel (inverse(V_mat) at :180 and :192, camera.pos at :180, the
// focal term at :191), and launches one HIP kernel over the requested rows.
#include <hip/hip_runtime.h>

#include <cmath>
#include <algorithm>
#include <cstring>
#include <initializer_list>
#include <memory>
#include <vector>

#include "../../include/sdf_abi.h"
#include "host_api.h"
#include "kernel_args.h"

// Layout contract with the ctypes mirror (sdf3d_amd/abi.py STRUCT_SIZES).
static_assert(sizeof(sdf_primitive) == 64, "sdf_primitive layout");
static_assert(sizeof(sdf_scene) == 8 + 64 * SDF_MAX_PRIMS + 32, "sdf_scene layout");
static_assert(sizeof(sdf_camera) == 88, "sdf_camera layout");
static_assert(sizeof(sdf_light) == 32, "sdf_light layout");
static_assert(sizeof(sdf_material) == 40, "sdf_material layout");
static_assert(sizeof(sdf_params) == 80, "sdf_params layout");
static_assert(sizeof(sdf_tiling) == 24, "sdf_tiling layout");
static_assert(sizeof(sdf_driver_config) == 36, "sdf_driver_config layout");

namespace sdf {

int tiling_run(const sdf_tiling& t) { return t.block_run > 1 ? t.block_run : 1; }
int tiling_step(const sdf_tiling& t) { return t.run_step > 1 ? t.run_step : 1; }
int tiling_gap_rows(const sdf_tiling& t) { return (tiling_step(t) - 1) * t.block_rows; }

int count_rows(int height, const sdf_tiling& t) {
  if (t.block_rows <= 0 || t.block_stride <= 0 || t.first_block < 0 || height < 0 ||
      t.block_run < 0 || t.run_step < 0 ||
      (long long)(tiling_run(t) - 1) * tiling_step(t) >= t.block_stride ||
      (t.flags & ~SDF_TILING_FRAME_ROWS) != 0)
    return SDF_E_INVALID_ARG;
  // spaced runs keep every 8-row tile of packed rows inside one block (the
  // kernels then find a tile's block once per wave)
  if (tiling_step(t) > 1 && t.block_rows % 8 != 0) return SDF_E_INVALID_ARG;
  // every period contributes its run of blocks, cut at the frame's last row
  long long rows = 0;
  const long long B = t.block_rows;
  for (long long b0 = t.first_block; b0 * B < height; b0 += t.block_stride)
    for (long long j = 0; j < tiling_run(t); ++j) {
      const long long b = b0 + j * tiling_step(t);
      if (b * B < height) rows += std::min<long long>((b + 1) * B, height) - b * B;
    }
  return (int)rows;
}

}  // namespace sdf

namespace {

// Inverse of a column-major 4x4 matrix via 2x2 sub-determinants, in double,
// rounded once to float.  GLSL's inverse() precision is unspecified; this is
// the correctly rounded exact inverse for all but pathological inputs.
bool invert_view(const float* mf, float* out) {
  double m[16];
  for (int i = 0; i < 16; ++i) m[i] = mf[i];
  // element (row r, col c) of a column-major matrix is m[c*4 + r]
  auto e = [&](int r, int c) { return m[c * 4 + r]; };
  const double s0 = e(0, 0) * e(1, 1) - e(1, 0) * e(0, 1);
  const double s1 = e(0, 0) * e(1, 2) - e(1, 0) * e(0, 2);
  const double s2 = e(0, 0) * e(1, 3) - e(1, 0) * e(0, 3);
  const double s3 = e(0, 1) * e(1, 2) - e(1, 1) * e(0, 2);
  const double s4 = e(0, 1) * e(1, 3) - e(1, 1) * e(0, 3);
  const double s5 = e(0, 2) * e(1, 3) - e(1, 2) * e(0, 3);
  const double c5 = e(2, 2) * e(3, 3) - e(3, 2) * e(2, 3);
  const double c4 = e(2, 1) * e(3, 3) - e(3, 1) * e(2, 3);
  const double c3 = e(2, 1) * e(3, 2) - e(3, 1) * e(2, 2);
  const double c2 = e(2, 0) * e(3, 3) - e(3, 0) * e(2, 3);
  const double c1 = e(2, 0) * e(3, 2) - e(3, 0) * e(2, 2);
  const double c0 = e(2, 0) * e(3, 1) - e(3, 0) * e(2, 1);
  const double det = s0 * c5 - s1 * c4 + s2 * c3 + s3 * c2 - s4 * c1 + s5 * c0;
  if (det == 0.0 || !std::isfinite(det)) return false;
  double inv[4][4];  // inv[r][c]
  inv[0][0] = (e(1, 1) * c5 - e(1, 2) * c4 + e(1, 3) * c3);
  inv[0][1] = (-e(0, 1) * c5 + e(0, 2) * c4 - e(0, 3) * c3);
  inv[0][2] = (e(3, 1) * s5 - e(3, 2) * s4 + e(3, 3) * s3);
  inv[0][3] = (-e(2, 1) * s5 + e(2, 2) * s4 - e(2, 3) * s3);
  inv[1][0] = (-e(1, 0) * c5 + e(1, 2) * c2 - e(1, 3) * c1);
  inv[1][1] = (e(0, 0) * c5 - e(0, 2) * c2 + e(0, 3) * c1);
  inv[1][2] = (-e(3, 0) * s5 + e(3, 2) * s2 - e(3, 3) * s1);
  inv[1][3] = (e(2, 0) * s5 - e(2, 2) * s2 + e(2, 3) * s1);
  inv[2][0] = (e(1, 0) * c4 - e(1, 1) * c2 + e(1, 3) * c0);
  inv[2][1] = (-e(0, 0) * c4 + e(0, 1) * c2 - e(0, 3) * c0);
  inv[2][2] = (e(3, 0) * s4 - e(3, 1) * s2 + e(3, 3) * s0);
  inv[2][3] = (-e(2, 0) * s4 + e(2, 1) * s2 - e(2, 3) * s0);
  inv[3][0] = (-e(1, 0) * c3 + e(1, 1) * c1 - e(1, 2) * c0);
  inv[3][1] = (e(0, 0) * c3 - e(0, 1) * c1 + e(0, 2) * c0);
  inv[3][2] = (-e(3, 0) * s3 + e(3, 1) * s1 - e(3, 2) * s0);
  inv[3][3] = (e(2, 0) * s3 - e(2, 1) * s1 + e(2, 2) * s0);
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 4; ++r) out[c * 4 + r] = static_cast<float>(inv[r][c] / det);
  return true;
}

bool finite3(const float* v) {
  return std::isfinite(v[0]) && std::isfinite(v[1]) && std::isfinite(v[2]);
}

int run_of(const sdf_tiling& t) { return sdf::tiling_run(t); }
using sdf::count_rows;

const sdf_tiling kWholeFrame = {8, 0, 1, 0, 1, 1};

// Per-frame preparation of the primitive parameter blocks the kernels read
// (layouts in render_kernel.inc).  Every derived value is computed in fp32
// with the operation order the oracle uses per evaluation (oracle_core.h), so
// the exact-precision kernel stays bit-identical; 1/x values are only used by
// the fast-precision kernel.
void prepare_prims(const sdf_scene& s, sdf_primitive* out) {
  std::memcpy(out, s.prims, sizeof(s.prims));
  for (int i = 0; i < s.count; ++i) {
    const sdf_primitive& in = s.prims[i];
    sdf_primitive& o = out[i];
    o.reserved = in.k > 0.0f ? 1.0f / in.k : 0.0f;
    o.p[11] = in.k * 0.25f;  // smooth-min k/4 (fast precision)
    // exact precision's smooth-min division n / k (render_kernel.inc smin,
    // cr_math.h smin_h / div_scaled): sc = 2^s with k sc in [0.5, 1) (s <=
    // 127, so a denormal k lands in [2^-22, 1)), and RN(1/(k sc)) by an IEEE
    // division.  k sc < 1: smin_h's clamp to [0, 1] is its max(., 0) alone
    float sc = 1.0f, ks = 1.0f;
    if (in.k > 0.0f && std::isfinite(in.k)) {
      int e = 0;
      (void)std::frexp(in.k, &e);                 // k = m 2^e, m in [0.5, 1)
      sc = std::ldexp(1.0f, std::min(-e, 127));
      ks = in.k * sc;                             // exact
    }
    o.p[9] = sc;
    o.p[10] = 1.0f / ks;
    // the prepared block's k slot carries k sc for the exact kernel (its
    // smooth-min reads k/4 from p[11] and k sc here; nothing else reads it)
    o.k = ks;
    const float* q = in.p;
    float* p = o.p;
    switch (in.kind) {
      case SDF_PRIM_ROUND_BOX: {
        const float r = q[6];
        p[3] = q[3] - r;
        p[4] = q[4] - r;
        p[5] = q[5] - r;
        p[6] = r;
        break;
      }
      case SDF_PRIM_CAPSULE: {
        const float bax = q[3] - q[0], bay = q[4] - q[1], baz = q[5] - q[2];
        const float baba = bax * bax + bay * bay + baz * baz;
        p[3] = bax;
        p[4] = bay;
        p[5] = baz;
        p[6] = q[6];
        p[7] = baba;
        p[8] = 1.0f / baba;
        break;
      }
      default:
        break;
    }
  }
}

// A small sphere containing the n spheres (c_i, r_i): the centre C minimises
// RC(C) = max_i |c_i - C| + r_i, which is convex in C.  Any C gives a valid
// bound; the search only makes it tighter (subgradient steps towards the
// farthest sphere with diminishing length from the centroid, and the
// two-sphere balls of every pair, keeping the best).  The tighter the
// cluster sphere, the more often the culling and the shadow march's lit
// tail (render_kernel.inc) skip it.  Cached per primitive list: sdf_render
// prepares a plan per call.
static double sphere_radius_at(const double (*c)[3], const double* r, int n, const double* C) {
  double R = 0;
  for (int i = 0; i < n; ++i) {
    const double dx = c[i][0] - C[0], dy = c[i][1] - C[1], dz = c[i][2] - C[2];
    R = std::max(R, std::sqrt(dx * dx + dy * dy + dz * dz) + r[i]);
  }
  return R;
}
static double cluster_sphere(const double (*c)[3], const double* r, int n, double* C) {
  thread_local double key[SDF_MAX_PRIMS * 4 + 1] = {-1};
  thread_local double kC[3], kR = 0;
  double k[SDF_MAX_PRIMS * 4 + 1] = {(double)n};
  for (int i = 0; i < n; ++i) {
    for (int j = 0; j < 3; ++j) k[1 + 4 * i + j] = c[i][j];
    k[4 + 4 * i] = r[i];
  }
  if (std::memcmp(k, key, sizeof(double) * (1 + 4 * n)) == 0) {
    std::memcpy(C, kC, sizeof(kC));
    return kR;
  }
  double B[3] = {0, 0, 0};
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 3; ++j) B[j] += c[i][j] / n;
  double RB = sphere_radius_at(c, r, n, B);
  // the ball of each pair, through both spheres' far points
  for (int i = 0; i < n; ++i)
    for (int m = i + 1; m < n; ++m) {
      double u[3], L = 0;
      for (int j = 0; j < 3; ++j) { u[j] = c[m][j] - c[i][j]; L += u[j] * u[j]; }
      L = std::sqrt(L);
      if (!(L > 0)) continue;
      const double off = 0.5 * (L + r[m] - r[i]);
      double T[3];
      for (int j = 0; j < 3; ++j) T[j] = c[i][j] + u[j] / L * off;
      const double RT = sphere_radius_at(c, r, n, T);
      if (RT < RB) { RB = RT; std::memcpy(B, T, sizeof(B)); }
    }
  // subgradient descent from the best so far
  double X[3];
  std::memcpy(X, B, sizeof(X));
  const double step0 = 0.25 * RB;
  for (int it = 0; it < 2000; ++it) {
    int far = 0;
    double best = -1, dist = 0;
    for (int i = 0; i < n; ++i) {
      const double dx = c[i][0] - X[0], dy = c[i][1] - X[1], dz = c[i][2] - X[2];
      const double d = std::sqrt(dx * dx + dy * dy + dz * dz);
      if (d + r[i] > best) { best = d + r[i]; far = i; dist = d; }
    }
    if (best < RB) { RB = best; std::memcpy(B, X, sizeof(B)); }
    if (!(dist > 0)) break;
    const double h = step0 / (1.0 + it);
    for (int j = 0; j < 3; ++j) X[j] += (c[far][j] - X[j]) / dist * h;
  }
  std::memcpy(key, k, sizeof(double) * (1 + 4 * n));
  std::memcpy(kC, B, sizeof(kC));
  kR = RB;
  std::memcpy(C, B, sizeof(kC));
  return RB;
}

// Bounding spheres and the cluster bound read by the fixed-scene kernels'
// culling (kernel_args.h "exact bounding-volume culling").  Radii are computed
// in double and rounded up.
void prepare_bounds(const sdf_scene& s, sdf::KernelArgs& a, bool exact = false) {
  std::memset(a.bound, 0, sizeof(a.bound));
  a.cluster_first = s.count;
  double cen[SDF_MAX_PRIMS][3], rad[SDF_MAX_PRIMS];
  bool cull[SDF_MAX_PRIMS];
  for (int i = 0; i < s.count; ++i) {
    const sdf_primitive& pr = s.prims[i];
    const float* q = pr.p;
    double c[3] = {q[0], q[1], q[2]}, R = 0;
    switch (pr.kind) {
      case SDF_PRIM_SPHERE: R = q[3]; break;
      case SDF_PRIM_BOX: R = std::sqrt(double(q[3]) * q[3] + double(q[4]) * q[4] + double(q[5]) * q[5]); break;
      case SDF_PRIM_ROUND_BOX: {
        // the box (b - r) rounded by r (render_kernel.inc sd_round_box; a
        // negative b - r only shrinks the shape: box_core falls with e)
        double e2 = 0;
        for (int j = 3; j < 6; ++j) {
          const double e = std::max(double(q[j]) - q[6], 0.0);
          e2 += e * e;
        }
        R = std::sqrt(e2) + std::fabs(double(q[6]));
        break;
      }
      case SDF_PRIM_TORUS: R = double(q[3]) + q[4]; break;
      case SDF_PRIM_CAPSULE: {
        for (int j = 0; j < 3; ++j) c[j] = 0.5 * (double(q[j]) + q[3 + j]);
        const double dx = double(q[3]) - q[0], dy = double(q[4]) - q[1], dz = double(q[5]) - q[2];
        R = 0.5 * std::sqrt(dx * dx + dy * dy + dz * dz) + q[6];
        break;
      }
      case SDF_PRIM_CYLINDER: R = std::sqrt(double(q[3]) * q[3] + double(q[4]) * q[4]); break;
      default: R = 0; break;
    }
    R = std::fabs(R) * (1.0 + 1e-6) + 1e-6;
    int kind = pr.kind;
    if (kind == SDF_PRIM_PLANE && q[0] == 0.0f && q[1] == 1.0f && q[2] == 0.0f) kind = sdf::kPrimPlaneY;
    cull[i] = sdf::cullable(kind, pr.op);
    const double k = pr.op == SDF_OP_SMOOTH_UNION ? pr.k : 0.0;
    for (int j = 0; j < 3; ++j) { cen[i][j] = c[j]; a.bound[i][j] = float(c[j]); }
    rad[i] = R;
    // K' = (k + R + margin) / (1 - kCullRel), rounded up (render_kernel.inc wave_near)
    a.bound[i][3] = float((k + R + sdf::kCullAbs) / (1.0 - sdf::kCullRel) * (1.0 + 1e-6));
    // exact kernel (the prepared block's `reserved`, unused there): the
    // offset of the gap an evaluated primitive's own value leaves in the
    // culling cache, k + margin + 1e-4 R (render_kernel.inc step_cached,
    // SDF_CULL_SGAP), rounded up
    if (exact && sdf::cullable(kind, pr.op))
      a.prims[i].reserved = float((k + sdf::kCullAbs + 1e-4 * R) * (1.0 + 1e-6));
  }
  int first = s.count;
  while (first > 0 && cull[first - 1]) --first;
  a.cluster_first = first;
  if (first < s.count) {
    double C[3];
    cluster_sphere(cen + first, rad + first, s.count - first, C);
    for (int j = 0; j < 3; ++j) C[j] = double(float(C[j]));   // the centre the kernel reads
    const double RC = sphere_radius_at(cen + first, rad + first, s.count - first, C);
    double kmax = 0;
    for (int i = first; i < s.count; ++i)
      if (s.prims[i].op == SDF_OP_SMOOTH_UNION) kmax = std::max(kmax, double(s.prims[i].k));
    for (int j = 0; j < 3; ++j) a.cluster[j] = float(C[j]);
    a.cluster[3] = float((kmax + RC * (1.0 + 1e-6) + 1e-6 + sdf::kCullAbs) /
                         (1.0 - sdf::kCullRel) * (1.0 + 1e-6));
  }
}

}  // namespace

namespace sdf {

// (kind, op) sequence of a primitive scene, the compile-time signature of a
// FixedScene kernel (an upward plane through its own kind, kPrimPlaneY)
int scene_signature(const sdf_scene& scene, int* sig) {
  const int n = scene.count;
  for (int i = 0; i < n; ++i) {
    const sdf_primitive& p = scene.prims[i];
    int kind = p.kind;
    if (kind == SDF_PRIM_PLANE && p.p[0] == 0.0f && p.p[1] == 1.0f && p.p[2] == 0.0f)
      kind = kPrimPlaneY;
    sig[i] = SDF_KO(kind, p.op);
  }
  return n;
}

int select_variant(const sdf_scene& scene) {
  if (scene.kind == SDF_SCENE_MANDELBULB) return kVariantBulb;
  int sig[SDF_MAX_PRIMS];
  const int n = scene_signature(scene, sig);
  auto match = [&](std::initializer_list<int> v) {
    if ((int)v.size() != n) return false;
    int i = 0;
    for (int k : v)
      if (sig[i++] != k) return false;
    return true;
  };
#define SDF_MATCH(id, ...) \
  if (match({__VA_ARGS__})) return id;
  SDF_FIXED_VARIANTS(SDF_MATCH)
#undef SDF_MATCH
  return kVariantGeneric;
}

}  // namespace sdf

namespace sdf {

void plan_set_camera(RenderPlan* plan, const sdf_camera* camera) {
  KernelArgs& a = plan->a;
  invert_view(camera->view, a.inv_view);
  const float* m = a.inv_view;
  // :180 camera.pos = (inverse(V_mat) * vec4(camera.pos, 1)).xyz, fp32
  for (int i = 0; i < 3; ++i)
    a.cam[i] = m[i] * camera->eye[0] + m[4 + i] * camera->eye[1] + m[8 + i] * camera->eye[2] +
               m[12 + i] * 1.0f;
  // :191 -2.0f / tan(camera.fov * PI / 360.0f), fp32
  const float ang = camera->fov_deg * camera->pi / 360.0f;
  a.focal = -2.0f / tanf(ang);
  a.aspect = camera->aspect > 0.0f ? camera->aspect : (float)a.width / (float)a.height;
}

int make_render_plan(const sdf_scene* scene, const sdf_camera* camera, const sdf_light* light,
                     const sdf_material* material, const sdf_params* params,
                     const sdf_tiling* tiling, void* rgba, int32_t* steps, RenderPlan* plan) {
  int rc = sdf_validate(scene, camera, light, material, params, tiling);
  if (rc != SDF_OK) return rc;
  if (!plan) return SDF_E_INVALID_ARG;
  const sdf_tiling t = tiling ? *tiling : kWholeFrame;
  const int rows = count_rows(params->height, t);
  std::memset(plan, 0, sizeof(*plan));
  plan->rows = rows;
  if (rows == 0) return SDF_OK;  // a rank that owns no block: nothing to write
  if (!rgba) return SDF_E_INVALID_ARG;

  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return SDF_E_NO_DEVICE;

  KernelArgs& a = plan->a;
  a.width = params->width;
  a.height = params->height;
  plan_set_camera(plan, camera);
  for (int i = 0; i < 3; ++i) {
    a.light_pos[i] = light->pos[i];
    a.mat_amb[i] = material->amb[i];
    a.mat_dif[i] = material->dif[i];
    a.mat_ref[i] = material->ref[i];
  }
  a.light_amb = light->ambient;
  a.shininess = material->shininess;
  a.max_steps = params->max_steps;
  a.max_dist = params->max_dist;
  a.eps = params->eps;
  a.shadow_k = params->shadow_k;
  a.normal_eps = params->normal_eps;
  a.shadow_offset = params->shadow_offset;
  a.flags = params->flags;
  a.normal_mode = params->normal_mode;
  a.format = params->output_format;
  a.ao_taps = (params->flags & SDF_FLAG_AO) ? params->ao_taps : 0;
  a.ao_step = params->ao_step;
  a.ao_base = params->ao_base;
  a.ao_falloff = params->ao_falloff;
  a.ao_strength = params->ao_strength;
  // AO tap heights, in the oracle's fp32 operation order (oracle_core.h
  // ambient_occlusion): t = i / (taps - 1); h = base + step * t
  for (int i = 0; i < a.ao_taps && i < kMaxAoTaps; ++i) {
    const float tt = a.ao_taps > 1 ? (float)i / (float)(a.ao_taps - 1) : 0.0f;
    a.ao_h[i] = params->ao_base + params->ao_step * tt;
  }
  // the AO taps' path lengths from P, visited in order (render_kernel.inc):
  // |h_0| + sum |h_k - h_(k-1)|, rounded up to fp32 so it never undercounts
  {
    double path = 0.0;
    for (int i = 0; i < a.ao_taps && i < kMaxAoTaps; ++i) {
      path += std::fabs((double)a.ao_h[i] - (i ? (double)a.ao_h[i - 1] : 0.0));
      float f = (float)path;
      if ((double)f < path) f = std::nextafter(f, INFINITY);
      a.ao_path[i] = f;
    }
  }
  a.inv_width = 1.0f / (float)params->width;
  a.inv_height = 1.0f / (float)params->height;
  a.block_rows = t.block_rows;
  a.chunk_rows = t.block_rows * run_of(t);
  a.run_gap_rows = sdf::tiling_gap_rows(t);
  a.first_block = t.first_block;
  a.block_stride = t.block_stride;
  a.rows = rows;
  a.frame_rows = (t.flags & SDF_TILING_FRAME_ROWS) ? 1 : 0;
  a.scene_kind = scene->kind;
  a.prim_count = scene->kind == SDF_SCENE_PRIMITIVES ? scene->count : 0;
  for (int i = 0; i < 3; ++i) a.bulb_center[i] = scene->bulb_center[i];
  a.bulb_scale = scene->bulb_scale;
  a.bulb_bail2 = scene->bulb_bailout * scene->bulb_bailout;
  a.bulb_iterations = scene->bulb_iterations;
  prepare_prims(*scene, a.prims);
  if (scene->kind == SDF_SCENE_PRIMITIVES)
    prepare_bounds(*scene, a, params->precision == SDF_PRECISION_EXACT);
  a.bulb_inv_scale = 1.0f / scene->bulb_scale;
  a.rgba = rgba;
  a.steps = steps;

  const bool generic = params->dispatch != SDF_DISPATCH_AUTO &&
                       scene->kind == SDF_SCENE_PRIMITIVES;
  if (params->dispatch == SDF_DISPATCH_UNCULLED) a.cluster_first = a.prim_count;
  plan->variant = generic ? kVariantGeneric : select_variant(*scene);
  plan->exact = params->precision == SDF_PRECISION_EXACT;
  // no built-in specialisation: a run-time compiled one (jit.cpp)
  plan->jit = plan->variant == kVariantGeneric && !generic && a.prim_count > 0;
  if (plan->jit) plan->nsig = scene_signature(*scene, plan->sig);
  plan->tiles_ntiles = params->output_format == SDF_FORMAT_TILES
                           ? ((params->width + 7) / 8) * ((rows + 7) / 8)
                           : 0;
  // TILES offsets and the `used` header word are uint32 (tiles.hip): a
  // stream whose worst case would not fit them is refused, not wrapped
  if (plan->tiles_ntiles > 0 && TilesLayout(plan->tiles_ntiles).stream_end > 0xffffffffull)
    return SDF_E_UNSUPPORTED;
  return SDF_OK;
}

int launch_render_plan(const RenderPlan& plan, void* stream) {
  if (plan.rows == 0) return SDF_OK;
  int err = -1;
  RenderArgs r;
  r.a = plan.a;
  r.o.cost = plan.order.cost;
  r.o.n = plan.order.n;
  r.o.reserved = 0;
  std::memcpy(r.o.order, plan.order.order, sizeof(uint16_t) * (size_t)std::max(plan.order.n, 0));
  if (plan.jit) err = launch_render_jit(r, plan.sig, plan.nsig, plan.exact, stream);
  if (err == -1)
    err = plan.exact ? launch_render_exact(r, plan.variant, stream)
                     : launch_render_fast(r, plan.variant, stream);
  if (err == hipSuccess && plan.tiles_ntiles > 0)
    err = launch_tiles_compact(plan.a.rgba, plan.tiles_ntiles, stream, plan.tiles_used);
  return err == hipSuccess ? SDF_OK : SDF_E_HIP;
}

// ---- render schedules (sdf_schedule) ---------------------------------------
// The kernels add each wave's shader-clock cycles to its 8-row block's cost
// word (RowOrder::cost).  Every `period` launches the schedule copies the
// words to pinned host memory behind the launch; once such a copy has landed
// (an event query: the host never waits), the cost of every block since the
// previous snapshot orders the blocks for the next launches, costliest first
// (LPT order: a frame's longest tiles start first, and short ones fill the
// end of the frame instead of the longest ones running alone).  The order is
// a permutation by construction and rides in the kernel arguments, so the
// measurement is a heuristic only: every block is rendered exactly once
// whatever the costs say.
struct Schedule {
  int rows = 0, nblocks = 0, period = 1;
  int dev = 0;
  unsigned long long* cost = nullptr;   // device, nblocks words (accumulating)
  unsigned long long* snap = nullptr;   // pinned host, nblocks words
  std::vector<unsigned long long> last; // the previous snapshot
  hipEvent_t ev = nullptr;
  bool pending = false;
  bool measure = false;                 // the launch being prepared measures its costs
  long long launches = 0;
  int n = 0;                            // 0 until the first order is known
  std::vector<uint16_t> order;
};

Schedule* schedule_create(int rows, int period) {
  auto* s = new Schedule();
  s->rows = rows;
  s->nblocks = (rows + 7) / 8;
  s->period = period > 0 ? period : 1;
  s->last.assign(s->nblocks, 0ull);
  s->order.resize(s->nblocks);
  bool ok = hipGetDevice(&s->dev) == hipSuccess && s->nblocks <= kMaxOrderBlocks;
  const size_t bytes = sizeof(unsigned long long) * std::max(s->nblocks, 1);
  ok = ok && hipMalloc((void**)&s->cost, bytes) == hipSuccess &&
       hipMemset(s->cost, 0, bytes) == hipSuccess &&
       hipHostMalloc((void**)&s->snap, bytes, hipHostMallocDefault) == hipSuccess &&
       hipEventCreateWithFlags(&s->ev, hipEventDisableTiming) == hipSuccess &&
       hipDeviceSynchronize() == hipSuccess;
  if (!ok) {
    schedule_destroy(s);
    return nullptr;
  }
  return s;
}

void schedule_destroy(Schedule* s) {
  if (!s) return;
  if (s->ev) {
    (void)hipEventSynchronize(s->ev);
    (void)hipEventDestroy(s->ev);
  }
  if (s->cost) (void)hipFree(s->cost);
  if (s->snap) (void)hipHostFree(s->snap);
  delete s;
}

int schedule_apply(Schedule* s, RenderPlan* plan) {
  plan->order.n = 0;
  plan->order.cost = nullptr;
  if (!s || plan->rows != s->rows) return SDF_OK;   // another shape: launch order, no costs
  const hipError_t q = s->pending ? hipEventQuery(s->ev) : hipErrorNotReady;
  if (s->pending && q != hipSuccess && q != hipErrorNotReady) {
    // the copy of the costs failed: stop waiting for it and
    // report the error; the next call measures again
    (void)hipGetLastError();
    s->pending = false;
    return SDF_E_HIP;
  }
  if (s->pending && q == hipSuccess) {
    s->pending = false;
    std::vector<std::pair<unsigned long long, int>> d(s->nblocks);
    unsigned long long total = 0;
    for (int b = 0; b < s->nblocks; ++b) {
      const unsigned long long v = s->snap[b] - s->last[b];
      s->last[b] = s->snap[b];
      d[b] = {v, b};
      total += v;
    }
    if (total > 0) {
      // costliest first; ties (and blocks not measured) in launch order
      std::stable_sort(d.begin(), d.end(), [](const auto& x, const auto& y) {
        return x.first > y.first;
      });
      for (int i = 0; i < s->nblocks; ++i) s->order[i] = (uint16_t)d[i].second;
      s->n = s->nblocks;
    }
  }
  // only the launch whose costs are copied out measures them (every wave's
  // clock reads and its atomic add cost the others nothing)
  s->measure = !s->pending && (s->launches % s->period) == 0;
  plan->order.cost = s->measure ? s->cost : nullptr;
  plan->order.n = s->n;
  if (s->n) std::memcpy(plan->order.order, s->order.data(), sizeof(uint16_t) * s->n);
  return SDF_OK;
}

int schedule_after(Schedule* s, void* stream) {
  if (!s) return SDF_OK;
  s->launches++;
  if (!s->measure) return SDF_OK;
  s->measure = false;
  if (hipMemcpyAsync(s->snap, s->cost, sizeof(unsigned long long) * s->nblocks,
                     hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
      hipEventRecord(s->ev, (hipStream_t)stream) != hipSuccess)
    return SDF_E_HIP;
  s->pending = true;
  return SDF_OK;
}

}  // namespace sdf

struct sdf_schedule {
  sdf::Schedule* s;
};

extern "C" {

int sdf_abi_version(void) { return SDF_ABI_VERSION; }

int sdf_schedule_create(int32_t rows, int32_t period, sdf_schedule** out) {
  if (!out) return SDF_E_INVALID_ARG;
  *out = nullptr;
  if (rows <= 0 || rows > 8 * sdf::kMaxOrderBlocks || period < 1) return SDF_E_INVALID_ARG;
  sdf::Schedule* s = sdf::schedule_create(rows, period);
  if (!s) return SDF_E_HIP;
  *out = new sdf_schedule{s};
  return SDF_OK;
}

int sdf_schedule_destroy(sdf_schedule* s) {
  if (!s) return SDF_OK;
  sdf::schedule_destroy(s->s);
  delete s;
  return SDF_OK;
}

int sdf_schedule_order(const sdf_schedule* s, int32_t* order, int32_t n) {
  if (!s || (n > 0 && !order)) return SDF_E_INVALID_ARG;
  for (int i = 0; i < n && i < s->s->n; ++i) order[i] = s->s->order[i];
  return s->s->n;
}

int sdf_render_scheduled(const sdf_scene* scene, const sdf_camera* camera, const sdf_light* light,
                         const sdf_material* material, const sdf_params* params,
                         const sdf_tiling* tiling, void* rgba, int32_t* steps,
                         sdf_schedule* schedule, void* stream) {
  sdf::RenderPlan plan;
  int rc = sdf::make_render_plan(scene, camera, light, material, params, tiling, rgba, steps,
                                 &plan);
  if (rc != SDF_OK) return rc;
  if (schedule) {
    rc = sdf::schedule_apply(schedule->s, &plan);
    if (rc != SDF_OK) return rc;
  }
  rc = sdf::launch_render_plan(plan, stream);
  if (rc == SDF_OK && schedule && plan.rows == schedule->s->rows)
    rc = sdf::schedule_after(schedule->s, stream);
  return rc;
}

int sdf_defaults(sdf_scene* scene, sdf_camera* camera, sdf_light* light,
                 sdf_material* material, sdf_params* params, int32_t width, int32_t height) {
  if (scene) {
    std::memset(scene, 0, sizeof(*scene));
    scene->kind = SDF_SCENE_PRIMITIVES;
    scene->count = 2;
    // sceneSDF (voxel_fragment.frag:73-81): min(min(INF, planeSDF), sphereSDF)
    sdf_primitive& plane = scene->prims[0];   // planeSDF :66-71 -> p.y
    plane.kind = SDF_PRIM_PLANE;
    plane.op = SDF_OP_UNION;
    plane.p[1] = 1.0f;
    sdf_primitive& sphere = scene->prims[1];  // sphereSDF :54-64
    sphere.kind = SDF_PRIM_SPHERE;
    sphere.op = SDF_OP_UNION;
    sphere.p[1] = 0.4f;
    sphere.p[3] = 0.2f;
    scene->bulb_scale = 1.0f;
    scene->bulb_iterations = 12;
    scene->bulb_bailout = 2.0f;
  }
  if (camera) {
    std::memset(camera, 0, sizeof(*camera));
    for (int i = 0; i < 4; ++i) camera->view[i * 5] = 1.0f;  // orbit/pan 0 (main.cpp:7-11)
    camera->eye[1] = 0.2f;                                     // :179
    camera->eye[2] = 2.0f;
    camera->fov_deg = 60.0f;                                   // :178
    camera->aspect = 0.0f;                                     // AR = W / H
    camera->pi = 3.1415925359f;                                // :15 (sic)
  }
  if (light) {
    std::memset(light, 0, sizeof(*light));
    light->pos[0] = 5.0f;                                      // :182
    light->pos[1] = 5.0f;
    light->ambient = 0.1f;                                     // :184
    light->color[0] = light->color[1] = light->color[2] = 0.7f; // :183 (unused)
  }
  if (material) {
    std::memset(material, 0, sizeof(*material));
    material->amb[1] = 0.2f;                                   // :186
    material->amb[2] = 0.8f;
    material->dif[1] = 0.2f;                                   // :187
    material->dif[2] = 0.8f;
    material->ref[0] = material->ref[1] = material->ref[2] = 0.5f; // :188
    material->shininess = 12.0f;                               // :189
  }
  if (params) {
    std::memset(params, 0, sizeof(*params));
    params->width = width > 0 ? width : 800;                   // main.cpp:4
    params->height = height > 0 ? height : 600;                // main.cpp:5
    params->max_steps = 100;                                   // :17
    params->max_dist = 100.0f;                                 // :18
    params->eps = 0.01f;                                       // :19
    params->shadow_k = 10.0f;                                  // :205
    params->normal_eps = 0.01f;                                // :21-23
    params->shadow_offset = 2.0f;                              // :205
    params->flags = SDF_FLAG_SHADOW;
    params->normal_mode = SDF_NORMAL_CENTRAL;
    params->ao_taps = 5;
    params->ao_step = 0.12f;
    params->ao_base = 0.01f;
    params->ao_falloff = 0.95f;
    params->ao_strength = 3.0f;
    params->precision = SDF_PRECISION_EXACT;
  }
  return SDF_OK;
}

int sdf_share_tiling(int32_t rank, int32_t world, int32_t share_root, int32_t share_peer,
                     sdf_tiling* tiling) {
  if (!tiling || world < 1 || rank < 0 || rank >= world || share_root < 1 || share_peer < 1)
    return SDF_E_INVALID_ARG;
  const int a = share_root, b = share_peer;
  if (world == 1) {
    *tiling = kWholeFrame;
  } else {
    // peers' blocks interleave (world - 1 apart), so the frame's last partial
    // period spreads over distinct ranks instead of one peer's whole run
    *tiling = sdf_tiling{8, rank == 0 ? 0 : a + rank - 1, a + b * (world - 1), 0,
                         rank == 0 ? a : b, rank == 0 || b == 1 ? 1 : world - 1};
  }
  return SDF_OK;
}

int sdf_owned_rows(int32_t height, const sdf_tiling* tiling) {
  return count_rows(height, tiling ? *tiling : kWholeFrame);
}

// Working range of the kernels: every coordinate, size and distance at most
// 1e15 in magnitude (and capsules of positive length), so that no square,
// dot product or distance the scene evaluation forms overflows -- every
// primitive value is then finite and the accumulated scene distance is never
// NaN, which the exact kernel's hardware minimum relies on (render_kernel.inc
// smin<HW>).
constexpr float kMaxCoord = 1e15f;
constexpr float kMinCapsule2 = 0x1p-30f;
constexpr float kMaxCapsule2 = 0x1p30f;

int sdf_validate(const sdf_scene* scene, const sdf_camera* camera, const sdf_light* light,
                 const sdf_material* material, const sdf_params* params,
                 const sdf_tiling* tiling) {
  if (!scene || !camera || !light || !material || !params) return SDF_E_INVALID_ARG;
  const sdf_params& p = *params;
  if (p.width <= 0 || p.height <= 0 || p.width > 65536 || p.height > 65536)
    return SDF_E_INVALID_ARG;
  if (p.max_steps < 0 || p.max_steps > (1 << 24)) return SDF_E_INVALID_ARG;
  // every length the marches add to a coordinate stays in the working range
  // (kMaxCoord below): normal_eps^2 and the AO tap lengths must not overflow,
  // which the exact kernels' one-compare cr_sqrt guard relies on
  for (float v : {p.max_dist, p.eps, p.shadow_k, p.normal_eps, p.shadow_offset})
    if (!(std::fabs(v) <= kMaxCoord)) return SDF_E_INVALID_ARG;
  if (p.flags & SDF_FLAG_AO)
    for (float v : {p.ao_step, p.ao_base, p.ao_falloff, p.ao_strength})
      if (!(std::fabs(v) <= kMaxCoord)) return SDF_E_INVALID_ARG;
  if (p.flags & ~(SDF_FLAG_SHADOW | SDF_FLAG_AO)) return SDF_E_INVALID_ARG;
  if (p.normal_mode != SDF_NORMAL_CENTRAL && p.normal_mode != SDF_NORMAL_TETRA)
    return SDF_E_INVALID_ARG;
  if (p.precision != SDF_PRECISION_EXACT && p.precision != SDF_PRECISION_FAST)
    return SDF_E_INVALID_ARG;
  if (p.dispatch < SDF_DISPATCH_AUTO || p.dispatch > SDF_DISPATCH_UNCULLED)
    return SDF_E_INVALID_ARG;
  if (p.output_format != SDF_FORMAT_TILES && sdf_format_bytes(p.output_format) < 0)
    return SDF_E_INVALID_ARG;
  if ((p.flags & SDF_FLAG_AO) && (p.ao_taps < 0 || p.ao_taps > sdf::kMaxAoTaps))
    return SDF_E_INVALID_ARG;
  if (count_rows(p.height, tiling ? *tiling : kWholeFrame) < 0) return SDF_E_INVALID_ARG;
  if (tiling && (tiling->flags & SDF_TILING_FRAME_ROWS) && p.output_format == SDF_FORMAT_TILES)
    return SDF_E_INVALID_ARG;   // a stream is made of packed tiles
  if (scene->kind == SDF_SCENE_PRIMITIVES) {
    if (scene->count < 0 || scene->count > SDF_MAX_PRIMS) return SDF_E_INVALID_ARG;
    for (int i = 0; i < scene->count; ++i) {
      const sdf_primitive& pr = scene->prims[i];
      if (pr.kind < 0 || pr.kind >= SDF_PRIM_KIND_COUNT) return SDF_E_INVALID_ARG;
      if (pr.op < 0 || pr.op >= SDF_OP_COUNT) return SDF_E_INVALID_ARG;
      const bool smooth = pr.op == SDF_OP_SMOOTH_UNION || pr.op == SDF_OP_SMOOTH_SUBTRACT ||
                          pr.op == SDF_OP_SMOOTH_INTERSECT;
      // a smooth blend radius in [2^-64, 1e15]: the exact smooth-min's
      // h h (k/4) relies on the lower end (render_kernel.inc smin)
      if (smooth && !(pr.k >= 0x1p-64f && pr.k <= kMaxCoord)) return SDF_E_INVALID_ARG;
      for (float v : pr.p)
        if (!std::isfinite(v) || std::fabs(v) > kMaxCoord) return SDF_E_INVALID_ARG;
      if (pr.kind == SDF_PRIM_CAPSULE) {
        // a segment of length in [2^-15, 2^15): dot(ba, ba), computed as the
        // kernels do, in [2^-30, 2^30) -- the exact kernel's Markstein
        // division of h = dot(pa, ba) / dot(ba, ba) (render_kernel.inc
        // sd_capsule) needs its divisor there
        const float bax = pr.p[3] - pr.p[0], bay = pr.p[4] - pr.p[1], baz = pr.p[5] - pr.p[2];
        const float baba = bax * bax + bay * bay + baz * baz;
        if (!(baba >= kMinCapsule2 && baba < kMaxCapsule2)) return SDF_E_INVALID_ARG;
      }
    }
  } else if (scene->kind == SDF_SCENE_MANDELBULB) {
    // local coordinates (p - c) * RN(1/scale) stay finite: |p - c| <= ~3e15
    // and 1/scale <= 1e15, so the exact kernel's Markstein steps (unbounded
    // above, BulbScene::local) never see an overflowing product
    if (!(scene->bulb_scale >= 1.0f / kMaxCoord && scene->bulb_scale <= kMaxCoord))
      return SDF_E_INVALID_ARG;
    for (float v : scene->bulb_center)
      if (!(std::fabs(v) <= kMaxCoord)) return SDF_E_INVALID_ARG;
    if (scene->bulb_iterations < 1 || scene->bulb_iterations > 64) return SDF_E_INVALID_ARG;
    // bailout in (0, 2^32]: its square stays finite, so every iteration's
    // x^2 + z^2 <= m <= bailout^2 is finite (the exact kernel's 1 / sqrt of it,
    // render_kernel.inc frsqrt, relies on that)
    if (!(scene->bulb_bailout > 0.0f && scene->bulb_bailout <= 4294967296.0f))
      return SDF_E_INVALID_ARG;
  } else {
    return SDF_E_INVALID_ARG;
  }
  for (float v : camera->view)
    if (!std::isfinite(v)) return SDF_E_INVALID_ARG;
  if (!finite3(camera->eye) || !std::isfinite(camera->fov_deg) || !std::isfinite(camera->pi))
    return SDF_E_INVALID_ARG;
  if (!finite3(light->pos)) return SDF_E_INVALID_ARG;
  float inv[16];
  if (!invert_view(camera->view, inv)) return SDF_E_INVALID_ARG;
  for (float v : inv)
    if (!(std::fabs(v) <= kMaxCoord)) return SDF_E_INVALID_ARG;
  // the hoisted camera position inverse(V_mat) * (eye, 1) (voxel_fragment.frag:180)
  for (int i = 0; i < 3; ++i) {
    const double c = (double)inv[i] * camera->eye[0] + (double)inv[4 + i] * camera->eye[1] +
                     (double)inv[8 + i] * camera->eye[2] + inv[12 + i];
    if (!(std::fabs(c) <= kMaxCoord)) return SDF_E_INVALID_ARG;
  }
  for (int i = 0; i < 3; ++i)
    if (std::fabs(camera->eye[i]) > kMaxCoord || std::fabs(light->pos[i]) > kMaxCoord)
      return SDF_E_INVALID_ARG;
  if (std::fabs(p.max_dist) > kMaxCoord) return SDF_E_INVALID_ARG;
  (void)material;
  return SDF_OK;
}

int sdf_format_bytes(int32_t format) {
  switch (format) {
    case SDF_FORMAT_RGBA32F: return 16;
    case SDF_FORMAT_RGBA16F: return 8;
    case SDF_FORMAT_RGBA8: return 4;
    case SDF_FORMAT_RGB32F: return 12;
    case SDF_FORMAT_TILES: return SDF_E_UNSUPPORTED;   // size is per stream
    case SDF_FORMAT_SHADE32F: return 16;
    default: return SDF_E_INVALID_ARG;
  }
}

// TILES buffer: the stream (header, offset table, worst-case records of 3 x
// 32 bit planes) and the encoder's scratch (kernel_args.h TilesLayout)
int64_t sdf_tiles_bytes(int32_t width, int32_t rows) {
  if (width <= 0 || rows < 0) return SDF_E_INVALID_ARG;
  const int64_t ntiles = int64_t((width + 7) / 8) * ((rows + 7) / 8);
  if (sdf::TilesLayout(ntiles).stream_end > 0xffffffffull) return SDF_E_UNSUPPORTED;
  return (int64_t)sdf::TilesLayout(ntiles).end;
}

int sdf_render(const sdf_scene* scene, const sdf_camera* camera, const sdf_light* light,
               const sdf_material* material, const sdf_params* params,
               const sdf_tiling* tiling, void* rgba, int32_t* steps, void* stream) {
  sdf::RenderPlan plan;
  const int rc = sdf::make_render_plan(scene, camera, light, material, params, tiling, rgba,
                                       steps, &plan);
  if (rc != SDF_OK) return rc;
  return sdf::launch_render_plan(plan, stream);
}

int sdf_jit_count(void) { return sdf::jit_compiled_count(); }

// SDF_KERNEL_ID_EXACT / _FAST: written by sdf3d_amd/build.py (kernel_id())
#include "kernel_id.inc"

const char* sdf_kernel_id(int32_t precision) {
  if (precision == SDF_PRECISION_EXACT) return SDF_KERNEL_ID_EXACT;
  if (precision == SDF_PRECISION_FAST) return SDF_KERNEL_ID_FAST;
  return nullptr;
}

int sdf_scene_bounds(const sdf_scene* scene, float* bounds, float* cluster,
                     int32_t* cluster_first) {
  if (!scene || !bounds || !cluster || !cluster_first) return SDF_E_INVALID_ARG;
  sdf_camera c;
  sdf_light l;
  sdf_material m;
  sdf_params p;
  sdf_defaults(nullptr, &c, &l, &m, &p, 0, 0);
  const int rc = sdf_validate(scene, &c, &l, &m, &p, nullptr);   // the scene's own checks
  if (rc != SDF_OK) return rc;
  if (scene->kind != SDF_SCENE_PRIMITIVES) return SDF_E_UNSUPPORTED;
  std::unique_ptr<sdf::KernelArgs> a(new sdf::KernelArgs());
  prepare_bounds(*scene, *a);
  std::memcpy(bounds, a->bound, sizeof(a->bound));
  std::memcpy(cluster, a->cluster, sizeof(a->cluster));
  *cluster_first = a->cluster_first;
  return SDF_OK;
}

namespace {
int decode_parts(const void* parts, int32_t nparts, int64_t part_stride, const sdf_tiling* tilings,
                 const int64_t* used, int32_t width, int32_t height, void* frame, uint32_t* status,
                 void* stream) {
  if (!parts || !frame || !tilings || nparts <= 0 || nparts > SDF_MAX_DECODE_PARTS ||
      width <= 0 || height <= 0)
    return SDF_E_INVALID_ARG;
  sdf::DecodeParts d{};
  d.status = status;
  if (used)
    for (int r = 0; r < nparts; ++r) d.used[r] = used[r] < 0 ? -1 : used[r];
  d.nparts = nparts;
  d.width = width;
  d.height = height;
  d.part_stride = part_stride;
  for (int r = 0; r < nparts; ++r) {
    const sdf_tiling& t = tilings[r];
    const int rows = count_rows(height, t);
    if (rows < 0 || t.flags != 0) return SDF_E_INVALID_ARG;
    // every part's stream must fit its pitch
    const int64_t n = int64_t((width + 7) / 8) * ((rows + 7) / 8);
    if ((int64_t)sdf::TilesLayout(n).stream_end > part_stride) return SDF_E_INVALID_ARG;
    d.rows[r] = rows;
    d.first_block[r] = t.first_block;
    d.block_stride[r] = t.block_stride;
    d.block_rows[r] = t.block_rows;
    d.chunk_rows[r] = t.block_rows * run_of(t);
    d.run_gap_rows[r] = sdf::tiling_gap_rows(t);
  }
  const int err = sdf::launch_tiles_decode(d, frame, parts, stream);
  return err == hipSuccess ? SDF_OK : SDF_E_HIP;
}
}  // namespace

int sdf_tiles_decode_tilings(const void* parts, int32_t nparts, int64_t part_stride,
                             const sdf_tiling* tilings, int32_t width, int32_t height,
                             void* frame, void* stream) {
  return decode_parts(parts, nparts, part_stride, tilings, nullptr, width, height, frame, nullptr,
                      stream);
}

int sdf_tiles_decode_checked(const void* parts, int32_t nparts, int64_t part_stride,
                             const sdf_tiling* tilings, const int64_t* used, int32_t width,
                             int32_t height, void* frame, uint32_t* status, void* stream) {
  if (status)
    return decode_parts(parts, nparts, part_stride, tilings, used, width, height, frame, status,
                        stream);
  // synchronous: status words of the library's own (pinned host memory the
  // device writes), read once the decode is done
  if (nparts <= 0 || nparts > SDF_MAX_DECODE_PARTS) return SDF_E_INVALID_ARG;
  uint32_t* st = nullptr;
  if (hipHostMalloc((void**)&st, sizeof(uint32_t) * nparts, hipHostMallocDefault) != hipSuccess)
    return SDF_E_HIP;
  std::memset(st, 0, sizeof(uint32_t) * nparts);
  int rc = decode_parts(parts, nparts, part_stride, tilings, used, width, height, frame, st, stream);
  if (rc == SDF_OK && hipStreamSynchronize((hipStream_t)stream) != hipSuccess) rc = SDF_E_HIP;
  if (rc == SDF_OK)
    for (int r = 0; r < nparts; ++r)
      if (st[r]) rc = SDF_E_COMM;
  (void)hipHostFree(st);
  return rc;
}

int sdf_tiles_decode(const void* parts, int32_t nparts, int64_t part_stride, int32_t width,
                     int32_t height, int32_t block_rows, void* frame, void* stream) {
  if (nparts <= 0 || nparts > SDF_MAX_DECODE_PARTS || block_rows <= 0) return SDF_E_INVALID_ARG;
  sdf_tiling t[SDF_MAX_DECODE_PARTS];
  for (int r = 0; r < nparts; ++r) t[r] = {block_rows, r, nparts, 0, 1};
  return sdf_tiles_decode_tilings(parts, nparts, part_stride, t, width, height, frame, stream);
}

int sdf_deinterleave(const void* parts, int32_t nparts, int32_t part_stride_rows,
                     int32_t width, int32_t height, int32_t block_rows, int32_t format,
                     void* frame, void* stream) {
  const int bpp = sdf_format_bytes(format);
  if (bpp < 0 || !parts || !frame || nparts <= 0 || width <= 0 || height <= 0 ||
      block_rows <= 0)
    return SDF_E_INVALID_ARG;
  // every part must hold its owned rows
  for (int r = 0; r < nparts; ++r) {
    const sdf_tiling t = {block_rows, r, nparts, 0, 1};
    if (count_rows(height, t) > part_stride_rows) return SDF_E_INVALID_ARG;
  }
  const int err =
      format == SDF_FORMAT_RGB32F
          ? sdf::launch_deinterleave_rgb(parts, nparts, part_stride_rows, width, height,
                                         block_rows, frame, stream)
          : sdf::launch_deinterleave(parts, nparts, part_stride_rows, width * bpp, height,
                                     block_rows, frame, stream);
  return err == hipSuccess ? SDF_OK : SDF_E_HIP;
}

int sdf_heatmap(const int32_t* steps, int32_t count, int32_t which, int32_t max_steps,
                int32_t format, void* out, void* stream) {
  if (count < 0 || which < 0 || which > 2 || max_steps < 0 || sdf_format_bytes(format) < 0 ||
      format == SDF_FORMAT_SHADE32F)   // colours only
    return SDF_E_INVALID_ARG;
  if (count == 0) return SDF_OK;
  if (!steps || !out) return SDF_E_INVALID_ARG;
  const int err = sdf::launch_heatmap(steps, count, which, max_steps, format, out, stream);
  return err == hipSuccess ? SDF_OK : SDF_E_HIP;
}

const char* sdf_strerror(int code) {
  switch (code) {
    case SDF_OK: return "success";
    case SDF_E_INVALID_ARG: return "invalid argument";
    case SDF_E_UNSUPPORTED: return "unsupported request";
    case SDF_E_HIP: return "HIP runtime error";
    case SDF_E_NO_DEVICE: return "no HIP device available";
    case SDF_E_COMM: return "RCCL unavailable or a collective failed";
    case SDF_E_TIMEOUT: return "frame driver wait timed out";
    default: return "unknown error";
  }
}

}  // extern "C"

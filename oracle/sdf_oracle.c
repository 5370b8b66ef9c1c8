/*
 * sdf_oracle.c -- TEST INFRASTRUCTURE ONLY: the CPU oracle for the SDF
 * sphere-tracing hot path (see oracle_core.h for the restatement itself and
 * its parity status).  Built by oracle/Makefile into oracle/build/
 * liboracle.so; loaded by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg through ctypes (oracle/oracle.py).  Never linked into or
 * called by the product library.
 *
 * Exports:
 *   sdf_oracle_defaults   the reference's hard-coded values, restated from
 *                         voxel_fragment.frag:15-23, :54-81, :178-189, :205
 *                         and main.cpp:4-11 (independently of the product's
 *                         sdf_defaults, which the tests compare against it)
 *   sdf_oracle_render     fp32 restatement (OpenMP over rows if nthreads > 1)
 *   sdf_oracle_render_f64 fp64 twin (diagnosis of branch flips only)
 *   sdf_oracle_replay     fp32 restatement with per-pixel break points imposed
 *                         (forced-step replay: is a kernel's outlier explained
 *                         by the step counts it recorded?  tests/parity.py)
 */
#include <math.h>
#include <stddef.h>
#include <string.h>

#include "../include/sdf_abi.h"

/* Uniform work hoisted out of the per-pixel code (the shader recomputes it
 * per pixel: voxel_fragment.frag:180, :191-192). */
typedef struct {
  float inv_view[16]; /* inverse(V_mat), column-major */
  float cam[3];       /* (inverse(V_mat) * vec4(camera.pos, 1)).xyz, :180 */
  float focal;        /* -2 / tan(fov * PI / 360), :191 */
  float aspect;       /* AR */
} oracle_uniforms;

/* ---- fp32 oracle ----
 * log and pow are the two transcendentals (Mandelbulb DE, specular
 * exponent).  GLSL leaves their precision to the implementation; the oracle
 * takes the tightest reading, correctly rounded fp32, evaluated in double and
 * rounded once, so its fp32 result does not depend on which libm's logf/powf
 * it links (the exact-precision kernel evaluates them the same way). */
static inline float cr_logf(float x) { return (float)log((double)x); }
static inline float cr_powf(float x, float y) { return (float)pow((double)x, (double)y); }
/* sdf_oracle_render_terms (below): each pixel's shading terms (ao, dif,
 * max(N.H, 0), 1) -- what SDF_FORMAT_SHADE32F and the TILES wire carry --
 * recorded by the restatement's instrumentation hook and written instead of
 * the colour while g_terms_out is set (one render at a time).  Tools that
 * define their own hook (tools/terms_probe.c) leave these out. */
#ifndef ORACLE_TERMS_HOOK
static _Thread_local float t_terms[3];
static int g_terms_out;
#define ORACLE_TERMS_HOOK(ao, dif, spec, x, ndl, sh) \
  (t_terms[0] = (float)(ao), t_terms[1] = (float)(dif), t_terms[2] = (float)(x))
#define ORACLE_PIXEL_OUT_HOOK(px)                                               \
  do {                                                                          \
    if (g_terms_out) {                                                          \
      (px)[0] = t_terms[0]; (px)[1] = t_terms[1]; (px)[2] = t_terms[2];          \
      (px)[3] = 1.0f;                                                           \
    }                                                                           \
  } while (0)
#define ORACLE_HAVE_TERMS 1
#endif

#define REAL float
#define FN(name) f32_##name
#define SQRT sqrtf
#define FABS fabsf
#define LOG cr_logf
#define POW cr_powf
#include "oracle_core.h"
#undef REAL
#undef FN
#undef SQRT
#undef FABS
#undef LOG
#undef POW

/* ---- fp64 twin ---- */
#define REAL double
#define FN(name) f64_##name
#define SQRT sqrt
#define FABS fabs
#define LOG log
#define POW pow
#include "oracle_core.h"

/* 4x4 inverse by cofactor expansion in double, rounded to float once.
 * GLSL inverse() precision is implementation-defined; this is the exact
 * inverse correctly rounded. */
static int invert4(const float* m, float* out) {
  double a[16], inv[16];
  for (int i = 0; i < 16; i++) a[i] = m[i];
  inv[0] = a[5] * a[10] * a[15] - a[5] * a[11] * a[14] - a[9] * a[6] * a[15] +
           a[9] * a[7] * a[14] + a[13] * a[6] * a[11] - a[13] * a[7] * a[10];
  inv[4] = -a[4] * a[10] * a[15] + a[4] * a[11] * a[14] + a[8] * a[6] * a[15] -
           a[8] * a[7] * a[14] - a[12] * a[6] * a[11] + a[12] * a[7] * a[10];
  inv[8] = a[4] * a[9] * a[15] - a[4] * a[11] * a[13] - a[8] * a[5] * a[15] +
           a[8] * a[7] * a[13] + a[12] * a[5] * a[11] - a[12] * a[7] * a[9];
  inv[12] = -a[4] * a[9] * a[14] + a[4] * a[10] * a[13] + a[8] * a[5] * a[14] -
            a[8] * a[6] * a[13] - a[12] * a[5] * a[10] + a[12] * a[6] * a[9];
  inv[1] = -a[1] * a[10] * a[15] + a[1] * a[11] * a[14] + a[9] * a[2] * a[15] -
           a[9] * a[3] * a[14] - a[13] * a[2] * a[11] + a[13] * a[3] * a[10];
  inv[5] = a[0] * a[10] * a[15] - a[0] * a[11] * a[14] - a[8] * a[2] * a[15] +
           a[8] * a[3] * a[14] + a[12] * a[2] * a[11] - a[12] * a[3] * a[10];
  inv[9] = -a[0] * a[9] * a[15] + a[0] * a[11] * a[13] + a[8] * a[1] * a[15] -
           a[8] * a[3] * a[13] - a[12] * a[1] * a[11] + a[12] * a[3] * a[9];
  inv[13] = a[0] * a[9] * a[14] - a[0] * a[10] * a[13] - a[8] * a[1] * a[14] +
            a[8] * a[2] * a[13] + a[12] * a[1] * a[10] - a[12] * a[2] * a[9];
  inv[2] = a[1] * a[6] * a[15] - a[1] * a[7] * a[14] - a[5] * a[2] * a[15] +
           a[5] * a[3] * a[14] + a[13] * a[2] * a[7] - a[13] * a[3] * a[6];
  inv[6] = -a[0] * a[6] * a[15] + a[0] * a[7] * a[14] + a[4] * a[2] * a[15] -
           a[4] * a[3] * a[14] - a[12] * a[2] * a[7] + a[12] * a[3] * a[6];
  inv[10] = a[0] * a[5] * a[15] - a[0] * a[7] * a[13] - a[4] * a[1] * a[15] +
            a[4] * a[3] * a[13] + a[12] * a[1] * a[7] - a[12] * a[3] * a[5];
  inv[14] = -a[0] * a[5] * a[14] + a[0] * a[6] * a[13] + a[4] * a[1] * a[14] -
            a[4] * a[2] * a[13] - a[12] * a[1] * a[6] + a[12] * a[2] * a[5];
  inv[3] = -a[1] * a[6] * a[11] + a[1] * a[7] * a[10] + a[5] * a[2] * a[11] -
           a[5] * a[3] * a[10] - a[9] * a[2] * a[7] + a[9] * a[3] * a[6];
  inv[7] = a[0] * a[6] * a[11] - a[0] * a[7] * a[10] - a[4] * a[2] * a[11] +
           a[4] * a[3] * a[10] + a[8] * a[2] * a[7] - a[8] * a[3] * a[6];
  inv[11] = -a[0] * a[5] * a[11] + a[0] * a[7] * a[9] + a[4] * a[1] * a[11] -
            a[4] * a[3] * a[9] - a[8] * a[1] * a[7] + a[8] * a[3] * a[5];
  inv[15] = a[0] * a[5] * a[10] - a[0] * a[6] * a[9] - a[4] * a[1] * a[10] +
            a[4] * a[2] * a[9] + a[8] * a[1] * a[6] - a[8] * a[2] * a[5];
  double det = a[0] * inv[0] + a[1] * inv[4] + a[2] * inv[8] + a[3] * inv[12];
  if (det == 0.0 || !isfinite(det)) return -1;
  for (int i = 0; i < 16; i++) out[i] = (float)(inv[i] / det);
  return 0;
}

static int make_uniforms(const sdf_camera* c, const sdf_params* p, oracle_uniforms* u) {
  if (invert4(c->view, u->inv_view) != 0) return SDF_E_INVALID_ARG;
  const float* m = u->inv_view;
  /* :180 camera.pos = (inverse(V_mat) * vec4(camera.pos, 1.0f)).xyz */
  for (int i = 0; i < 3; i++)
    u->cam[i] = m[i] * c->eye[0] + m[4 + i] * c->eye[1] + m[8 + i] * c->eye[2] + m[12 + i] * 1.0f;
  /* :191 -2.0f/tan(camera.fov*PI/360.0f), all in fp32 */
  float ang = c->fov_deg * c->pi / 360.0f;
  u->focal = -2.0f / tanf(ang);
  u->aspect = c->aspect > 0.0f ? c->aspect : (float)p->width / (float)p->height;
  return SDF_OK;
}

static int owned_rows(int height, const sdf_tiling* t) {
  int run = t->block_run > 1 ? t->block_run : 1;
  int step = t->run_step > 1 ? t->run_step : 1;
  if (t->block_rows <= 0 || t->block_stride <= 0 || t->first_block < 0 || t->block_run < 0 ||
      t->run_step < 0 || (long long)(run - 1) * step >= t->block_stride ||
      (step > 1 && t->block_rows % 8 != 0))
    return SDF_E_INVALID_ARG;
  int nblocks = (height + t->block_rows - 1) / t->block_rows;
  int rows = 0;
  /* blocks b >= first_block whose offset o = (b - first_block) % block_stride
     in the period is a multiple of step below run * step */
  for (int b = t->first_block; b < nblocks; b++) {
    int o = (b - t->first_block) % t->block_stride;
    if (o % step != 0 || o / step >= run) continue;
    int r = height - b * t->block_rows;
    rows += r < t->block_rows ? r : t->block_rows;
  }
  return rows;
}

int sdf_oracle_owned_rows(int height, const sdf_tiling* t) { return owned_rows(height, t); }

int sdf_oracle_defaults(sdf_scene* s, sdf_camera* c, sdf_light* l, sdf_material* m,
                        sdf_params* p, int width, int height) {
  if (s) {
    memset(s, 0, sizeof(*s));
    s->kind = SDF_SCENE_PRIMITIVES;
    s->count = 2;
    /* sceneSDF :73-81: plane first, then sphere, both hard min. */
    s->prims[0].kind = SDF_PRIM_PLANE;           /* planeSDF :66-71: p.y */
    s->prims[0].op = SDF_OP_UNION;
    s->prims[0].p[1] = 1.0f;
    s->prims[1].kind = SDF_PRIM_SPHERE;          /* sphereSDF :54-64 */
    s->prims[1].op = SDF_OP_UNION;
    s->prims[1].p[0] = 0.0f; s->prims[1].p[1] = 0.4f; s->prims[1].p[2] = 0.0f;
    s->prims[1].p[3] = 0.2f;
    s->bulb_scale = 1.0f;
    s->bulb_iterations = 12;
    s->bulb_bailout = 2.0f;
  }
  if (c) {
    memset(c, 0, sizeof(*c));
    /* main.cpp:7-11 orbit/pan start at 0 -> V_mat = identity (assumption
     * about Neutrino). */
    c->view[0] = c->view[5] = c->view[10] = c->view[15] = 1.0f;
    c->eye[0] = 0.0f; c->eye[1] = 0.2f; c->eye[2] = 2.0f;   /* :179 */
    c->fov_deg = 60.0f;                                      /* :178 */
    c->aspect = 0.0f;                                        /* AR = W/H */
    c->pi = 3.1415925359f;                                   /* :15 */
  }
  if (l) {
    memset(l, 0, sizeof(*l));
    l->pos[0] = 5.0f; l->pos[1] = 5.0f; l->pos[2] = 0.0f;   /* :182 */
    l->color[0] = l->color[1] = l->color[2] = 0.7f;         /* :183 */
    l->ambient = 0.1f;                                       /* :184 */
  }
  if (m) {
    memset(m, 0, sizeof(*m));
    m->amb[0] = 0.0f; m->amb[1] = 0.2f; m->amb[2] = 0.8f;   /* :186 */
    m->dif[0] = 0.0f; m->dif[1] = 0.2f; m->dif[2] = 0.8f;   /* :187 */
    m->ref[0] = m->ref[1] = m->ref[2] = 0.5f;               /* :188 */
    m->shininess = 12.0f;                                    /* :189 */
  }
  if (p) {
    memset(p, 0, sizeof(*p));
    p->width = width > 0 ? width : 800;                      /* main.cpp:4 */
    p->height = height > 0 ? height : 600;                   /* main.cpp:5 */
    p->max_steps = 100;                                      /* :17 */
    p->max_dist = 100.0f;                                    /* :18 */
    p->eps = 0.01f;                                          /* :19 */
    p->shadow_k = 10.0f;                                     /* :205 */
    p->normal_eps = 0.01f;                                   /* :21-23 */
    p->shadow_offset = 2.0f;                                 /* :205 */
    p->flags = SDF_FLAG_SHADOW;
    p->normal_mode = SDF_NORMAL_CENTRAL;
    p->ao_taps = 5;
    p->ao_step = 0.12f;
    p->ao_base = 0.01f;
    p->ao_falloff = 0.95f;
    p->ao_strength = 3.0f;
    p->precision = SDF_PRECISION_EXACT;
  }
  return SDF_OK;
}

static int render(int twin, const sdf_scene* s, const sdf_camera* c, const sdf_light* l,
                  const sdf_material* m, const sdf_params* p, const sdf_tiling* tiling,
                  float* rgba, int* steps, const int* force, int nthreads) {
  if (!s || !c || !l || !m || !p || !rgba) return SDF_E_INVALID_ARG;
  if (p->width <= 0 || p->height <= 0) return SDF_E_INVALID_ARG;
  sdf_tiling whole = {8, 0, 1, 0, 1, 1};
  const sdf_tiling* t = tiling ? tiling : &whole;
  int rows = owned_rows(p->height, t);
  if (rows < 0) return rows;
  oracle_uniforms u;
  int rc = make_uniforms(c, p, &u);
  if (rc) return rc;
  if (nthreads < 1) nthreads = 1;
  if (twin)
    f64_render_rows(s, l, m, p, &u, t, rows, rgba, steps, force, nthreads);
  else
    f32_render_rows(s, l, m, p, &u, t, rows, rgba, steps, force, nthreads);
  return SDF_OK;
}

int sdf_oracle_render(const sdf_scene* s, const sdf_camera* c, const sdf_light* l,
                      const sdf_material* m, const sdf_params* p, const sdf_tiling* t,
                      float* rgba, int* steps, int nthreads) {
  return render(0, s, c, l, m, p, t, rgba, steps, 0, nthreads);
}

int sdf_oracle_render_f64(const sdf_scene* s, const sdf_camera* c, const sdf_light* l,
                          const sdf_material* m, const sdf_params* p, const sdf_tiling* t,
                          float* rgba, int* steps, int nthreads) {
  return render(1, s, c, l, m, p, t, rgba, steps, 0, nthreads);
}

#ifdef ORACLE_HAVE_TERMS
/* The fp32 restatement's shading terms per pixel instead of its colour
 * (test infrastructure: the SHADE32F / TILES terms' reference). */
int sdf_oracle_render_terms(const sdf_scene* s, const sdf_camera* c, const sdf_light* l,
                            const sdf_material* m, const sdf_params* p, const sdf_tiling* t,
                            float* rgba, int nthreads) {
  g_terms_out = 1;
  const int rc = render(0, s, c, l, m, p, t, rgba, 0, 0, nthreads);
  g_terms_out = 0;
  return rc;
}
#endif

/* Forced-step replay: the fp32 restatement with each pixel's primary and
 * shadow marches run for exactly force[2i], force[2i+1] iterations (capped
 * at max_steps; oracle_core.h march_limit); pixels with force[2i] == -2 are
 * skipped and their rgba / steps left as the caller filled them. */
int sdf_oracle_replay(const sdf_scene* s, const sdf_camera* c, const sdf_light* l,
                      const sdf_material* m, const sdf_params* p, const sdf_tiling* t,
                      const int* force, float* rgba, int* steps, int nthreads) {
  if (!force) return SDF_E_INVALID_ARG;
  return render(0, s, c, l, m, p, t, rgba, steps, force, nthreads);
}

/* Scene-SDF probe for known-answer tests: d = sceneSDF(p) in fp32. */
float sdf_oracle_scene_sdf(const sdf_scene* s, float x, float y, float z) {
  return f32_scene_sdf(s, f32_mk(x, y, z));
}

/* Uniforms probe: writes inv_view[16], cam[3], focal, aspect (21 floats). */
int sdf_oracle_uniforms(const sdf_camera* c, const sdf_params* p, float* out21) {
  oracle_uniforms u;
  int rc = make_uniforms(c, p, &u);
  if (rc) return rc;
  memcpy(out21, u.inv_view, 16 * sizeof(float));
  memcpy(out21 + 16, u.cam, 3 * sizeof(float));
  out21[19] = u.focal;
  out21[20] = u.aspect;
  return SDF_OK;
}

/* Probes for known-answer tests (fp32 oracle internals). */
float sdf_oracle_raymarch(const sdf_scene* s, const sdf_params* p, const float* pos,
                          const float* dir, int* steps) {
  return f32_raymarch(s, p, f32_mk(pos[0], pos[1], pos[2]), f32_mk(dir[0], dir[1], dir[2]),
                      steps);
}

float sdf_oracle_shadow(const sdf_scene* s, const sdf_params* p, const float* pos,
                        const float* dir, float k, int* steps) {
  return f32_shadow(s, p, f32_mk(pos[0], pos[1], pos[2]), f32_mk(dir[0], dir[1], dir[2]), k,
                    steps);
}

void sdf_oracle_normal(const sdf_scene* s, const sdf_params* p, const float* pos, float* out) {
  f32_v3 q = f32_mk(pos[0], pos[1], pos[2]);
  f32_v3 n = p->normal_mode == SDF_NORMAL_TETRA ? f32_normal_tetra(s, q, p->normal_eps)
                                                : f32_normal_central(s, q, p->normal_eps);
  out[0] = n.x; out[1] = n.y; out[2] = n.z;
}

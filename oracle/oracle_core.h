/*
 * oracle_core.h -- TEST INFRASTRUCTURE ONLY (the CPU oracle).
 *
 * Scalar CPU restatement of the reference fragment shader
 * /root/reference/Code/shader/voxel_fragment.frag (ezorzin/SDF3D @ 2025-01-17)
 * and of the pixel -> `quad` mapping of voxel_geometry.geom:26-52, with the
 * GLSL 4.60 semantics listed in SURVEY.md Appendix A (select-based min/max/
 * clamp, normalize(v) = v / length(v), left-to-right dot products, loop
 * breaks tested after the state update).
 *
 * This header is included twice by sdf_oracle.c: once with REAL = float (the
 * oracle proper, compiled -ffp-contract=off, no fast-math) and once with
 * REAL = double (the fp64 twin used only to diagnose branch flips).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load the compiled oracle, and only as the checker / CPU baseline.  The
 * product path (sdf3d_amd, libsdf3d.so) never links or calls it.
 *
 * Parity status: the reference's device code is GLSL with no tests, fixtures
 * or golden images, and it cannot be compiled or run in this environment (no
 * GLSL compiler, no headless GL).  The reference-scene
 * path below is therefore pinned only by analytic known-answer tests
 * (tests/test_oracle_kat.py) and is otherwise "parity unpinned" against
 * reference-produced outputs.  The extension features (smooth-min CSG, extra
 * primitives, tetrahedral normals, AO, Mandelbulb) have no reference at all;
 * their formulas are frozen in DESIGN.md "Scene spec" and here.
 */

#ifndef REAL
#error "define REAL before including oracle_core.h"
#endif
#ifndef FN
#error "define FN(name) before including oracle_core.h"
#endif

typedef struct { REAL x, y, z; } FN(v3);

static inline FN(v3) FN(mk)(REAL x, REAL y, REAL z) { FN(v3) r = {x, y, z}; return r; }
static inline FN(v3) FN(add)(FN(v3) a, FN(v3) b) { return FN(mk)(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline FN(v3) FN(sub)(FN(v3) a, FN(v3) b) { return FN(mk)(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline FN(v3) FN(muls)(FN(v3) a, REAL s) { return FN(mk)(a.x * s, a.y * s, a.z * s); }
/* GLSL dot, summed left to right. */
static inline REAL FN(dot)(FN(v3) a, FN(v3) b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline REAL FN(length)(FN(v3) a) { return SQRT(FN(dot)(a, a)); }
/* GLSL normalize(v) = v / length(v). */
static inline FN(v3) FN(normalize)(FN(v3) a) {
  REAL l = FN(length)(a);
  return FN(mk)(a.x / l, a.y / l, a.z / l);
}
/* GLSL 4.60: min(x,y) = y < x ? y : x; max(x,y) = x < y ? y : x;
 * clamp(x,a,b) = min(max(x,a),b)  (SURVEY.md Appendix A). */
static inline REAL FN(gmin)(REAL x, REAL y) { return y < x ? y : x; }
static inline REAL FN(gmax)(REAL x, REAL y) { return x < y ? y : x; }
static inline REAL FN(gclamp)(REAL x, REAL a, REAL b) { return FN(gmin)(FN(gmax)(x, a), b); }

/* ---- primitives ----------------------------------------------------------- */

/* sphereSDF, voxel_fragment.frag:54-64: length(position - s) - r. */
static inline REAL FN(sd_sphere)(FN(v3) p, const float* q) {
  FN(v3) c = FN(mk)(q[0], q[1], q[2]);
  return FN(length)(FN(sub)(p, c)) - (REAL)q[3];
}

/* planeSDF, voxel_fragment.frag:66-71 is position.y; generalised to
 * dot(p, n) + h, which equals p.y for n = (0,1,0), h = 0. */
static inline REAL FN(sd_plane)(FN(v3) p, const float* q) {
  FN(v3) n = FN(mk)(q[0], q[1], q[2]);
  return FN(dot)(p, n) + (REAL)q[3];
}

/* Extension (DESIGN.md Scene spec): axis-aligned box,
 * q = |p - c| - b; length(max(q,0)) + min(max(q.x, max(q.y, q.z)), 0). */
static inline REAL FN(box_core)(FN(v3) v, REAL bx, REAL by, REAL bz) {
  REAL qx = FABS(v.x) - bx, qy = FABS(v.y) - by, qz = FABS(v.z) - bz;
  FN(v3) o = FN(mk)(FN(gmax)(qx, 0), FN(gmax)(qy, 0), FN(gmax)(qz, 0));
  REAL outside = FN(length)(o);
  REAL inside = FN(gmin)(FN(gmax)(qx, FN(gmax)(qy, qz)), 0);
  return outside + inside;
}
static inline REAL FN(sd_box)(FN(v3) p, const float* q) {
  FN(v3) v = FN(sub)(p, FN(mk)(q[0], q[1], q[2]));
  return FN(box_core)(v, q[3], q[4], q[5]);
}
/* Extension: rounded box = box with half extents (b - r), minus r. */
static inline REAL FN(sd_round_box)(FN(v3) p, const float* q) {
  FN(v3) v = FN(sub)(p, FN(mk)(q[0], q[1], q[2]));
  REAL r = q[6];
  return FN(box_core)(v, (REAL)q[3] - r, (REAL)q[4] - r, (REAL)q[5] - r) - r;
}
/* Extension: torus in the xz plane: length((length(v.xz) - R, v.y)) - r. */
static inline REAL FN(sd_torus)(FN(v3) p, const float* q) {
  FN(v3) v = FN(sub)(p, FN(mk)(q[0], q[1], q[2]));
  REAL lxz = SQRT(v.x * v.x + v.z * v.z);
  REAL qx = lxz - (REAL)q[3];
  return SQRT(qx * qx + v.y * v.y) - (REAL)q[4];
}
/* Extension: capsule a-b radius r:
 * h = clamp(dot(pa,ba)/dot(ba,ba), 0, 1); length(pa - ba*h) - r. */
static inline REAL FN(sd_capsule)(FN(v3) p, const float* q) {
  FN(v3) a = FN(mk)(q[0], q[1], q[2]);
  FN(v3) b = FN(mk)(q[3], q[4], q[5]);
  FN(v3) pa = FN(sub)(p, a), ba = FN(sub)(b, a);
  REAL h = FN(gclamp)(FN(dot)(pa, ba) / FN(dot)(ba, ba), 0, 1);
  return FN(length)(FN(sub)(pa, FN(muls)(ba, h))) - (REAL)q[6];
}
/* Extension: capped y-axis cylinder radius r, half height hh:
 * d = (length(v.xz) - r, |v.y| - hh); min(max(d.x,d.y),0) + length(max(d,0)). */
static inline REAL FN(sd_cylinder)(FN(v3) p, const float* q) {
  FN(v3) v = FN(sub)(p, FN(mk)(q[0], q[1], q[2]));
  REAL dx = SQRT(v.x * v.x + v.z * v.z) - (REAL)q[3];
  REAL dy = FABS(v.y) - (REAL)q[4];
  REAL inside = FN(gmin)(FN(gmax)(dx, dy), 0);
  REAL ox = FN(gmax)(dx, 0), oy = FN(gmax)(dy, 0);
  return inside + SQRT(ox * ox + oy * oy);
}

/* Polynomial smooth-min (extension): h = max(k - |a-b|, 0) / k;
 * min(a,b) - h*h*k*0.25.  Equals min(a,b) exactly when |a-b| >= k. */
static inline REAL FN(smin)(REAL a, REAL b, REAL k) {
  REAL h = FN(gmax)(k - FABS(a - b), 0) / k;
  return FN(gmin)(a, b) - h * h * k * (REAL)0.25;
}

/* Power-8 Mandelbulb distance estimator, trig-free polynomial form
 * (extension, DESIGN.md Scene spec).  Local coordinates q; returns the DE. */
static inline REAL FN(mandelbulb)(FN(v3) q, int iters, REAL bail2) {
  FN(v3) w = q;
  REAL m = FN(dot)(w, w);
  REAL dz = 1;
  for (int i = 0; i < iters; i++) {
    REAL m2 = m * m;
    REAL m4 = m2 * m2;
    dz = (REAL)8 * SQRT(m4 * m2 * m) * dz + (REAL)1;
    REAL x = w.x, x2 = x * x, x4 = x2 * x2;
    REAL y = w.y, y2 = y * y, y4 = y2 * y2;
    REAL z = w.z, z2 = z * z, z4 = z2 * z2;
    /* iq's trig-free power-8 map, with the x/z factors taken in xz-normalised
     * coordinates (xn, zn) = (x, z) / sqrt(k3): the same polynomial without
     * the fp32 underflow of inversesqrt(k3^7) near the y axis. */
    REAL k3 = FN(gmax)(x2 + z2, (REAL)1e-30f);
    REAL r = (REAL)1 / SQRT(k3);
    REAL s = k3 * r;
    REAL xn = x * r, zn = z * r;
    REAL xn2 = xn * xn, zn2 = zn * zn, xn4 = xn2 * xn2, zn4 = zn2 * zn2;
    REAL k1 = x4 + y4 + z4 - (REAL)6 * y2 * z2 - (REAL)6 * x2 * y2 + (REAL)2 * z2 * x2;
    REAL k4 = x2 - y2 + z2;
    REAL yk = y * k4 * k1;
    w.x = q.x + (REAL)64 * yk * xn * zn * (xn2 - zn2) * (xn4 - (REAL)6 * xn2 * zn2 + zn4) * s;
    w.y = q.y + (REAL)-16 * y2 * k3 * k4 * k4 + k1 * k1;
    w.z = q.z + (REAL)-8 * yk *
                    (xn4 * xn4 - (REAL)28 * xn4 * xn2 * zn2 + (REAL)70 * xn4 * zn4 -
                     (REAL)28 * xn2 * zn2 * zn4 + zn4 * zn4) * s;
    m = FN(dot)(w, w);
    if (m > bail2) {
#ifdef ORACLE_BULB_ITER_HOOK
      ORACLE_BULB_ITER_HOOK(i + 1);
#endif
      return (REAL)0.25 * LOG(m) * SQRT(m) / dz;
    }
  }
#ifdef ORACLE_BULB_ITER_HOOK
  ORACLE_BULB_ITER_HOOK(iters);
#endif
  return (REAL)0.25 * LOG(m) * SQRT(m) / dz;
}

/* sceneSDF, voxel_fragment.frag:73-81: sdf = INF, then one combine per
 * primitive (the reference: min(min(INF, plane), sphere)). */
static REAL FN(scene_sdf)(const sdf_scene* s, FN(v3) p) {
  if (s->kind == SDF_SCENE_MANDELBULB) {
    REAL sc = s->bulb_scale;
    FN(v3) q = FN(mk)((p.x - (REAL)s->bulb_center[0]) / sc,
                      (p.y - (REAL)s->bulb_center[1]) / sc,
                      (p.z - (REAL)s->bulb_center[2]) / sc);
    /* Outside the bounding sphere |q| = 1.5 the set (radius < 1.25) is at
     * least |q| - 1.25 away: return that bound (keeps the polynomial DE away
     * from fp32 overflow far from the set). */
    REAL m0 = FN(dot)(q, q);
    if (m0 > (REAL)2.25) {
#ifdef ORACLE_BULB_ITER_HOOK
      ORACLE_BULB_ITER_HOOK(0);   /* outside the bounding sphere: no map iterations */
#endif
      return (SQRT(m0) - (REAL)1.25) * sc;
    }
    REAL bail = s->bulb_bailout;
    return FN(mandelbulb)(q, s->bulb_iterations, bail * bail) * sc;
  }
  REAL d = (REAL)INFINITY;  /* INF = 1.0f/0.0f, :20, :75 */
  for (int i = 0; i < s->count; i++) {
    const sdf_primitive* pr = &s->prims[i];
    REAL v;
    switch (pr->kind) {
      case SDF_PRIM_SPHERE: v = FN(sd_sphere)(p, pr->p); break;
      case SDF_PRIM_PLANE: v = FN(sd_plane)(p, pr->p); break;
      case SDF_PRIM_BOX: v = FN(sd_box)(p, pr->p); break;
      case SDF_PRIM_ROUND_BOX: v = FN(sd_round_box)(p, pr->p); break;
      case SDF_PRIM_TORUS: v = FN(sd_torus)(p, pr->p); break;
      case SDF_PRIM_CAPSULE: v = FN(sd_capsule)(p, pr->p); break;
      default: v = FN(sd_cylinder)(p, pr->p); break;
    }
    REAL k = pr->k;
    switch (pr->op) {
      case SDF_OP_UNION: d = FN(gmin)(d, v); break;              /* :77-78 */
      case SDF_OP_SMOOTH_UNION: d = FN(smin)(d, v, k); break;
      case SDF_OP_SUBTRACT: d = FN(gmax)(d, -v); break;
      case SDF_OP_INTERSECT: d = FN(gmax)(d, v); break;
      case SDF_OP_SMOOTH_SUBTRACT: d = -FN(smin)(-d, v, k); break;
      default: d = -FN(smin)(-d, -v, k); break;                  /* SMOOTH_INTERSECT */
    }
  }
  return d;
}

/* Forced-step REPLAY (diagnosis only, tests/parity.py): force >= 0 imposes
 * the march's break point -- exactly min(force, max_steps) iterations, the
 * break test ignored -- so the oracle can be evaluated at the step counts a
 * kernel recorded; force < 0 is the shader's own loop. */
static inline int FN(march_limit)(int max_steps, int force) {
  return (force >= 0 && force < max_steps) ? force : max_steps;
}

/* raymarch, voxel_fragment.frag:86-103.  The break test comes after the
 * increment (:97-99); there is no miss branch. */
static REAL FN(raymarch_n)(const sdf_scene* s, const sdf_params* pa, FN(v3) pos,
                           FN(v3) dir, int force, int32_t* steps) {
  REAL distance = 0;
  REAL max_dist = pa->max_dist, eps = pa->eps;
  int i, n = FN(march_limit)(pa->max_steps, force);
  for (i = 0; i < n; i++) {
    FN(v3) ray = FN(add)(pos, FN(muls)(dir, distance));
    REAL sdf = FN(scene_sdf)(s, ray);
    distance += sdf;
    if (force < 0 && (distance > max_dist || sdf < eps)) { i++; break; }
  }
  *steps = i;
  return distance;
}
static REAL FN(raymarch)(const sdf_scene* s, const sdf_params* pa, FN(v3) pos,
                         FN(v3) dir, int32_t* steps) {
  return FN(raymarch_n)(s, pa, pos, dir, -1, steps);
}

/* shadow, voxel_fragment.frag:105-132 ("improved" soft shadow).  At i == 0
 * the candidate is k*h/max(0, 0) = +inf. */
static REAL FN(shadow_n)(const sdf_scene* s, const sdf_params* pa, FN(v3) pos,
                         FN(v3) dir, REAL k, int force, int32_t* steps) {
  REAL distance = 0;
  REAL sdf = (REAL)INFINITY;
  REAL shadow = 1;
  REAL max_dist = pa->max_dist, eps = pa->eps;
  int i, n = FN(march_limit)(pa->max_steps, force);
  for (i = 0; i < n; i++) {
    FN(v3) ray = FN(add)(pos, FN(muls)(dir, distance));
    REAL sdf_new = FN(scene_sdf)(s, ray);
    REAL intersection = (i == 0) ? (REAL)0 : sdf_new * sdf_new / ((REAL)2 * sdf);
    REAL d_est = SQRT(sdf_new * sdf_new - intersection * intersection);
    shadow = FN(gmin)(shadow, k * d_est / FN(gmax)(0, distance - intersection));
    sdf = sdf_new;
    distance += sdf_new;
    if (force < 0 && (distance > max_dist || shadow < eps)) { i++; break; }
  }
  *steps = i;
  return FN(gclamp)(shadow, 0, 1);
}
static REAL FN(shadow)(const sdf_scene* s, const sdf_params* pa, FN(v3) pos,
                       FN(v3) dir, REAL k, int32_t* steps) {
  return FN(shadow_n)(s, pa, pos, dir, k, -1, steps);
}

/* normal, voxel_fragment.frag:134-155: 6-tap central differences. */
static FN(v3) FN(normal_central)(const sdf_scene* s, FN(v3) p, REAL h) {
  REAL L, R, nx, ny, nz;
  L = FN(scene_sdf)(s, FN(mk)(p.x - h, p.y, p.z));
  R = FN(scene_sdf)(s, FN(mk)(p.x + h, p.y, p.z));
  nx = R - L;
  L = FN(scene_sdf)(s, FN(mk)(p.x, p.y - h, p.z));
  R = FN(scene_sdf)(s, FN(mk)(p.x, p.y + h, p.z));
  ny = R - L;
  L = FN(scene_sdf)(s, FN(mk)(p.x, p.y, p.z - h));
  R = FN(scene_sdf)(s, FN(mk)(p.x, p.y, p.z + h));
  nz = R - L;
  return FN(normalize)(FN(mk)(nx, ny, nz));
}

/* Extension: 4-tap tetrahedral differences, taps e0 = (1,-1,-1),
 * e1 = (-1,-1,1), e2 = (-1,1,-1), e3 = (1,1,1); n = sum e_i f(p + e_i h). */
static FN(v3) FN(normal_tetra)(const sdf_scene* s, FN(v3) p, REAL h) {
  REAL f0 = FN(scene_sdf)(s, FN(mk)(p.x + h, p.y - h, p.z - h));
  REAL f1 = FN(scene_sdf)(s, FN(mk)(p.x - h, p.y - h, p.z + h));
  REAL f2 = FN(scene_sdf)(s, FN(mk)(p.x - h, p.y + h, p.z - h));
  REAL f3 = FN(scene_sdf)(s, FN(mk)(p.x + h, p.y + h, p.z + h));
  REAL nx = f0 - f1 - f2 + f3;
  REAL ny = -f0 - f1 + f2 + f3;
  REAL nz = -f0 + f1 - f2 + f3;
  return FN(normalize)(FN(mk)(nx, ny, nz));
}

/* Extension: n-tap ambient occlusion along the normal. */
static REAL FN(ambient_occlusion)(const sdf_scene* s, const sdf_params* pa,
                                  FN(v3) p, FN(v3) n) {
  REAL occ = 0, sca = 1;
  int taps = pa->ao_taps;
  for (int i = 0; i < taps; i++) {
    REAL t = taps > 1 ? (REAL)i / (REAL)(taps - 1) : (REAL)0;
    REAL h = (REAL)pa->ao_base + (REAL)pa->ao_step * t;
    REAL d = FN(scene_sdf)(s, FN(add)(p, FN(muls)(n, h)));
    occ = occ + (h - d) * sca;
    sca = sca * (REAL)pa->ao_falloff;
  }
  return FN(gclamp)((REAL)1 - (REAL)pa->ao_strength * occ, 0, 1);
}

/* Fragment stage main(), voxel_fragment.frag:160-211, for one pixel.
 * cam / ray come from the caller (uniform work hoisted, :180, :191-192).
 * `force` (replay only): NULL, or the (primary, shadow) break points to
 * impose (march_limit). */
static void FN(shade_pixel)(const sdf_scene* s, const sdf_light* li,
                            const sdf_material* M, const sdf_params* pa,
                            FN(v3) cam, FN(v3) ray, float* out, int32_t* st,
                            const int32_t* force) {
  int32_t sp = 0, ss = 0;
  REAL d = FN(raymarch_n)(s, pa, cam, ray, force ? force[0] : -1, &sp); /* :195 */
  FN(v3) P = FN(add)(cam, FN(muls)(ray, d));                       /* :196 */
  FN(v3) N = pa->normal_mode == SDF_NORMAL_TETRA                   /* :197 */
                 ? FN(normal_tetra)(s, P, pa->normal_eps)
                 : FN(normal_central)(s, P, pa->normal_eps);
  FN(v3) L = FN(mk)(li->pos[0], li->pos[1], li->pos[2]);
  FN(v3) view = FN(normalize)(FN(sub)(cam, P));                    /* :200 */
  FN(v3) incident = FN(normalize)(FN(sub)(L, P));                  /* :201 */
  FN(v3) halfway = FN(normalize)(FN(add)(incident, view));         /* :203 */
  REAL spec = POW(FN(gmax)(FN(dot)(N, halfway), 0), (REAL)M->shininess); /* :204 */
  REAL sh = 1;
  if (pa->flags & SDF_FLAG_SHADOW) {                               /* :205 */
    REAL off = pa->shadow_offset, eps = pa->eps;
    FN(v3) o = FN(mk)(P.x + N.x * off * eps, P.y + N.y * off * eps, P.z + N.z * off * eps);
    sh = FN(shadow_n)(s, pa, o, incident, (REAL)pa->shadow_k, force ? force[1] : -1, &ss);
  }
#ifdef ORACLE_PIXEL_HOOK
  ORACLE_PIXEL_HOOK(FN(dot)(N, incident) > 0);   /* instrumentation (tools/) only */
#endif
  REAL dif = FN(gclamp)(FN(dot)(N, incident), 0, 1) * sh;         /* :205 */
  REAL la = li->ambient;
  REAL amb[3] = {la * (REAL)M->amb[0], la * (REAL)M->amb[1], la * (REAL)M->amb[2]}; /* :206 */
  if ((pa->flags & SDF_FLAG_AO) && pa->ao_taps > 0) {
    REAL ao = FN(ambient_occlusion)(s, pa, P, N);
    amb[0] = amb[0] * ao; amb[1] = amb[1] * ao; amb[2] = amb[2] * ao;
#ifdef ORACLE_TERMS_HOOK
    ORACLE_TERMS_HOOK(ao, dif, spec, FN(gmax)(FN(dot)(N, halfway), 0), FN(gclamp)(FN(dot)(N, incident), 0, 1), sh);   /* instrumentation (tools/) only */
  } else {
    ORACLE_TERMS_HOOK(1, dif, spec, FN(gmax)(FN(dot)(N, halfway), 0), FN(gclamp)(FN(dot)(N, incident), 0, 1), sh);
#endif
  }
  for (int c = 0; c < 3; c++)                                      /* :207-210 */
    out[c] = (float)(amb[c] + dif * (REAL)M->dif[c] + spec * (REAL)M->ref[c]);
  out[3] = 1.0f;
  if (st) { st[0] = sp; st[1] = ss; }
}

/* Render the rows owned by `t` (packed order) on the host.  `force`
 * (replay only; NULL otherwise): per-pixel (primary, shadow) break points,
 * laid out like `steps`; a pixel whose primary entry is -2 is skipped (its
 * outputs are left untouched), so a replay can visit only the pixels a test
 * needs. */
static void FN(render_rows)(const sdf_scene* s, const sdf_light* li,
                            const sdf_material* M, const sdf_params* pa,
                            const oracle_uniforms* u, const sdf_tiling* t,
                            int rows, float* rgba, int32_t* steps,
                            const int32_t* force, int nthreads) {
  int W = pa->width, H = pa->height;
  (void)nthreads;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) if (nthreads > 1)
  for (int pr = 0; pr < rows; pr++) {
    /* period blk, row `within` of its run of blocks (sdf_abi.h sdf_tiling) */
    int run = t->block_run > 1 ? t->block_run : 1;
    int step = t->run_step > 1 ? t->run_step : 1;
    int blk = pr / (run * t->block_rows), within = pr % (run * t->block_rows);
    int j = within / t->block_rows;   /* the run's j-th block, step blocks apart */
    int y = (t->first_block + blk * t->block_stride + j * step) * t->block_rows +
            within % t->block_rows;
    (void)H;
    /* quad.y = (2y+1)/H - 1 (voxel_geometry.geom:26-52 + GL raster). */
    float qy = (float)(2 * y + 1) / (float)H - 1.0f;
    for (int x = 0; x < W; x++) {
      const int32_t* fo = force ? force + 2 * ((size_t)pr * W + x) : 0;
      if (fo && fo[0] == -2) continue;
      float qx = (float)(2 * x + 1) / (float)W - 1.0f;
      /* :191 ray = normalize(vec3(quad.x*AR, quad.y, focal)) */
      FN(v3) r0 = FN(normalize)(FN(mk)((REAL)qx * (REAL)u->aspect, qy, u->focal));
      /* :192 ray = normalize((inverse(V_mat) * vec4(ray, 0)).xyz) */
      const float* m = u->inv_view;
      FN(v3) r1 = FN(mk)(m[0] * r0.x + m[4] * r0.y + m[8] * r0.z + m[12] * (REAL)0,
                         m[1] * r0.x + m[5] * r0.y + m[9] * r0.z + m[13] * (REAL)0,
                         m[2] * r0.x + m[6] * r0.y + m[10] * r0.z + m[14] * (REAL)0);
      FN(v3) ray = FN(normalize)(r1);
      FN(v3) cam = FN(mk)(u->cam[0], u->cam[1], u->cam[2]);
      size_t o = (size_t)pr * W + x;
      FN(shade_pixel)(s, li, M, pa, cam, ray, rgba + 4 * o, steps ? steps + 2 * o : 0, fo);
#ifdef ORACLE_PIXEL_OUT_HOOK
      ORACLE_PIXEL_OUT_HOOK(rgba + 4 * o);   /* sdf_oracle_render_terms only */
#endif
    }
  }
}

/*
 * bulb_divergence.c -- MEASUREMENT TOOL (not product, not a test): where the
 * Mandelbulb kernel's idle lanes come from, and what re-packing live rays
 * through LDS (the "ray compaction" north_star names)
 * could at best recover.
 *
 * It runs the CPU oracle (oracle/oracle_core.h, via oracle/sdf_oracle.c) on
 * the C5 frame with two instrumentation hooks that are no-ops in every other
 * build: ORACLE_BULB_ITER_HOOK records the number of map iterations of every
 * distance-estimator call (0 outside the bounding sphere), ORACLE_PIXEL_HOOK
 * whether N.L > 0 (the kernel skips the shadow march otherwise).  Per 8x8
 * tile -- one wave64 of the kernel -- it then replays SIMT execution of the
 * kernel's stages in lockstep (primary march, 4 normal taps, 5 AO taps, the
 * shadow march of the lanes with N.L > 0) with a per-phase instruction cost
 * model of the fast kernel (wave-instructions per march step, per map
 * prologue/epilogue, per map iteration, per cheap outside-the-sphere DE):
 *
 *   actual     : lanes that finished their march idle until the wave's last
 *                one does; inside a DE the map loop runs the active lanes'
 *                largest iteration count, lanes that bailed out idle;
 *   compacted  : IDEAL ray compaction -- the tile's DE calls of a stage are
 *                re-packed 64 at a time in step order (every lane busy at
 *                every march step, repacking itself free), the map loop still
 *                runs each pack's largest iteration count;
 *   inner_only : the opposite bound -- march divergence kept, map iterations
 *                perfectly packed (no bailout divergence).
 *
 * Prints JSON: lane utilisation (active lanes x instructions / 64 x
 * instructions, the quantity PMC's SQ_THREAD_CYCLES_VALU / 64
 * SQ_ACTIVE_INST_VALU measures) and wave-instruction totals per scenario.
 *
 *   gcc -O2 -fopenmp -Iinclude tools/bulb_divergence.c -o /tmp/bd -lm &&
 *   /tmp/bd [width height row_stride]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define MAXT 4096
static __thread int t_trace[MAXT];
static __thread int t_n;
static __thread int t_lit;
#define ORACLE_BULB_ITER_HOOK(k) (t_n < MAXT ? (void)(t_trace[t_n++] = (k)) : (void)0)
#define ORACLE_PIXEL_HOOK(lit) (t_lit = (lit))

#include "../oracle/sdf_oracle.c"

/* fast-kernel wave-instruction costs per phase (render_kernel.inc, fast
 * precision; VALU counts read off the ISA, rounded) */
#define C_STEP 12   /* march step: position, t update, break tests, loop */
#define C_OUT 8     /* DE outside the bounding sphere: sqrt, sub, mul */
#define C_MAP 26    /* map prologue + epilogue: q, m, log, sqrt, rcp, muls */
#define C_ITER 47   /* one map iteration */

typedef struct { double lanes, instr, calls; } Acc;   /* sum(active x instr), sum(instr), DE calls */

static void add(Acc* a, int active, double instr) {
  if (active <= 0) return;
  a->lanes += active * instr;
  a->instr += instr;
}

/* one lockstep DE call over `n` lanes with iteration counts it[] (-1 =
 * lane not taking part) */
static void de_call(Acc* a, const int* it, int n, int pack_inner) {
  int act = 0, outside = 0, inside = 0, maxit = 0, sumit = 0;
  for (int l = 0; l < n; l++) {
    if (it[l] < 0) continue;
    act++;
    if (it[l] == 0) outside++;
    else {
      inside++;
      if (it[l] > maxit) maxit = it[l];
      sumit += it[l];
    }
  }
  if (act > 0) a->calls += 1;
  add(a, act, C_STEP);
  add(a, outside, C_OUT);
  add(a, inside, C_MAP);
  if (pack_inner) {
    /* iterations re-packed 64 at a time */
    for (int left = sumit; left > 0; left -= 64) add(a, left < 64 ? left : 64, C_ITER);
  } else {
    for (int j = 0; j < maxit; j++) {
      int on = 0;
      for (int l = 0; l < n; l++)
        if (it[l] > j) on++;
      add(a, on, C_ITER);
    }
  }
}

int main(int argc, char** argv) {
  int W = argc > 1 ? atoi(argv[1]) : 3840, H = argc > 2 ? atoi(argv[2]) : 2160;
  int stride = argc > 3 ? atoi(argv[3]) : 8;  /* every stride-th tile row */
  sdf_scene s; sdf_camera c; sdf_light l; sdf_material m; sdf_params p;
  sdf_oracle_defaults(&s, &c, &l, &m, &p, W, H);
  /* C5 (sdf3d_amd/scenes.py config("C5")) */
  s.kind = SDF_SCENE_MANDELBULB; s.count = 0;
  s.bulb_center[0] = 0.0f; s.bulb_center[1] = 0.3f; s.bulb_center[2] = 0.0f;
  s.bulb_scale = 0.45f; s.bulb_iterations = 12; s.bulb_bailout = 2.0f;
  p.max_steps = 128; p.flags = SDF_FLAG_SHADOW | SDF_FLAG_AO; p.normal_mode = SDF_NORMAL_TETRA;
  oracle_uniforms u;
  if (make_uniforms(&c, &p, &u)) return 1;
  const int tx = (W + 7) / 8, ty = (H + 7) / 8;
  double res[3][3] = {{0}};
  long tiles = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : tiles)
  for (int tyi = 0; tyi < ty; tyi += stride) {
    /* per pixel of one tile row: traces */
    static __thread int tr[64][MAXT];
    static __thread int nt[64], sp[64], ss[64], lit[64];
    for (int txi = 0; txi < tx; txi++) {
      int n = 0;
      for (int k = 0; k < 64; k++) {
        int x = txi * 8 + (k & 7), y = tyi * 8 + (k >> 3);
        nt[k] = -1;
        if (x >= W || y >= H) continue;
        float qy = (float)(2 * y + 1) / (float)H - 1.0f;
        float qx = (float)(2 * x + 1) / (float)W - 1.0f;
        f32_v3 r0 = f32_normalize(f32_mk(qx * u.aspect, qy, u.focal));
        const float* mm = u.inv_view;
        f32_v3 r1 = f32_mk(mm[0] * r0.x + mm[4] * r0.y + mm[8] * r0.z,
                           mm[1] * r0.x + mm[5] * r0.y + mm[9] * r0.z,
                           mm[2] * r0.x + mm[6] * r0.y + mm[10] * r0.z);
        f32_v3 ray = f32_normalize(r1);
        f32_v3 cam = f32_mk(u.cam[0], u.cam[1], u.cam[2]);
        float out[4];
        int st[2];
        t_n = 0;
        f32_shade_pixel(&s, &l, &m, &p, cam, ray, out, st, 0);
        memcpy(tr[k], t_trace, sizeof(int) * t_n);
        nt[k] = t_n; sp[k] = st[0]; ss[k] = st[1]; lit[k] = t_lit;
        n++;
      }
      if (!n) continue;
      tiles++;
      /* stage slices of each lane's trace: [sp primary][4 normal][ss shadow][5 AO] */
      for (int scen = 0; scen < 3; scen++) {
        Acc a = {0, 0, 0};
        int it[64];
        /* primary march */
        int maxs = 0;
        for (int k = 0; k < 64; k++) if (nt[k] >= 0 && sp[k] > maxs) maxs = sp[k];
        if (scen == 1) {
          /* ideal compaction: the tile's primary DE calls in step order, 64 a pack */
          int total = 0;
          for (int s_ = 0; s_ < maxs; s_++)
            for (int k = 0; k < 64; k++) if (nt[k] >= 0 && sp[k] > s_) total++;
          int pack[64], np = 0;
          for (int s_ = 0; s_ < maxs; s_++)
            for (int k = 0; k < 64; k++) {
              if (nt[k] < 0 || sp[k] <= s_) continue;
              pack[np++] = tr[k][s_];
              if (np == 64) { de_call(&a, pack, 64, 0); np = 0; }
            }
          if (np) { for (int k = np; k < 64; k++) pack[k] = -1; de_call(&a, pack, 64, 0); }
          (void)total;
        } else {
          for (int s_ = 0; s_ < maxs; s_++) {
            for (int k = 0; k < 64; k++) it[k] = (nt[k] >= 0 && sp[k] > s_) ? tr[k][s_] : -1;
            de_call(&a, it, 64, scen == 2);
          }
        }
        /* 4 normal taps + 5 AO taps: every lane, lockstep */
        for (int j = 0; j < 9; j++) {
          for (int k = 0; k < 64; k++) {
            if (nt[k] < 0) { it[k] = -1; continue; }
            int idx = j < 4 ? sp[k] + j : sp[k] + 4 + ss[k] + (j - 4);
            it[k] = tr[k][idx];
          }
          de_call(&a, it, 64, scen == 2);
        }
        /* shadow march: lanes with N.L > 0 (the kernel skips the others) */
        int maxh = 0;
        for (int k = 0; k < 64; k++) if (nt[k] >= 0 && lit[k] && ss[k] > maxh) maxh = ss[k];
        if (scen == 1) {
          int pack[64], np = 0;
          for (int s_ = 0; s_ < maxh; s_++)
            for (int k = 0; k < 64; k++) {
              if (nt[k] < 0 || !lit[k] || ss[k] <= s_) continue;
              pack[np++] = tr[k][sp[k] + 4 + s_];
              if (np == 64) { de_call(&a, pack, 64, 0); np = 0; }
            }
          if (np) { for (int k = np; k < 64; k++) pack[k] = -1; de_call(&a, pack, 64, 0); }
        } else {
          for (int s_ = 0; s_ < maxh; s_++) {
            for (int k = 0; k < 64; k++)
              it[k] = (nt[k] >= 0 && lit[k] && ss[k] > s_) ? tr[k][sp[k] + 4 + s_] : -1;
            de_call(&a, it, 64, scen == 2);
          }
        }
#pragma omp atomic
        res[scen][0] += a.lanes;
#pragma omp atomic
        res[scen][1] += a.instr;
#pragma omp atomic
        res[scen][2] += a.calls;
      }
    }
  }
  const char* name[3] = {"actual", "compacted", "inner_only"};
  printf("{\"config\": \"C5 %dx%d, every %dth tile row (%ld tiles)\", \"costs\": "
         "{\"step\": %d, \"outside\": %d, \"map\": %d, \"iter\": %d}",
         W, H, stride, tiles, C_STEP, C_OUT, C_MAP, C_ITER);
  for (int i = 0; i < 3; i++)
    printf(", \"%s\": {\"lane_util\": %.4f, \"wave_instr_per_tile\": %.1f, \"vs_actual\": %.4f, "
           "\"de_calls_per_tile\": %.1f}",
           name[i], res[i][0] / (64.0 * res[i][1]), res[i][1] / tiles, res[i][1] / res[0][1],
           res[i][2] / tiles);
  /* compaction pays only while its own per-call cost (ray state moved through
   * LDS, per-lane stage selects, refill bookkeeping) stays below this */
  printf(", \"compaction_breakeven_instr_per_de_call\": %.1f}\n",
         (res[0][1] - res[1][1]) / res[1][2]);
  return 0;
}

/*
 * bulb_shadow_tail.c -- MEASUREMENT TOOL (not product, not a test): how much
 * of the Mandelbulb's shadow march runs outside the bounding sphere, per
 * wave (8x8 tile, lanes with N.L > 0 in lockstep).  Runs the CPU oracle on
 * the C5 frame with the iteration hook of tools/bulb_divergence.c and
 * counts, per tile, the shadow march's lockstep wave-steps: all, those where
 * every active lane's DE is the cheap outside-the-sphere bound, and the
 * trailing run of such steps (the "exit tail" an analytic shortcut would
 * remove).  Prints JSON.
 *
 *   gcc -O2 -fopenmp -Iinclude tools/bulb_shadow_tail.c -o /tmp/bst -lm && /tmp/bst [W H stride]
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

int main(int argc, char** argv) {
  int W = argc > 1 ? atoi(argv[1]) : 3840, H = argc > 2 ? atoi(argv[2]) : 2160;
  int stride = argc > 3 ? atoi(argv[3]) : 8;
  sdf_scene s; sdf_camera c; sdf_light l; sdf_material m; sdf_params p;
  sdf_oracle_defaults(&s, &c, &l, &m, &p, W, H);
  s.kind = SDF_SCENE_MANDELBULB; s.count = 0;
  s.bulb_center[0] = 0.0f; s.bulb_center[1] = 0.3f; s.bulb_center[2] = 0.0f;
  s.bulb_scale = 0.45f; s.bulb_iterations = 12; s.bulb_bailout = 2.0f;
  p.max_steps = 128; p.flags = SDF_FLAG_SHADOW | SDF_FLAG_AO; p.normal_mode = SDF_NORMAL_TETRA;
  oracle_uniforms u;
  if (make_uniforms(&c, &p, &u)) return 1;
  const int tx = (W + 7) / 8, ty = (H + 7) / 8;
  double steps = 0, all_out = 0, tail = 0, lane_steps = 0, lane_out = 0, lane_tail = 0,
         inside_iters = 0, prim_steps = 0;
  long tiles = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : tiles, steps, all_out, tail, lane_steps, lane_out, lane_tail, inside_iters, prim_steps)
  for (int tyi = 0; tyi < ty; tyi += stride) {
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
      int maxp = 0;
      for (int k = 0; k < 64; k++) if (nt[k] >= 0 && sp[k] > maxp) maxp = sp[k];
      prim_steps += maxp;
      int maxh = 0;
      for (int k = 0; k < 64; k++) if (nt[k] >= 0 && lit[k] && ss[k] > maxh) maxh = ss[k];
      int run = 0;
      for (int s_ = 0; s_ < maxh; s_++) {
        int act = 0, out_ = 0;
        for (int k = 0; k < 64; k++) {
          if (nt[k] < 0 || !lit[k] || ss[k] <= s_) continue;
          act++;
          int it = tr[k][sp[k] + 4 + s_];
          if (it == 0) out_++; else inside_iters += it;
        }
        steps += 1; lane_steps += act; lane_out += out_;
        if (out_ == act) { all_out += 1; run++; } else run = 0;
      }
      tail += run;
      /* per lane: trailing outside steps of its own march */
      for (int k = 0; k < 64; k++) {
        if (nt[k] < 0 || !lit[k]) continue;
        int r = 0;
        for (int s_ = ss[k] - 1; s_ >= 0 && tr[k][sp[k] + 4 + s_] == 0; s_--) r++;
        lane_tail += r;
      }
    }
  }
  printf("{\"tiles\": %ld, \"primary_wave_steps_per_tile\": %.2f, \"shadow_wave_steps_per_tile\": %.2f, "
         "\"all_lanes_outside_per_tile\": %.2f, \"trailing_all_outside_per_tile\": %.2f, "
         "\"lane_shadow_steps\": %.1f, \"lane_outside_frac\": %.3f, \"lane_trailing_outside_frac\": %.3f, "
         "\"inside_map_iters_per_tile\": %.1f}\n",
         tiles, prim_steps / tiles, steps / tiles, all_out / tiles, tail / tiles, lane_steps / tiles,
         lane_out / (lane_steps > 0 ? lane_steps : 1), lane_tail / (lane_steps > 0 ? lane_steps : 1),
         inside_iters / tiles);
  return 0;
}

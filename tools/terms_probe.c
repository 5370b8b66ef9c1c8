/*
 * terms_probe.c -- MEASUREMENT TOOL (not product, not a test): the oracle's
 * colours and shading terms of one frame, for tools/terms_cost.py, which
 * compares their TILES stream sizes (the wire's choice of what to carry,
 * DESIGN.md 6 "TILES wire format").
 *
 * It runs the CPU oracle (oracle/sdf_oracle.c, fp32 restatement) with the
 * instrumentation hook ORACLE_TERMS_HOOK (a no-op in every other build) and
 * writes, for H x W pixels (row 0 = bottom), float32 [H][W][3] colours then
 * [H][W][3] terms (ao, dif, max(N.H, 0)).  The frame's structs come from a
 * file written by terms_cost.py (sdf_scene, sdf_camera, sdf_light,
 * sdf_material, sdf_params, back to back).
 *
 *   gcc -O2 -fopenmp -Iinclude tools/terms_probe.c -o /tmp/terms_probe -lm
 *   /tmp/terms_probe W H frame.bin out.bin
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static __thread float t_terms[3];
#define ORACLE_TERMS_HOOK(ao, dif, spec, x, ndl, sh) \
  (t_terms[0] = (float)(ao), t_terms[1] = (float)(dif), t_terms[2] = (float)(x))

#include "../oracle/sdf_oracle.c"

int main(int argc, char** argv) {
  if (argc != 5) return 2;
  const int W = atoi(argv[1]), H = atoi(argv[2]);
  sdf_scene s; sdf_camera c; sdf_light l; sdf_material m; sdf_params p;
  FILE* f = fopen(argv[3], "rb");
  if (!f) return 1;
  if (fread(&s, sizeof s, 1, f) + fread(&c, sizeof c, 1, f) + fread(&l, sizeof l, 1, f) +
          fread(&m, sizeof m, 1, f) + fread(&p, sizeof p, 1, f) != 5)
    return 1;
  fclose(f);
  oracle_uniforms u;
  if (make_uniforms(&c, &p, &u)) return 1;
  float* col = malloc((size_t)W * H * 3 * 4);
  float* trm = malloc((size_t)W * H * 3 * 4);
#pragma omp parallel for schedule(dynamic, 4)
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      const float qy = (float)(2 * y + 1) / (float)H - 1.0f;
      const float qx = (float)(2 * x + 1) / (float)W - 1.0f;
      f32_v3 r0 = f32_normalize(f32_mk(qx * u.aspect, qy, u.focal));
      const float* mm = u.inv_view;
      f32_v3 r1 = f32_mk(mm[0] * r0.x + mm[4] * r0.y + mm[8] * r0.z,
                         mm[1] * r0.x + mm[5] * r0.y + mm[9] * r0.z,
                         mm[2] * r0.x + mm[6] * r0.y + mm[10] * r0.z);
      f32_v3 ray = f32_normalize(r1);
      f32_v3 cam = f32_mk(u.cam[0], u.cam[1], u.cam[2]);
      float out[4];
      int st[2];
      t_terms[0] = 1.0f;
      t_terms[1] = t_terms[2] = 0.0f;
      f32_shade_pixel(&s, &l, &m, &p, cam, ray, out, st, 0);
      const size_t o = ((size_t)y * W + x) * 3;
      memcpy(col + o, out, 12);
      memcpy(trm + o, t_terms, 12);
    }
  FILE* g = fopen(argv[4], "wb");
  if (!g) return 1;
  fwrite(col, 4, (size_t)W * H * 3, g);
  fwrite(trm, 4, (size_t)W * H * 3, g);
  fclose(g);
  return 0;
}

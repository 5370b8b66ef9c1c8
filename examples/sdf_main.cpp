// sdf_main.cpp -- headless counterpart of the reference host program
// (/root/reference/Code/src/main.cpp): create the renderer once, loop over
// frames (the reference's `while(!gl->closed())` with arcball input, :87-98,
// becomes an orbit sequence), time each frame (the reference's unreported
// cl->get_tic()/get_toc(), :89/:97) and clean up.  The last frame is written
// as a PPM instead of being presented in a window (:95-96).
//
//   sdf_main [width height frames out.ppm scene]     scene: ref | csg8 | bulb
#include <cstdio>
#include <cstdlib>
#include <string>

#include "../include/sdf3d.hpp"

int main(int argc, char** argv) {
  const int W = argc > 1 ? std::atoi(argv[1]) : 800;   // main.cpp:4 SX
  const int H = argc > 2 ? std::atoi(argv[2]) : 600;   // main.cpp:5 SY
  const int frames = argc > 3 ? std::atoi(argv[3]) : 8;
  const std::string out = argc > 4 ? argv[4] : "sdf_main.ppm";
  const std::string kind = argc > 5 ? argv[5] : "ref";
  try {
    sdf::Frame f = sdf::Frame::reference(W, H);
    if (kind == "csg8") {
      const int S = SDF_OP_SMOOTH_UNION;
      const float k = 0.1f;
      sdf::Scene s;
      s.plane(0, 1, 0, 0)
          .sphere(0, 0.4f, 0, 0.2f, S, k)
          .box(-0.7f, 0.15f, -0.3f, 0.15f, 0.15f, 0.15f, S, k)
          .torus(0.7f, 0.1f, -0.3f, 0.2f, 0.06f, S, k)
          .capsule(-0.35f, 0.1f, 0.4f, 0.05f, 0.45f, 0.3f, 0.07f, S, k)
          .cylinder(0.45f, 0.25f, 0.35f, 0.12f, 0.25f, S, k)
          .round_box(0, 0.12f, -0.8f, 0.5f, 0.12f, 0.1f, 0.04f, S, k)
          .sphere(0.25f, 0.55f, -0.15f, 0.12f, S, k);
      f.scene = s.raw();
      f.params.max_steps = 128;
      f.params.flags = SDF_FLAG_SHADOW | SDF_FLAG_AO;
      f.params.normal_mode = SDF_NORMAL_TETRA;
    } else if (kind == "bulb") {
      f.scene = sdf::Scene().mandelbulb(0, 0.3f, 0, 0.45f).raw();
      f.params.max_steps = 128;
      f.params.flags = SDF_FLAG_SHADOW | SDF_FLAG_AO;
      f.params.normal_mode = SDF_NORMAL_TETRA;
    }
    f.params.precision = SDF_PRECISION_FAST;

    hipStream_t stream;
    sdf::check_hip(hipStreamCreate(&stream), "hipStreamCreate");
    hipEvent_t t0, t1;
    sdf::check_hip(hipEventCreate(&t0), "hipEventCreate");
    sdf::check_hip(hipEventCreate(&t1), "hipEventCreate");
    {
      sdf::Renderer r(W, H, stream);
      for (int i = 0; i < frames; ++i) {
        f.orbit(360.0f * i / frames, 0.0f);
        sdf::check_hip(hipEventRecord(t0, stream), "hipEventRecord");
        r.render(f);
        sdf::check_hip(hipEventRecord(t1, stream), "hipEventRecord");
        sdf::check_hip(hipEventSynchronize(t1), "hipEventSynchronize");
        float ms = 0;
        sdf::check_hip(hipEventElapsedTime(&ms, t0, t1), "hipEventElapsedTime");
        std::printf("frame %d: %.3f ms (%.1f Mpixels/s)\n", i, ms, W * H / (ms * 1e3));
      }
      sdf::write_ppm(out, r.download(), W, H);
    }
    (void)hipEventDestroy(t0);
    (void)hipEventDestroy(t1);
    (void)hipStreamDestroy(stream);
    std::printf("wrote %s\n", out.c_str());
  } catch (const std::exception& e) {
    std::fprintf(stderr, "sdf_main: %s\n", e.what());
    return 1;
  }
  return 0;
}

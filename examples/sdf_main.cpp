// sdf_main.cpp -- headless counterpart of the reference host program
// (/root/reference/Code/src/main.cpp): create the renderer once, loop over
// frames (the reference's `while(!gl->closed())` with arcball input, :87-98,
// becomes an orbit sequence), time each frame (the reference's unreported
// cl->get_tic()/get_toc(), :89/:97) and clean up.  The last frame is written
// as a PPM instead of being presented in a window (:95-96).
//
//   sdf_main [width height frames out.ppm scene]     scene: ref | csg8 | bulb
//
// Multi-GPU: launched once per GPU by any launcher that sets RANK,
// WORLD_SIZE and LOCAL_RANK (e.g. `torchrun --nproc-per-node 8 --no-python
// sdf_main 3840 2160 200 out.ppm csg8`), or with SDF3D_DRIVER=1 on one GPU,
// it runs the native frame driver (sdf_driver_*): every rank renders its row
// blocks of every frame and rank 0 assembles them over RCCL.  The two RCCL
// unique ids travel through files in SDF3D_ID_DIR (default /tmp) named by
// SDF3D_RUN_ID (default: torchrun's TORCHELASTIC_RUN_ID); SDF3D_RCCL names
// the librccl to load (default librccl.so.1); SDF3D_ROOT_AS_PEER=1 makes
// rank 0 ship its rows to itself (the multi-rank sequence on one GPU).
//
// Navigation: by default frame i orbits the camera by 360 i / frames degrees;
// SDF3D_NAV=arcball drives V_mat from sdf::Arcball (the reference's mouse and
// gamepad navigation, main.cpp:37-45, :93-94) fed with a scripted input
// sequence (nav_input: orbit drag, pan drag, release, gamepad sticks), and
//   sdf_main --views N
// prints the first N V_mats of that sequence (no GPU work; the tests compare
// them with sdf3d_amd.camera.Arcball fed the same script).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>

#include "../include/sdf3d.hpp"

namespace {

std::string env(const char* name, const char* dflt) {
  const char* v = std::getenv(name);
  return v && *v ? v : dflt;
}

// The scripted navigation input of frame i (period 90 frames at 60 Hz),
// restated in tests/test_camera.py nav_input.
void nav_input(sdf::Arcball& a, int i) {
  const double dt = 1.0 / 60.0;
  const int ph = i % 90;
  if (ph < 30) a.mouse(dt, 0.004, 0.0015, true, false);          // orbit drag
  else if (ph < 45) a.mouse(dt, -0.002, 0.001, false, true);     // pan drag
  else if (ph < 60) a.mouse(dt, 0.0, 0.0, false, false);         // released: decay
  else if (ph < 80) a.gamepad(dt, 0.8, -0.5, 0.2, 0.35);        // sticks (rx inside the deadzone)
  else a.gamepad(dt, 0.1, 0.0, 0.0, 0.0);                        // sticks released
}

// V_mat of frame i under SDF3D_NAV (see the header comment).
struct Navigator {
  bool arcball = env("SDF3D_NAV", "orbit") == "arcball";
  sdf::Arcball ball;
  int next = 0;
  void frame(sdf::Frame& f, int i, int frames) {
    if (!arcball) {
      f.orbit(360.0f * i / frames, 0.0f);
      return;
    }
    while (next <= i) nav_input(ball, next++);
    ball.apply(f);
  }
};

int run_driver(sdf::Frame f, int frames, const std::string& out) {
  const int rank = std::atoi(env("RANK", "0").c_str());
  const int world = std::atoi(env("WORLD_SIZE", "1").c_str());
  const int local = std::atoi(env("LOCAL_RANK", "0").c_str());
  const bool peer_root = env("SDF3D_ROOT_AS_PEER", "0") == "1";
  sdf::check_hip(hipSetDevice(local), "hipSetDevice");
  const std::string rccl = env("SDF3D_RCCL", "librccl.so.1");
  const std::string dir = env("SDF3D_ID_DIR", "/tmp");
  const std::string run = env("SDF3D_RUN_ID", env("TORCHELASTIC_RUN_ID", "default").c_str());
  std::unique_ptr<sdf::Comm> lengths, data;
  if (world > 1 || peer_root) {
    const std::string a = "sdf3d_" + run + "_lengths.id", b = "sdf3d_" + run + "_data.id";
    lengths.reset(new sdf::Comm(sdf::exchange_id(dir, a, rank, rccl), world, rank, rccl));
    data.reset(new sdf::Comm(sdf::exchange_id(dir, b, rank, rccl), world, rank, rccl));
    if (rank == 0) {  // every rank has joined both communicators: the files are spent
      std::remove((dir + "/" + a).c_str());
      std::remove((dir + "/" + b).c_str());
    }
  }
  // shares: SDF3D_SHARES="a:b", else what the cost model of bench.py picks
  // for this world size (sdf3d_amd/multigpu.py choose_shares)
  static const int kShares[9][2] = {{1, 1}, {1, 1}, {1, 1}, {1, 1}, {3, 4},
                                    {3, 4}, {1, 2}, {1, 2}, {1, 7}};
  int share_root = kShares[world < 9 ? world : 8][0], share_peer = kShares[world < 9 ? world : 8][1];
  if (std::sscanf(env("SDF3D_SHARES", "").c_str(), "%d:%d", &share_root, &share_peer) != 2) {
    share_root = kShares[world < 9 ? world : 8][0];
    share_peer = kShares[world < 9 ? world : 8][1];
  }
  // N > 1: frames shipped two at a time (one length all-gather and one
  // send/recv group per pair), 4 buffer sets, a pair gathered 2 frames after
  // its last render
  const bool ship = world > 1 || peer_root;
  sdf_driver_config cfg = {rank, world, share_root, share_peer, ship ? 4 : 3, ship ? 2 : 1,
                           peer_root ? SDF_DRIVER_ROOT_AS_PEER : 0, 60000, ship ? 2 : 1};
  f.params.output_format = SDF_FORMAT_RGBA32F;
  sdf::FrameDriver drv(f, cfg, lengths.get(), data.get());
  int64_t last = -1;
  for (int i = 0; i < 5; ++i) last = drv.step();  // warm-up
  drv.drain();
  Navigator nav;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < frames; ++i) {
    nav.frame(f, i, frames);                        // the arcball's V_mat (main.cpp:93-94)
    drv.set_camera(f.camera);
    last = drv.step();
  }
  drv.drain();
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (rank == 0) {
    std::printf("rank 0 of %d: %d frames %dx%d in %.3f ms: %.1f fps, %.1f Mpixels/s "
                "(driver host %.1f us/frame)\n",
                world, frames, f.params.width, f.params.height, s * 1e3, frames / s,
                double(f.params.width) * f.params.height * frames / s / 1e6,
                drv.host_us_per_frame());
    sdf::write_ppm(out, drv.download(last), f.params.width, f.params.height);
    std::printf("wrote %s\n", out.c_str());
  }
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc > 2 && std::string(argv[1]) == "--views") {
    sdf::Arcball ball;
    float v[16];
    for (int i = 0; i < std::atoi(argv[2]); ++i) {
      nav_input(ball, i);
      ball.view(v);
      for (int k = 0; k < 16; ++k) {
        uint32_t u;
        std::memcpy(&u, &v[k], 4);
        std::printf("%08x%c", u, k == 15 ? '\n' : ' ');
      }
    }
    return 0;
  }
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
    // EXACT (the default): the oracle's fp32 operation sequence, every pixel
    // bit-identical to it at 4K.  SDF3D_PRECISION=fast opts into FMA
    // contraction and hardware sqrt/rcp: 1.47x faster on C4, but a few
    // grazing pixels end their march a step apart (C4: 48 pixels over 1e-4,
    // max 0.72; C5: 2,123, max 0.34; profiles/parity_fullsize.json)
    f.params.precision =
        env("SDF3D_PRECISION", "exact") == "fast" ? SDF_PRECISION_FAST : SDF_PRECISION_EXACT;
    if (std::getenv("WORLD_SIZE") || env("SDF3D_DRIVER", "0") == "1")
      return run_driver(f, frames, out);

    hipStream_t stream;
    sdf::check_hip(hipStreamCreate(&stream), "hipStreamCreate");
    hipEvent_t t0, t1;
    sdf::check_hip(hipEventCreate(&t0), "hipEventCreate");
    sdf::check_hip(hipEventCreate(&t1), "hipEventCreate");
    {
      sdf::Renderer r(W, H, stream);
      Navigator nav;
      for (int i = 0; i < frames; ++i) {
        nav.frame(f, i, frames);
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

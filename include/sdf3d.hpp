// sdf3d.hpp -- C++ host/scene API over the C-ABI of include/sdf_abi.h.
//
// Mirrors the shape of the reference host program (/root/reference/Code/src/
// main.cpp): objects created once (main.cpp:48-56), the device program set up
// once (:67-77), a per-frame draw in a loop (:87-98) and explicit cleanup
// (:103-107).  Where the reference hard-codes the scene, camera, light and
// material inside the fragment shader (voxel_fragment.frag:178-189), this API
// takes them as values; sdf::Frame::reference() reproduces the hard-coded ones.
//
// Header-only; link against libsdf3d.so and amdhip64.  Errors are reported as
// sdf::Error exceptions on this side of the boundary (the C-ABI itself never
// throws).
#pragma once

#include <hip/hip_runtime.h>

#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "sdf_abi.h"

namespace sdf {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& what)
      : std::runtime_error(what + ": " + sdf_strerror(c)), code(c) {}
};

inline void check(int rc, const char* what) {
  if (rc != SDF_OK) throw Error(rc, what);
}
inline void check_hip(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
// The loaded libsdf3d must implement the ABI these headers describe (struct
// layouts and signatures change with SDF_ABI_VERSION); checked once by every
// object that calls into it.
inline void check_abi() {
  static const int v = sdf_abi_version();
  if (v != SDF_ABI_VERSION)
    throw Error(SDF_E_UNSUPPORTED, "libsdf3d ABI " + std::to_string(v) + " != headers' " +
                                       std::to_string(SDF_ABI_VERSION));
}

// Scene builder: primitives combined left to right into d (d starts at +INF,
// voxel_fragment.frag:75).
class Scene {
 public:
  Scene() { std::memset(&s_, 0, sizeof(s_)); s_.kind = SDF_SCENE_PRIMITIVES; s_.bulb_scale = 1.0f;
            s_.bulb_iterations = 12; s_.bulb_bailout = 2.0f; }
  explicit Scene(const sdf_scene& s) : s_(s) {}

  Scene& sphere(float cx, float cy, float cz, float r, int op = SDF_OP_UNION, float k = 0) {
    return add(SDF_PRIM_SPHERE, op, k, {cx, cy, cz, r});
  }
  Scene& plane(float nx, float ny, float nz, float h, int op = SDF_OP_UNION, float k = 0) {
    return add(SDF_PRIM_PLANE, op, k, {nx, ny, nz, h});
  }
  Scene& box(float cx, float cy, float cz, float hx, float hy, float hz, int op = SDF_OP_UNION,
             float k = 0) {
    return add(SDF_PRIM_BOX, op, k, {cx, cy, cz, hx, hy, hz});
  }
  Scene& round_box(float cx, float cy, float cz, float hx, float hy, float hz, float r,
                   int op = SDF_OP_UNION, float k = 0) {
    return add(SDF_PRIM_ROUND_BOX, op, k, {cx, cy, cz, hx, hy, hz, r});
  }
  Scene& torus(float cx, float cy, float cz, float R, float r, int op = SDF_OP_UNION,
               float k = 0) {
    return add(SDF_PRIM_TORUS, op, k, {cx, cy, cz, R, r});
  }
  Scene& capsule(float ax, float ay, float az, float bx, float by, float bz, float r,
                 int op = SDF_OP_UNION, float k = 0) {
    return add(SDF_PRIM_CAPSULE, op, k, {ax, ay, az, bx, by, bz, r});
  }
  Scene& cylinder(float cx, float cy, float cz, float r, float half_h, int op = SDF_OP_UNION,
                  float k = 0) {
    return add(SDF_PRIM_CYLINDER, op, k, {cx, cy, cz, r, half_h});
  }
  Scene& mandelbulb(float cx, float cy, float cz, float scale, int iterations = 12,
                    float bailout = 2.0f) {
    s_.kind = SDF_SCENE_MANDELBULB;
    s_.count = 0;
    s_.bulb_center[0] = cx; s_.bulb_center[1] = cy; s_.bulb_center[2] = cz;
    s_.bulb_scale = scale; s_.bulb_iterations = iterations; s_.bulb_bailout = bailout;
    return *this;
  }
  const sdf_scene& raw() const { return s_; }
  sdf_scene& raw() { return s_; }

 private:
  Scene& add(int kind, int op, float k, std::initializer_list<float> p) {
    if (s_.count >= SDF_MAX_PRIMS) throw Error(SDF_E_INVALID_ARG, "Scene: too many primitives");
    sdf_primitive& pr = s_.prims[s_.count++];
    std::memset(&pr, 0, sizeof(pr));
    pr.kind = kind; pr.op = op; pr.k = k;
    int i = 0;
    for (float v : p) pr.p[i++] = v;
    return *this;
  }
  sdf_scene s_;
};

// Everything one frame needs besides the output.
struct Frame {
  sdf_scene scene;
  sdf_camera camera;
  sdf_light light;
  sdf_material material;
  sdf_params params;

  // The reference shader's hard-coded frame (voxel_fragment.frag:15-23,
  // :54-81, :178-189, :205) at width x height (<= 0: 800 x 600, main.cpp:4-5).
  static Frame reference(int width = 0, int height = 0) {
    check_abi();
    Frame f;
    check(sdf_defaults(&f.scene, &f.camera, &f.light, &f.material, &f.params, width, height),
          "sdf_defaults");
    return f;
  }
  // Orbit the camera about the origin: V_mat = Rx(pitch) * Ry(yaw), column-major
  // (the reference gets V_mat from Neutrino's arcball, main.cpp:93-94).
  Frame& orbit(float yaw_deg, float pitch_deg) {
    const double y = yaw_deg * M_PI / 180.0, p = pitch_deg * M_PI / 180.0;
    const double cy = std::cos(y), sy = std::sin(y), cp = std::cos(p), sp = std::sin(p);
    // rows of Rx*Ry
    const double m[4][4] = {{cy, 0, sy, 0}, {sp * sy, cp, -sp * cy, 0},
                            {-cp * sy, sp, cp * cy, 0}, {0, 0, 0, 1}};
    for (int c = 0; c < 4; ++c)
      for (int r = 0; r < 4; ++r) camera.view[c * 4 + r] = static_cast<float>(m[r][c]);
    return *this;
  }
};

// Arcball navigation producing V_mat: the reference
// drives V_mat from Neutrino's mouse and gamepad navigation with these rates
// (main.cpp:37-45: orbit 1 rev/s, pan 5 m/s, decay 1.25 s; gamepad orbit 1,
// pan 1, decay 1.25, deadzone 0.30), called once per frame (:93-94).
// Neutrino's implementation is not vendored, so the dynamics are this
// framework's own (parity unpinned), identical to sdf3d_amd/camera.py (the
// tests compare the two sequences bit for bit):
//   * while a mouse button drags, orbit (or pan) velocity = rate * motion / dt;
//     released, the velocity decays by exp(-dt / decay_time) per update;
//   * a gamepad stick outside the deadzone sets the velocity to
//     rate * 2 pi (orbit, rev/s) or rate (pan) times the stick value rescaled
//     from [deadzone, 1] to [0, 1]; inside it, the velocity decays;
//   * pitch is clamped to [-pi/2, pi/2]; V_mat = T(pan) * Rx(pitch) * Ry(yaw).
// All arithmetic in double, the matrix rounded to float once.
class Arcball {
 public:
  struct Rates {
    double orbit_rate = 1.0, pan_rate = 5.0, decay_time = 1.25;     // mouse, main.cpp:37-39
    double pad_orbit_rate = 1.0, pad_pan_rate = 1.0, pad_decay_time = 1.25,
           pad_deadzone = 0.30;                                       // gamepad, main.cpp:42-45
  };
  Arcball() = default;
  explicit Arcball(const Rates& r) : r_(r) {}

  // Mouse: pointer motion (dx, dy) in normalised screen units over dt seconds.
  void mouse(double dt, double dx, double dy, bool orbit, bool pan) {
    if (!(dt > 0)) return;
    if (orbit) vyaw_ = r_.orbit_rate * dx / dt, vpitch_ = r_.orbit_rate * dy / dt;
    if (pan) vpx_ = r_.pan_rate * dx / dt, vpy_ = r_.pan_rate * dy / dt;
    integrate(dt, !orbit, !pan, r_.decay_time);
  }
  // Gamepad: left stick (lx, ly) orbits, right stick (rx, ry) pans, in [-1, 1].
  void gamepad(double dt, double lx, double ly, double rx, double ry) {
    if (!(dt > 0)) return;
    const double ax = dead(lx), ay = dead(ly), bx = dead(rx), by = dead(ry);
    const bool orbit = ax != 0.0 || ay != 0.0, pan = bx != 0.0 || by != 0.0;
    const double two_pi = 2.0 * M_PI;
    if (orbit) vyaw_ = r_.pad_orbit_rate * two_pi * ax, vpitch_ = r_.pad_orbit_rate * two_pi * ay;
    if (pan) vpx_ = r_.pad_pan_rate * bx, vpy_ = r_.pad_pan_rate * by;
    integrate(dt, !orbit, !pan, r_.pad_decay_time);
  }
  // V_mat, column-major float (sdf_camera.view).
  void view(float* out16) const {
    const double cy = std::cos(yaw_), sy = std::sin(yaw_), cp = std::cos(pitch_),
                 sp = std::sin(pitch_);
    const double m[4][4] = {{cy, 0, sy, pan_x_}, {sp * sy, cp, -sp * cy, pan_y_},
                            {-cp * sy, sp, cp * cy, 0}, {0, 0, 0, 1}};
    for (int c = 0; c < 4; ++c)
      for (int r = 0; r < 4; ++r) out16[c * 4 + r] = static_cast<float>(m[r][c]);
  }
  void apply(Frame& f) const { view(f.camera.view); }
  double yaw() const { return yaw_; }
  double pitch() const { return pitch_; }

 private:
  double dead(double a) const {
    const double z = r_.pad_deadzone, m = std::fabs(a);
    if (!(m > z)) return 0.0;
    return std::copysign(std::min((m - z) / (1.0 - z), 1.0), a);
  }
  void integrate(double dt, bool decay_orbit, bool decay_pan, double tau) {
    yaw_ += vyaw_ * dt;
    pitch_ = std::max(-M_PI / 2, std::min(M_PI / 2, pitch_ + vpitch_ * dt));
    pan_x_ += vpx_ * dt;
    pan_y_ += vpy_ * dt;
    if (decay_orbit || decay_pan) {
      const double k = tau > 0 ? std::exp(-dt / tau) : 0.0;
      if (decay_orbit) vyaw_ *= k, vpitch_ *= k;
      if (decay_pan) vpx_ *= k, vpy_ *= k;
    }
  }
  Rates r_;
  double yaw_ = 0, pitch_ = 0, pan_x_ = 0, pan_y_ = 0;
  double vyaw_ = 0, vpitch_ = 0, vpx_ = 0, vpy_ = 0;
};

// Owns a device framebuffer and renders frames into it on one HIP stream.
// The buffer holds width x height pixels of up to 16 bytes (any sdf_format).
class Renderer {
 public:
  Renderer(int width, int height, hipStream_t stream = nullptr)
      : w_(width), h_(height), stream_(stream) {
    check_abi();
    check_hip(hipMalloc(&rgba_, size_t(w_) * h_ * 16), "hipMalloc");
  }
  ~Renderer() { if (rgba_) (void)hipFree(rgba_); }
  Renderer(const Renderer&) = delete;
  Renderer& operator=(const Renderer&) = delete;

  // One frame (the reference's gl->plot(sh, proj_mode), main.cpp:95).
  void render(const Frame& f, const sdf_tiling* tiling = nullptr, int32_t* steps = nullptr) {
    if (f.params.width != w_ || f.params.height != h_)
      throw Error(SDF_E_INVALID_ARG, "Renderer: frame size differs from framebuffer");
    check(sdf_render(&f.scene, &f.camera, &f.light, &f.material, &f.params, tiling, rgba_, steps,
                     stream_),
          "sdf_render");
  }
  // Blocking copy of an RGBA32F framebuffer (row 0 = bottom, GL order).
  std::vector<float> download() const {
    std::vector<float> out(size_t(w_) * h_ * 4);
    copy_out(out.data(), out.size() * sizeof(float));
    return out;
  }
  // Blocking copy of the framebuffer bytes of any format.
  std::vector<unsigned char> download_bytes(int format) const {
    const int bpp = sdf_format_bytes(format);
    if (bpp < 0) throw Error(bpp, "download_bytes");
    std::vector<unsigned char> out(size_t(w_) * h_ * bpp);
    copy_out(out.data(), out.size());
    return out;
  }
  float* device_rgba() const { return rgba_; }
  int width() const { return w_; }
  int height() const { return h_; }

 private:
  void copy_out(void* dst, size_t bytes) const {
    check_hip(hipMemcpyAsync(dst, rgba_, bytes, hipMemcpyDeviceToHost, stream_),
              "hipMemcpyAsync");
    check_hip(hipStreamSynchronize(stream_), "hipStreamSynchronize");
  }
  int w_, h_;
  hipStream_t stream_;
  float* rgba_ = nullptr;
};

// ---- multi-device frames (sdf_comm_* / sdf_driver_*) ------------------------

// One RCCL communicator over `world` processes (one per GPU), created from a
// unique id rank 0 makes; the caller moves the id between processes.
class Comm {
 public:
  using Id = std::vector<unsigned char>;
  static Id unique_id(const std::string& rccl_path = "") {
    check_abi();
    Id id(SDF_COMM_ID_BYTES);
    check(sdf_comm_unique_id(rccl_path.empty() ? nullptr : rccl_path.c_str(), id.data()),
          "sdf_comm_unique_id");
    return id;
  }
  // Blocks until every rank has joined, at most timeout_ms (then throws
  // SDF_E_TIMEOUT: a peer that failed, or an id that is not this launch's).
  Comm(const Id& id, int world, int rank, const std::string& rccl_path = "",
       int timeout_ms = 120000) {
    check_abi();
    check(sdf_comm_create(rccl_path.empty() ? nullptr : rccl_path.c_str(), id.data(), world, rank,
                          timeout_ms, &c_),
          "sdf_comm_create");
  }
  ~Comm() { if (c_) (void)sdf_comm_destroy(c_); }
  Comm(const Comm&) = delete;
  Comm& operator=(const Comm&) = delete;
  sdf_comm* get() const { return c_; }

 private:
  sdf_comm* c_ = nullptr;
};

// Moves communicator ids through a directory every rank can see (a node's
// local disk or /dev/shm): rank 0 writes `name` atomically (write, then
// rename), the others wait for it.  Pure-C++ launches (no MPI, no Python)
// use this; a Python host uses torch.distributed (sdf3d_amd/driver.py).
//
// A file left by an earlier launch that died before rank 0 removed it must
// not be taken for this launch's.  So the file carries a launch tag (the
// launcher's MASTER_ADDR/MASTER_PORT, TORCHELASTIC_RUN_ID and
// TORCHELASTIC_RESTART_COUNT, plus SDF3D_LAUNCH_NONCE when the launcher
// sets one) that peers compare with their own, and peers ignore a file
// written before their own first call here, less `skew_s` (ranks of one
// launch start within seconds of each other).  An id that still slips
// through cannot hang anyone: Comm's join gives up after its timeout.
inline std::string launch_tag() {
  std::string t;
  for (const char* k : {"MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID",
                        "TORCHELASTIC_RESTART_COUNT", "SDF3D_LAUNCH_NONCE"}) {
    const char* v = std::getenv(k);
    t += std::string(k) + "=" + (v ? v : "") + ";";
  }
  return t;
}

inline Comm::Id exchange_id(const std::string& dir, const std::string& name, int rank,
                            const std::string& rccl_path = "", double timeout_s = 120.0,
                            double skew_s = 30.0) {
  static const auto first_call = std::chrono::system_clock::now();
  const std::string path = dir + "/" + name;
  const std::string tag = launch_tag();
  if (rank == 0) {
    Comm::Id id = Comm::unique_id(rccl_path);
    const std::string tmp = path + ".tmp";
    const uint32_t n = static_cast<uint32_t>(tag.size());
    FILE* fp = std::fopen(tmp.c_str(), "wb");
    if (!fp || std::fwrite(&n, sizeof(n), 1, fp) != 1 ||
        std::fwrite(tag.data(), 1, n, fp) != n ||
        std::fwrite(id.data(), 1, id.size(), fp) != id.size() || std::fclose(fp) != 0 ||
        std::rename(tmp.c_str(), path.c_str()) != 0)
      throw std::runtime_error("cannot write " + path);
    return id;
  }
  const auto not_before = first_call - std::chrono::milliseconds(long(skew_s * 1e3));
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    struct stat sb;
    if (stat(path.c_str(), &sb) == 0 &&
        std::chrono::system_clock::from_time_t(sb.st_mtime) >= not_before) {
      if (FILE* fp = std::fopen(path.c_str(), "rb")) {
        uint32_t n = 0;
        std::string got;
        Comm::Id id(SDF_COMM_ID_BYTES);
        bool ok = std::fread(&n, sizeof(n), 1, fp) == 1 && n < (1u << 16);
        if (ok) {
          got.resize(n);
          ok = std::fread(&got[0], 1, n, fp) == n &&
               std::fread(id.data(), 1, id.size(), fp) == id.size();
        }
        std::fclose(fp);
        if (ok && got == tag) return id;
      }
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
      throw std::runtime_error("timed out waiting for " + path + " of this launch");
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
}

// The native frame loop across the node (include/sdf_abi.h sdf_driver_*):
// every rank steps every frame; rank 0 holds the assembled frames.  The
// reference's `while (!gl->closed()) { ... gl->plot(sh, proj_mode); }`
// (main.cpp:87-98) becomes `while (...) { drv.set_camera(...); drv.step(); }`.
class FrameDriver {
 public:
  FrameDriver(const Frame& f, const sdf_driver_config& cfg, Comm* lengths = nullptr,
              Comm* data = nullptr)
      : w_(f.params.width), h_(f.params.height), format_(f.params.output_format) {
    check_abi();
    check(sdf_driver_create(&f.scene, &f.camera, &f.light, &f.material, &f.params, &cfg,
                            lengths ? lengths->get() : nullptr, data ? data->get() : nullptr, &d_),
          "sdf_driver_create");
  }
  ~FrameDriver() { if (d_) (void)sdf_driver_destroy(d_); }
  FrameDriver(const FrameDriver&) = delete;
  FrameDriver& operator=(const FrameDriver&) = delete;

  void set_camera(const sdf_camera& c) { check(sdf_driver_set_camera(d_, &c), "sdf_driver_set_camera"); }
  int64_t step() {
    int64_t i = -1;
    check(sdf_driver_step(d_, &i), "sdf_driver_step");
    return i;
  }
  void drain() { check(sdf_driver_drain(d_), "sdf_driver_drain"); }
  // Rank 0: blocking copy of frame i (one of the last nbuf, shipped).
  std::vector<float> download(int64_t i) const {
    if (format_ != SDF_FORMAT_RGBA32F) throw Error(SDF_E_UNSUPPORTED, "download: not RGBA32F");
    std::vector<float> out(size_t(w_) * h_ * 4);
    void* src = nullptr;
    check(sdf_driver_frame(d_, i, &src), "sdf_driver_frame");
    check_hip(hipDeviceSynchronize(), "hipDeviceSynchronize");
    check_hip(hipMemcpy(out.data(), src, out.size() * sizeof(float), hipMemcpyDeviceToHost),
              "hipMemcpy");
    return out;
  }
  // Host seconds of the driver's own calls per frame, waits excluded.
  double host_us_per_frame() const {
    double v[3] = {0, 0, 0};
    check(sdf_driver_stats(d_, v, 3), "sdf_driver_stats");
    return v[0] > 0 ? (v[1] - v[2]) / v[0] * 1e6 : 0.0;
  }

 private:
  int w_, h_, format_;
  sdf_driver* d_ = nullptr;
};

// One RGBA32F frame across several devices of this process (sdf_render_multi):
// devices[0] holds `rgba` and `stream`; the others render TILES streams the
// root decodes through peer-mapped memory.  Successive calls on one stream.
inline void render_multi(const Frame& f, const std::vector<int>& devices, float* rgba,
                         hipStream_t stream, int share_root = 0, int share_peer = 0) {
  check_abi();
  std::vector<int32_t> d(devices.begin(), devices.end());
  check(sdf_render_multi(&f.scene, &f.camera, &f.light, &f.material, &f.params,
                         static_cast<int32_t>(d.size()), d.data(), share_root, share_peer, rgba,
                         stream),
        "sdf_render_multi");
}

// A camera path known in advance (sdf_render_frames): frame i of `f`'s scene
// seen through cameras[i] into rgba[i] (steps[i] when `steps` is non-empty),
// by the persistent frame-sequence kernel; the pixels of one sdf_render per
// camera.  Asynchronous on `stream`.
inline void render_frames(const Frame& f, const std::vector<sdf_camera>& cameras,
                          const std::vector<void*>& rgba, hipStream_t stream,
                          const std::vector<int32_t*>& steps = {}) {
  check_abi();
  if (rgba.size() != cameras.size() || (!steps.empty() && steps.size() != cameras.size()))
    throw Error(SDF_E_INVALID_ARG, "render_frames: one output per camera");
  check(sdf_render_frames(&f.scene, cameras.data(), static_cast<int32_t>(cameras.size()),
                          &f.light, &f.material, &f.params, rgba.data(),
                          steps.empty() ? nullptr : steps.data(), stream),
        "sdf_render_frames");
}

// Binary PPM of an RGBA float framebuffer, clamped and quantised to 8 bits
// (what the reference's window would show), flipped to top-down row order.
inline void write_ppm(const std::string& path, const std::vector<float>& rgba, int w, int h) {
  FILE* fp = std::fopen(path.c_str(), "wb");
  if (!fp) throw std::runtime_error("cannot open " + path);
  std::fprintf(fp, "P6\n%d %d\n255\n", w, h);
  std::vector<unsigned char> row(size_t(w) * 3);
  for (int y = h - 1; y >= 0; --y) {
    for (int x = 0; x < w; ++x)
      for (int c = 0; c < 3; ++c) {
        float v = rgba[(size_t(y) * w + x) * 4 + c];
        v = v < 0.f ? 0.f : (v > 1.f ? 1.f : v);
        row[size_t(x) * 3 + c] = static_cast<unsigned char>(std::lround(v * 255.0f));
      }
    std::fwrite(row.data(), 1, row.size(), fp);
  }
  std::fclose(fp);
}

}  // namespace sdf

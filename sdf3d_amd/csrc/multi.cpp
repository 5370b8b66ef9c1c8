// multi.cpp -- single-process multi-device frames (include/sdf_abi.h
// sdf_render_multi).
//
// The reference host is one process with one GL context
// (/root/reference/Code/src/main.cpp:34-110).  A host of that shape that
// wants the node's GPUs calls sdf_render_multi once per frame instead of
// sdf_render: no launcher, no communicator, no id exchange.  The devices
// split the frame as the multi-process driver does (driver.cpp):
//   * the root (devices[0]) renders its row blocks straight into the
//     caller's RGBA32F frame, on the caller's stream;
//   * every other device renders its blocks as a TILES stream (lossless,
//     ~3.2 B/pixel on C4) into a buffer of its own, on its own stream;
//   * the root's decode kernel reads those streams in place, through
//     peer-mapped device memory over xGMI (hipDeviceEnablePeerAccess): only
//     the compressed bytes cross the links, and no copy or length readback
//     is needed.
// Ordering, all on the GPU (the call returns after enqueueing):
//   caller stream --e_ready[s]--> peer streams (render into buffer set s,
//   after the decode that last read set s) --e_done[s][r]--> caller stream
//   (decode into the frame) --e_ready[s] recorded after it.
// Two buffer sets alternate between calls, so the peers render frame i+1
// while the root still decodes frame i.  A device may appear more than once
// in `devices` (its "peers" then share it): that runs the whole path on one
// GPU (tests/test_gpu_multi.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/sdf_abi.h"
#include "host_api.h"
#include "kernel_args.h"

namespace {

constexpr int kSets = 2;

struct Peer {
  int dev = 0;
  hipStream_t s = nullptr;
  void* buf[kSets] = {nullptr, nullptr};
  hipEvent_t done[kSets] = {nullptr, nullptr};
};

struct MultiContext {
  std::vector<int> devices;
  int W = 0, H = 0, share_root = 1, share_peer = 1;
  std::vector<sdf_tiling> tilings;
  std::vector<int> rows;
  std::vector<Peer> peers;                 // index r - 1 for rank r >= 1
  hipEvent_t ready[kSets] = {nullptr, nullptr};  // on the root device
  int next_set = 0;
  sdf::DecodeParts decode{};
  sdf::RenderPlan root_plan{}, peer_plan{};

  ~MultiContext() {
    for (Peer& p : peers) {
      (void)hipSetDevice(p.dev);
      for (int k = 0; k < kSets; ++k) {
        if (p.buf[k]) (void)hipFree(p.buf[k]);
        if (p.done[k]) (void)hipEventDestroy(p.done[k]);
      }
      if (p.s) (void)hipStreamDestroy(p.s);
    }
    if (!devices.empty()) {
      (void)hipSetDevice(devices[0]);
      for (hipEvent_t e : ready)
        if (e) (void)hipEventDestroy(e);
    }
  }
};

std::mutex g_mu;
std::unique_ptr<MultiContext> g_ctx;

int hip_ok(hipError_t e) { return e == hipSuccess ? SDF_OK : SDF_E_HIP; }

// Build the context for this device list, frame size and shares.
int make_context(const std::vector<int>& devs, int W, int H, int a, int b,
                 std::unique_ptr<MultiContext>* out) {
  auto c = std::make_unique<MultiContext>();
  c->devices = devs;
  c->W = W;
  c->H = H;
  c->share_root = a;
  c->share_peer = b;
  const int n = (int)devs.size();
  for (int r = 0; r < n; ++r) {
    sdf_tiling t;
    if (sdf_share_tiling(r, n, a, b, &t) != SDF_OK) return SDF_E_INVALID_ARG;
    const int rows = sdf::count_rows(H, t);
    if (rows < 0) return SDF_E_INVALID_ARG;
    c->tilings.push_back(t);
    c->rows.push_back(rows);
  }
  const int root = devs[0];
  if (hipSetDevice(root) != hipSuccess) return SDF_E_NO_DEVICE;
  for (hipEvent_t& e : c->ready)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return SDF_E_HIP;
  for (int r = 1; r < n; ++r) {
    const int d = devs[r];
    if (d != root) {
      // the root's decode reads this device's buffers
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, root, d) != hipSuccess || !can) return SDF_E_UNSUPPORTED;
      const hipError_t e = hipDeviceEnablePeerAccess(d, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return SDF_E_HIP;
      (void)hipGetLastError();  // clear a sticky "already enabled"
    }
  }
  c->peers.resize(n - 1);
  for (int r = 1; r < n; ++r) {
    Peer& p = c->peers[r - 1];
    p.dev = devs[r];
    if (hipSetDevice(p.dev) != hipSuccess) return SDF_E_NO_DEVICE;
    if (hipStreamCreateWithFlags(&p.s, hipStreamNonBlocking) != hipSuccess) return SDF_E_HIP;
    const int64_t bytes = sdf_tiles_bytes(W, c->rows[r]);
    if (bytes < 0) return (int)bytes;
    for (int k = 0; k < kSets; ++k) {
      if (hipMalloc(&p.buf[k], (size_t)std::max<int64_t>(bytes, 256)) != hipSuccess)
        return SDF_E_HIP;
      if (hipEventCreateWithFlags(&p.done[k], hipEventDisableTiming) != hipSuccess)
        return SDF_E_HIP;
    }
  }
  sdf::DecodeParts& D = c->decode;
  D.nparts = n;
  D.width = W;
  D.height = H;
  D.part_stride = 0;
  for (int r = 0; r < n; ++r) {
    const sdf_tiling& t = c->tilings[r];
    // the root's rows are rendered in place: no stream (rows 0 decodes nothing)
    D.rows[r] = r == 0 ? 0 : c->rows[r];
    D.first_block[r] = t.first_block;
    D.block_stride[r] = t.block_stride;
    D.block_rows[r] = t.block_rows;
    D.chunk_rows[r] = t.block_rows * sdf::tiling_run(t);
    D.run_gap_rows[r] = sdf::tiling_gap_rows(t);
  }
  if (hipSetDevice(root) != hipSuccess) return SDF_E_NO_DEVICE;
  *out = std::move(c);
  return SDF_OK;
}

// The default shares of rank 0 : others per period (bench.py / sdf_main.cpp,
// sdf3d_amd/multigpu.py choose_shares): rank 0 also decodes everyone's streams.
void default_shares(int n, int* a, int* b) {
  static const int kShares[9][2] = {{1, 1}, {1, 1}, {1, 1}, {1, 1}, {3, 4},
                                    {3, 4}, {1, 2}, {1, 2}, {2, 7}};
  const int k = n < 9 ? n : 8;
  *a = kShares[k][0];
  *b = kShares[k][1];
}

}  // namespace

static int render_multi(const sdf_scene* scene, const sdf_camera* camera,
                        const sdf_light* light, const sdf_material* material,
                        const sdf_params* params, int32_t ndev, const int32_t* devices,
                        int32_t share_root, int32_t share_peer, void* rgba, void* stream) {
  if (!params || !devices || !rgba || ndev < 1 || ndev > SDF_MAX_DECODE_PARTS)
    return SDF_E_INVALID_ARG;
  if (params->output_format != SDF_FORMAT_RGBA32F) return SDF_E_UNSUPPORTED;
  int rc = sdf_validate(scene, camera, light, material, params, nullptr);
  if (rc != SDF_OK) return rc;
  int a = share_root, b = share_peer;
  if (a <= 0 || b <= 0) default_shares(ndev, &a, &b);
  int prev = 0;
  (void)hipGetDevice(&prev);
  struct Restore {
    int d;
    ~Restore() { (void)hipSetDevice(d); }
  } restore{prev};
  std::vector<int> devs(devices, devices + ndev);
  std::lock_guard<std::mutex> lock(g_mu);
  if (!g_ctx || g_ctx->devices != devs || g_ctx->W != params->width ||
      g_ctx->H != params->height || g_ctx->share_root != a || g_ctx->share_peer != b) {
    // the old context's buffers may still be read by queued work
    if (g_ctx) {
      for (int d : g_ctx->devices) {
        (void)hipSetDevice(d);
        (void)hipDeviceSynchronize();
      }
    }
    g_ctx.reset();
    std::unique_ptr<MultiContext> c;
    rc = make_context(devs, params->width, params->height, a, b, &c);
    if (rc != SDF_OK) return rc;
    g_ctx = std::move(c);
  }
  MultiContext& c = *g_ctx;
  const int root = devs[0];
  hipStream_t s = (hipStream_t)stream;
  const int k = c.next_set;
  c.next_set = (k + 1) % kSets;
  // the root's rows straight into the frame, on the caller's stream
  if (hipSetDevice(root) != hipSuccess) return SDF_E_NO_DEVICE;
  sdf_params pf = *params;
  sdf_tiling t0 = c.tilings[0];
  t0.flags = SDF_TILING_FRAME_ROWS;
  if (c.rows[0] > 0) {
    rc = sdf::make_render_plan(scene, camera, light, material, &pf, &t0, rgba, nullptr,
                               &c.root_plan);
    if (rc == SDF_OK) rc = sdf::launch_render_plan(c.root_plan, s);
    if (rc != SDF_OK) return rc;
  }
  if (ndev == 1) return SDF_OK;
  // peers: TILES streams into buffer set k, once the decode that last read
  // it (recorded on the caller's stream) is done
  sdf_params pt = *params;
  pt.output_format = SDF_FORMAT_TILES;
  for (int r = 1; r < ndev; ++r) {
    Peer& p = c.peers[r - 1];
    if (c.rows[r] == 0) continue;
    if (hipSetDevice(p.dev) != hipSuccess) return SDF_E_NO_DEVICE;
    rc = hip_ok(hipStreamWaitEvent(p.s, c.ready[k], 0));
    if (rc == SDF_OK)
      rc = sdf::make_render_plan(scene, camera, light, material, &pt, &c.tilings[r], p.buf[k],
                                 nullptr, &c.peer_plan);
    if (rc == SDF_OK) rc = sdf::launch_render_plan(c.peer_plan, p.s);
    if (rc == SDF_OK) rc = hip_ok(hipEventRecord(p.done[k], p.s));
    if (rc != SDF_OK) return rc;
    c.decode.part_ptr[r] = p.buf[k];
  }
  // the root decodes every peer's stream in place (peer-mapped reads)
  if (hipSetDevice(root) != hipSuccess) return SDF_E_NO_DEVICE;
  for (int r = 1; r < ndev; ++r)
    if (c.rows[r] > 0) {
      rc = hip_ok(hipStreamWaitEvent(s, c.peers[r - 1].done[k], 0));
      if (rc != SDF_OK) return rc;
    }
  rc = hip_ok((hipError_t)sdf::launch_tiles_decode(c.decode, rgba, nullptr, s));
  if (rc == SDF_OK) rc = hip_ok(hipEventRecord(c.ready[k], s));
  return rc;
}

extern "C" int sdf_render_multi(const sdf_scene* scene, const sdf_camera* camera,
                                const sdf_light* light, const sdf_material* material,
                                const sdf_params* params, int32_t ndev, const int32_t* devices,
                                int32_t share_root, int32_t share_peer, void* rgba,
                                void* stream) {
  const int rc = render_multi(scene, camera, light, material, params, ndev, devices, share_root,
                              share_peer, rgba, stream);
  // HIP keeps the last error per thread: a call refused here must not leave
  // it for the caller's next, unrelated, check
  if (rc != SDF_OK) (void)hipGetLastError();
  return rc;
}

extern "C" int sdf_render_multi_release(void) {
  std::lock_guard<std::mutex> lock(g_mu);
  if (g_ctx) {
    for (int d : g_ctx->devices) {
      (void)hipSetDevice(d);
      (void)hipDeviceSynchronize();
    }
  }
  g_ctx.reset();
  return SDF_OK;
}

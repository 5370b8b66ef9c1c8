// frames.cpp -- sdf_render_frames: a sequence of whole frames of one scene,
// rendered by a persistent kernel (the frame loop of the reference,
// /root/reference/Code/src/main.cpp:87-98, run on the device for a camera
// path known in advance: an orbit, an animation, an offline sequence).
//
// Each launch takes up to kFramesPerLaunch frames.  Its grid is sized to the
// device (8 waves per SIMD on every CU); the waves take 8x8 tiles of all its
// frames, in order, from one work counter (render_kernel.inc render_frames),
// so no frame ends with an idle tail while its slowest tiles finish, and the
// scene's registers are loaded once per wave instead of once per tile.  The
// pixels are those of sdf_render bit for bit (same shade_pixel).
//
// Work counters: a small per-device pool, zeroed on the caller's stream
// before each launch.  A slot is reused round-robin after kCounterSlots
// launches; each slot's last launch records an event that its next user's
// stream waits for before zeroing it, so any number of launches may be in
// flight on any streams (a reused slot must not be reset under a
// kernel still taking tiles from it).
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/sdf_abi.h"
#include "host_api.h"
#include "kernel_args.h"

namespace sdf {
namespace {

constexpr int kCounterSlots = 64;
constexpr int kSlotBytes = kFrameQueues * kQueueStride * 4;   // one launch's queue counters

struct DeviceFrames {
  uint8_t* counters = nullptr;
  int blocks = 0;                    // persistent grid: 8 waves x 4 SIMDs per CU / 4 waves
  std::mutex mu;                     // slot choice + its event wait/record, per device
  unsigned next = 0;
  hipEvent_t done[kCounterSlots] = {};   // the slot's last launch (recorded after it)
  bool used[kCounterSlots] = {};
};

std::mutex g_mu;
std::vector<DeviceFrames*> g_dev;

DeviceFrames* device_state(int dev) {
  std::lock_guard<std::mutex> lock(g_mu);
  if ((int)g_dev.size() <= dev) g_dev.resize(dev + 1, nullptr);
  if (!g_dev[dev]) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      return nullptr;
    void* p = nullptr;
    if (hipMalloc(&p, kCounterSlots * kSlotBytes) != hipSuccess) return nullptr;
    auto* d = new DeviceFrames;
    d->counters = static_cast<uint8_t*>(p);
    d->blocks = cus * 8;   // 256-thread groups: 4 waves each, 32 waves per CU
    for (hipEvent_t& e : d->done) {
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess) continue;
      // undo this attempt whole: the next call starts afresh
      e = nullptr;
      for (hipEvent_t& x : d->done)
        if (x) (void)hipEventDestroy(x);
      (void)hipFree(d->counters);
      delete d;
      return nullptr;
    }
    g_dev[dev] = d;
  }
  return g_dev[dev];
}

// measurement overrides (tools/frames_probe.py): SDF3D_FRAMES_QUEUES,
// SDF3D_FRAMES_CHUNK
int env_int(const char* name, int dflt, int lo, int hi) {
  const char* e = std::getenv(name);
  if (!e || !*e) return dflt;
  const int v = std::atoi(e);
  return v < lo ? lo : (v > hi ? hi : v);
}

// SDF3D_FRAMES_SCHEDULE=static: the static schedule (measurement only)
int frames_schedule() {
  const char* e = std::getenv("SDF3D_FRAMES_SCHEDULE");
  return e && std::strcmp(e, "static") == 0 ? 1 : 0;
}

}  // namespace
}  // namespace sdf

extern "C" int sdf_render_frames(const sdf_scene* scene, const sdf_camera* cameras, int32_t n,
                                 const sdf_light* light, const sdf_material* material,
                                 const sdf_params* params, void* const* rgba,
                                 int32_t* const* steps, void* stream) {
  if (n < 0 || (n > 0 && (!cameras || !rgba))) return SDF_E_INVALID_ARG;
  if (n == 0) return SDF_OK;
  if (!params) return SDF_E_INVALID_ARG;
  if (params->output_format == SDF_FORMAT_TILES) return SDF_E_UNSUPPORTED;
  for (int i = 0; i < n; ++i) {
    const int rc = sdf_validate(scene, &cameras[i], light, material, params, nullptr);
    if (rc != SDF_OK) return rc;
    if (!rgba[i]) return SDF_E_INVALID_ARG;
  }
  sdf::RenderPlan plan;
  int rc = sdf::make_render_plan(scene, &cameras[0], light, material, params, nullptr, rgba[0],
                                 steps ? steps[0] : nullptr, &plan);
  if (rc != SDF_OK) return rc;
  if (plan.jit) {
    // a run-time specialised scene: its kernel is per frame (jit.cpp)
    for (int i = 0; i < n; ++i) {
      if (i) sdf::plan_set_camera(&plan, &cameras[i]);
      plan.a.rgba = rgba[i];
      plan.a.steps = steps ? steps[i] : nullptr;
      rc = sdf::launch_render_plan(plan, stream);
      if (rc != SDF_OK) return rc;
    }
    return SDF_OK;
  }
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return SDF_E_HIP;
  sdf::DeviceFrames* ds = sdf::device_state(dev);
  if (!ds) return SDF_E_HIP;

  sdf::FramesArgs fa;   // copied into the kernel-argument segment at each launch
  fa.a = plan.a;
  fa.tiles_x = (params->width + 7) / 8;
  fa.tiles_per_frame = fa.tiles_x * ((params->height + 7) / 8);
  const int per_launch = sdf::kFramesPerLaunch;
  for (int f0 = 0; f0 < n; f0 += per_launch) {
    const int nf = n - f0 < per_launch ? n - f0 : per_launch;
    std::memset(fa.frame, 0, sizeof(fa.frame));
    for (int j = 0; j < nf; ++j) {
      sdf::RenderPlan cam_plan;
      cam_plan.a = plan.a;
      sdf::plan_set_camera(&cam_plan, &cameras[f0 + j]);
      sdf::FrameCam& fc = fa.frame[j];
      std::memcpy(fc.inv_view, cam_plan.a.inv_view, sizeof(fc.inv_view));
      std::memcpy(fc.cam, cam_plan.a.cam, sizeof(fc.cam));
      fc.focal = cam_plan.a.focal;
      fc.aspect = cam_plan.a.aspect;
      fc.rgba = rgba[f0 + j];
      fc.steps = steps ? steps[f0 + j] : nullptr;
    }
    fa.nframes = nf;
    std::lock_guard<std::mutex> lock(ds->mu);
    const unsigned slot = ds->next++ % sdf::kCounterSlots;
    fa.counter = reinterpret_cast<uint32_t*>(ds->counters + slot * sdf::kSlotBytes);
    // the slot's previous launch (on whatever stream) ends before it is reset
    if (ds->used[slot] &&
        hipStreamWaitEvent((hipStream_t)stream, ds->done[slot], 0) != hipSuccess)
      return SDF_E_HIP;
    // no more groups than tiles need (4 waves per group)
    const long long items = (long long)nf * fa.tiles_per_frame;
    const long long want = (items + 3) / 4;
    const int blocks = want < ds->blocks ? (int)want : ds->blocks;
    const int nq = sdf::env_int("SDF3D_FRAMES_QUEUES", sdf::kDefaultQueues, 1, sdf::kFrameQueues);
    fa.queues = blocks < nq ? blocks : nq;
    fa.schedule = sdf::frames_schedule();
    fa.chunk = sdf::env_int("SDF3D_FRAMES_CHUNK", sdf::kChunkTiles, 1, 64);
    if (hipMemsetAsync(fa.counter, 0, fa.queues * sdf::kQueueStride * 4, (hipStream_t)stream) !=
        hipSuccess)
      return SDF_E_HIP;
    const int err = plan.exact ? sdf::launch_frames_exact(fa, plan.variant, blocks, stream)
                               : sdf::launch_frames_fast(fa, plan.variant, blocks, stream);
    if (err != hipSuccess) return SDF_E_HIP;
    if (hipEventRecord(ds->done[slot], (hipStream_t)stream) != hipSuccess) return SDF_E_HIP;
    ds->used[slot] = true;
  }
  return SDF_OK;
}

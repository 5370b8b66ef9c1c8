// host_api.h -- library-internal host interfaces shared by the C-ABI
// (sdf_abi.cpp) and the native frame driver (driver.cpp).  Not installed.
#pragma once

#include "../../include/sdf_abi.h"
#include "kernel_args.h"

namespace sdf {

// One validated, prepared render launch: the kernel arguments of an
// sdf_render call (camera hoisted, primitive blocks and culling bounds
// prepared) plus the kernel that serves it.  Building one costs a few
// microseconds of host time; launching one is the kernel launch alone
// (plus the TILES compaction).  sdf_render builds and launches one per call;
// the frame driver keeps one per buffer set and re-launches it every frame.
struct RenderPlan {
  KernelArgs a;
  int variant;             // built-in variant, or kVariantGeneric
  bool jit;                // a run-time specialised kernel is tried first
  bool exact;
  int sig[SDF_MAX_PRIMS];  // the scene signature (jit)
  int nsig;
  int rows;                // 0: nothing to render
  int tiles_ntiles;        // > 0: TILES output, compacted after the render
  uint32_t* tiles_used = nullptr;   // TILES: also receives the stream's length (device)
  RowOrder order{};        // dispatch order of the 8-row blocks (a Schedule's; n = 0: none)
};

// A render schedule (sdf_schedule): the dispatch order of a plan's 8-row
// blocks from the cost the kernels measured for them in earlier frames.
struct Schedule;
Schedule* schedule_create(int rows, int period);
void schedule_destroy(Schedule* s);
// before a launch: the latest order (once a cost snapshot has landed) into
// plan->order, and the cost buffer the kernel adds to
// SDF_E_HIP when the last cost copy failed (the schedule then measures anew)
int schedule_apply(Schedule* s, RenderPlan* plan);
// after the launch on `stream`: every `period` launches a snapshot of the
// costs is copied to the host, behind the launch
int schedule_after(Schedule* s, void* stream);

// Rows a tiling owns (sdf_owned_rows), or SDF_E_INVALID_ARG.
int count_rows(int height, const sdf_tiling& t);
int tiling_run(const sdf_tiling& t);
int tiling_step(const sdf_tiling& t);
int tiling_gap_rows(const sdf_tiling& t);  // (step - 1) * block_rows

// Validate and prepare (tiling NULL = the whole frame).  SDF_OK or an SDF_E_*.
int make_render_plan(const sdf_scene* scene, const sdf_camera* camera, const sdf_light* light,
                     const sdf_material* material, const sdf_params* params,
                     const sdf_tiling* tiling, void* rgba, int32_t* steps, RenderPlan* plan);
// Replace the camera of a prepared plan (validated by the caller).
void plan_set_camera(RenderPlan* plan, const sdf_camera* camera);
// Enqueue a prepared plan on `stream`.  SDF_OK or SDF_E_HIP.
int launch_render_plan(const RenderPlan& plan, void* stream);

}  // namespace sdf

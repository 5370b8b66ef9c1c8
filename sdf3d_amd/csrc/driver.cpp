// driver.cpp -- the native multi-device frame driver (include/sdf_abi.h
// sdf_comm_* / sdf_driver_*).
//
// The reference draws one frame per iteration of its host loop
// (/root/reference/Code/src/main.cpp:87-98, `gl->plot` at :95) on one GL
// context.  Here every rank of a node renders its row blocks of each frame
// and rank 0 assembles the frame; this file is the per-frame loop around the
// kernels, in C++ so that the host cost per frame stays far below the GPU's
// (at N = 8 a rank's share of the 4K frame renders in ~0.06 ms; the same
// loop through torch.distributed costs ~0.12 ms of host time per frame,
// tools/driver_probe.py).
//
// Frames are shipped in BATCHES of `batch` consecutive frames (round 4:
// one length all-gather and one send/recv group per batch instead of per
// frame, so rank 0's host calls and RCCL launches per frame shrink by the
// batch).  Per step i on rank r (b = i mod nbuf):
//   rs[b]  render(i): rank 0 its rows into frame[b] in place, the others
//          their TILES stream into local[b]; the compaction also writes the
//          stream's length into lens[b]                         -> ev_render[b]
//   ship every batch whose last frame is <= i - lag (g its slot):
//     host   wait ev_size[g]: every rank's stream lengths of the batch
//     ds     wait ev_render of its frames; group { send each local[b']
//            (exactly its length) to rank 0 | rank 0: recv every peer's into
//            gathered[b'] }                                      -> ev_gather[g]
//     rs[b'] wait ev_gather[g]; rank 0: decode gathered[b'] into frame[b']
//   if frame i ends a batch (slot g, first buffer b0):
//     ss     wait ev_render of its frames; all-gather of lens[b0 .. b0 +
//            batch) (batch int32 per rank); copy to pinned host -> ev_size[g]
// nbuf % batch == 0, so a batch's lengths are contiguous; lag <= nbuf - batch,
// so a batch is shipped before any of its buffer sets is rendered again.
// Two communicators, each used from one stream only (as torch's process
// groups are): the lengths on ss, the streams on ds.  Every rank issues the
// same RCCL calls in the same order on each, and the two overlap: a frame's
// transfer never waits behind the next frame's length all-gather (which
// waits for a render).  On one stream the two RCCL launches per frame
// serialise: 0.065 against 0.029 ms of host-bound loop per frame
// (tools/driver_probe.py).  Every use of buffer set b is ordered on rs[b]
// (the next render into it follows the decode or waits for the send; on
// rank 0 the next recv into gathered[b] waits for the render that follows
// the decode).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: functions are resolved in the RCCL loaded at run time
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sdf_abi.h"
#include "host_api.h"
#include "kernel_args.h"

namespace {

struct Rccl {
  void* handle = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  // optional: non-blocking creation (sdf_comm_create); without it a helper
  // thread runs the blocking ncclCommInitRank
  ncclResult_t (*CommInitRankConfig)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  // optional: flushes a communicator before it is destroyed; a non-blocking
  // one answers ncclInProgress until that is done (sdf_comm_destroy)
  ncclResult_t (*CommFinalize)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t,
                            hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
};

// One Rccl per library path, loaded once: dlopen of a library the process
// already has mapped (PyTorch's librccl.so) returns that same instance.
Rccl* load_rccl(const char* path) {
  static std::mutex mu;
  static std::vector<std::pair<std::string, Rccl*>> loaded;
  std::lock_guard<std::mutex> lock(mu);
  const std::string key = path && *path ? path : "librccl.so";
  for (auto& e : loaded)
    if (e.first == key) return e.second;
  void* h = dlopen(key.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) return nullptr;
  Rccl* r = new Rccl();
  r->handle = h;
  bool ok = true;
  auto sym = [&](auto& fn, const char* name) {
    fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
    ok = ok && fn != nullptr;
  };
  sym(r->GetUniqueId, "ncclGetUniqueId");
  sym(r->CommInitRank, "ncclCommInitRank");
  sym(r->CommDestroy, "ncclCommDestroy");
  sym(r->CommAbort, "ncclCommAbort");
  sym(r->CommGetAsyncError, "ncclCommGetAsyncError");
  sym(r->AllGather, "ncclAllGather");
  sym(r->Send, "ncclSend");
  sym(r->Recv, "ncclRecv");
  sym(r->GroupStart, "ncclGroupStart");
  sym(r->GroupEnd, "ncclGroupEnd");
  r->CommInitRankConfig = reinterpret_cast<decltype(r->CommInitRankConfig)>(
      dlsym(h, "ncclCommInitRankConfig"));
  r->CommFinalize = reinterpret_cast<decltype(r->CommFinalize)>(dlsym(h, "ncclCommFinalize"));
  if (!ok) {
    delete r;
    dlclose(h);
    return nullptr;
  }
  loaded.emplace_back(key, r);
  return r;
}

}  // namespace

struct sdf_comm {
  Rccl* api;
  ncclComm_t comm;
  int nranks, rank, device;
  bool nonblocking = false;   // created by ncclCommInitRankConfig, blocking = 0
  int timeout_ms = 60000;     // the creation's limit, also teardown's
};

struct sdf_driver {
  int dev = 0;
  int W = 0, H = 0, rank = 0, world = 1, nbuf = 0, lag = 1, flags = 0, timeout_ms = 60000;
  int batch = 1, ngroups = 0;       // frames per ship; batch slots (nbuf / batch)
  bool collectives = false;  // anything shipped at all
  bool sender = false;       // this rank ships a TILES stream
  bool root = false;
  int format = SDF_FORMAT_RGBA32F;
  sdf_comm* size_comm = nullptr;   // lengths (all-gather), on ss
  sdf_comm* data_comm = nullptr;   // streams (send / recv), on ds
  sdf_scene scene;
  sdf_light light;
  sdf_material material;
  sdf_params params;
  sdf_camera camera;
  std::vector<sdf_tiling> tilings;  // every rank's share (packed)
  std::vector<int> rows;
  std::vector<long long> data_off, stream_end;
  std::vector<char> sends;          // rank r ships a stream
  long long pitch = 0;              // gathered part pitch
  std::vector<void*> local, frames, gathered;
  int32_t* sizes_dev = nullptr;     // per batch slot: batch int32 per rank (all-gathered)
  int32_t* sizes_host = nullptr;
  int32_t* zero_dev = nullptr;
  uint32_t* lens_dev = nullptr;     // per buffer set: its stream's length (tiles_move)
  // rank 0: per part, nonzero once a decode found that rank's stream
  // malformed (pinned host memory the decode kernel writes; DecodeParts)
  uint32_t* bad_host = nullptr;
  std::vector<sdf::RenderPlan> plan_send, plan_frame;
  sdf::DecodeParts decode{};
  std::vector<hipStream_t> rs;      // per buffer set (at most kRenderStreams distinct)
  std::vector<hipStream_t> streams;  // the distinct render streams
  hipStream_t ss = nullptr, ds = nullptr;
  std::vector<hipEvent_t> ev_render;          // per buffer set
  std::vector<hipEvent_t> ev_size, ev_gather;  // per batch slot
  struct Batch {
    long long first;   // frame index
    int n;             // frames (< batch only for the one a drain closes)
    int b0;            // buffer set of the first frame (the rest follow it)
    int g;             // batch slot
  };
  std::deque<Batch> pending;
  long long batch_first = 0;   // first frame of the batch being stepped
  int buf_next = 0;            // buffer set of the next frame
  long long nbatches = 0;      // batches closed so far (slot = nbatches mod ngroups)
  // frame index -> buffer set of the last nbuf frames (ring at index mod nbuf):
  // a drain that closes a short batch moves the next batch to the next
  // multiple of `batch`, so that every batch's buffer sets (and lengths) are
  // contiguous
  std::vector<std::pair<long long, int>> frame_buf;
  // buffer set -> the frame last rendered into it: a frame is handed out only
  // while its buffer set still holds it (a drain that closes a short batch
  // moves the next frames onto other buffer sets, so frame_buf alone can name
  // a set that a later frame has taken over)
  std::vector<long long> buf_frame;
  long long next = 0;
  long long shipped = -1;  // highest frame whose streams are shipped and decoded (rank 0)
  int error = SDF_OK;  // sticky: a failed driver refuses further frames
  // host-time accounting (sdf_driver_stats): seconds inside step/drain, and
  // the part of it spent waiting for the GPU or a peer
  double t_calls = 0.0, t_wait = 0.0;
  double t_render = 0.0, t_lengths = 0.0, t_group = 0.0, t_decode = 0.0;  // launches
  long long n_steps = 0;
};

namespace {

// SDF3D_DRIVER_DEBUG=1: every failed HIP / RCCL call is reported on stderr
// with its source line and error (diagnosis of multi-rank runs)
bool debug_on() {
  static const bool on = [] {
    const char* e = std::getenv("SDF3D_DRIVER_DEBUG");
    return e && *e && *e != '0';
  }();
  return on;
}
// SDF3D_DRIVER_DEBUG=2: also hand out the frames of a driver that has failed
// (fault diagnosis only: a malformed stream's tiles then hold older pixels)
bool debug_read_failed() {
  static const bool on = [] {
    const char* e = std::getenv("SDF3D_DRIVER_DEBUG");
    return e && std::atoi(e) >= 2;
  }();
  return on;
}
int hip_ok(hipError_t e, int line = __builtin_LINE()) {
  if (e == hipSuccess) return SDF_OK;
  if (debug_on())
    std::fprintf(stderr, "sdf driver: HIP error %d (%s) at driver.cpp:%d\n", (int)e,
                 hipGetErrorString(e), line);
  return SDF_E_HIP;
}
int nccl_ok(ncclResult_t e, int line = __builtin_LINE()) {
  if (e == ncclSuccess) return SDF_OK;
  if (debug_on()) std::fprintf(stderr, "sdf driver: RCCL error %d at driver.cpp:%d\n", (int)e, line);
  return SDF_E_COMM;
}

// A communicator created non-blocking (sdf_comm_create) may answer any call
// with ncclInProgress while RCCL finishes it in the background; the next call
// on it must wait for the communicator to settle (ncclCommGetAsyncError
// leaving ncclInProgress), polled here with a limit.
ncclResult_t settle(const sdf_comm* c, ncclResult_t rc, int timeout_ms) {
  if (rc != ncclInProgress) return rc;
  const auto t0 = std::chrono::steady_clock::now();
  const auto limit = std::chrono::milliseconds(timeout_ms > 0 ? timeout_ms : 60000);
  for (unsigned n = 0;; ++n) {
    ncclResult_t st = ncclSuccess;
    if (c->api->CommGetAsyncError(c->comm, &st) != ncclSuccess) return ncclSystemError;
    if (st != ncclInProgress) return st;
    if ((n & 63) == 63) {
      if (std::chrono::steady_clock::now() - t0 > limit) return ncclInProgress;
      sched_yield();
    }
  }
}

int fail(sdf_driver* d, int rc) {
  if (rc != SDF_OK && d->error == SDF_OK) d->error = rc;
  return rc;
}

// Abort the communicators so that no rank blocks forever on a peer that
// failed: the process can then report the error and exit.
void abort_comms(sdf_driver* d) {
  for (sdf_comm* c : {d->size_comm, d->data_comm})
    if (c && c->comm) {
      c->api->CommAbort(c->comm);
      c->comm = nullptr;
    }
}

// Wait for `done()` on the host, polling; gives up after the driver's limit
// or at the first asynchronous RCCL error.
using Clock = std::chrono::steady_clock;
double seconds_since(Clock::time_point t0) {
  return std::chrono::duration<double>(Clock::now() - t0).count();
}

template <class Query>
int host_wait(sdf_driver* d, Query done) {
  hipError_t q = done();
  if (q == hipSuccess) return SDF_OK;
  const auto t0 = Clock::now();
  struct Account {
    sdf_driver* d;
    Clock::time_point t0;
    ~Account() { d->t_wait += seconds_since(t0); }
  } account{d, t0};
  for (unsigned n = 0; q == hipErrorNotReady; q = done(), ++n) {
    if ((n & 1023) == 1023) {
      for (sdf_comm* c : {d->size_comm, d->data_comm}) {
        ncclResult_t ae = ncclSuccess;
        if (c && c->comm && c->api->CommGetAsyncError(c->comm, &ae) == ncclSuccess &&
            ae != ncclSuccess && ae != ncclInProgress) {
          abort_comms(d);
          return fail(d, SDF_E_COMM);
        }
      }
      const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                          std::chrono::steady_clock::now() - t0).count();
      if (ms > d->timeout_ms) {
        abort_comms(d);
        return fail(d, SDF_E_TIMEOUT);
      }
    }
    sched_yield();
  }
  return fail(d, hip_ok(q));
}

int wait_event(sdf_driver* d, hipEvent_t e) {
  return host_wait(d, [e] { return hipEventQuery(e); });
}

// ship(batch): the agreed lengths are on the host; move the batch's streams
// to rank 0 in one group and decode them there.
int ship(sdf_driver* d, const sdf_driver::Batch& bt) {
  const int g = bt.g;
  int rc = wait_event(d, d->ev_size[g]);
  if (rc != SDF_OK) return rc;
  // rank r's length of the batch's f-th frame: sz[r * batch + f]
  const int32_t* sz = d->sizes_host + (size_t)g * d->batch * d->world;
  for (int f = 0; f < bt.n; ++f)
    for (int r = 0; r < d->world; ++r) {
      const int32_t n = sz[(size_t)r * d->batch + f];
      if (d->sends[r] && (n < 0 || d->data_off[r] + n > d->stream_end[r]))
        return fail(d, SDF_E_COMM);  // a length no stream of that rank can have
    }
  for (int f = 0; f < bt.n && rc == SDF_OK; ++f)
    rc = hip_ok(hipStreamWaitEvent(d->ds, d->ev_render[bt.b0 + f], 0));
  if (rc != SDF_OK) return fail(d, rc);
  const Rccl& R = *d->data_comm->api;
  ncclComm_t comm = d->data_comm->comm;
  auto tg = Clock::now();
  rc = nccl_ok(R.GroupStart());
  for (int f = 0; f < bt.n && rc == SDF_OK; ++f) {
    const int b = bt.b0 + f;
    if (d->sender)
      rc = nccl_ok(R.Send(d->local[b],
                          (size_t)(d->data_off[d->rank] + sz[(size_t)d->rank * d->batch + f]),
                          ncclUint8, 0, comm, d->ds));
    if (d->root)
      for (int r = 0; r < d->world && rc == SDF_OK; ++r)
        if (d->sends[r])
          rc = nccl_ok(R.Recv(static_cast<char*>(d->gathered[b]) + (size_t)r * d->pitch,
                              (size_t)(d->data_off[r] + sz[(size_t)r * d->batch + f]), ncclUint8,
                              r, comm, d->ds));
  }
  // (a non-blocking communicator may still be enqueueing: settle before the
  // event below is recorded behind the group's kernels)
  const int rc_end = nccl_ok(settle(d->data_comm, R.GroupEnd(), d->timeout_ms));
  d->t_group += seconds_since(tg);
  if (rc == SDF_OK) rc = rc_end;
  if (rc != SDF_OK) return fail(d, rc);
  rc = hip_ok(hipEventRecord(d->ev_gather[g], d->ds));
  for (int f = 0; f < bt.n && rc == SDF_OK; ++f) {
    const int b = bt.b0 + f;
    rc = hip_ok(hipStreamWaitEvent(d->rs[b], d->ev_gather[g], 0));
    if (rc == SDF_OK && d->root) {
      // each received stream must be exactly the length its rank announced
      for (int r = 0; r < d->world; ++r)
        d->decode.used[r] = d->sends[r] ? sz[(size_t)r * d->batch + f] : -1;
      tg = Clock::now();
      rc = hip_ok((hipError_t)sdf::launch_tiles_decode(d->decode, d->frames[b], d->gathered[b],
                                                       d->rs[b]));
      d->t_decode += seconds_since(tg);
    }
  }
  if (rc == SDF_OK) d->shipped = bt.first + bt.n - 1;
  return fail(d, rc);
}

// The stream lengths of the batch [first, first + n) to every rank: one
// all-gather of `batch` int32 per rank (entries past n are ignored), copied
// to pinned host memory; the batch then waits in `pending` for its ship.
int gather_lengths(sdf_driver* d, long long first, int n, int b0) {
  const auto tr = Clock::now();
  const int g = (int)(d->nbatches++ % d->ngroups);
  int rc = SDF_OK;
  for (int f = 0; f < n && rc == SDF_OK; ++f)
    rc = hip_ok(hipStreamWaitEvent(d->ss, d->ev_render[b0 + f], 0));
  if (rc != SDF_OK) return fail(d, rc);
  int32_t* sz = d->sizes_dev + (size_t)g * d->batch * d->world;
  const void* src = d->sender ? (const void*)(d->lens_dev + b0) : (const void*)d->zero_dev;
  rc = nccl_ok(settle(d->size_comm,
                      d->size_comm->api->AllGather(src, sz, (size_t)d->batch, ncclInt32,
                                                   d->size_comm->comm, d->ss),
                      d->timeout_ms));
  if (rc == SDF_OK)
    rc = hip_ok(hipMemcpyAsync(d->sizes_host + (size_t)g * d->batch * d->world, sz,
                               sizeof(int32_t) * d->batch * d->world, hipMemcpyDeviceToHost,
                               d->ss));
  if (rc == SDF_OK) rc = hip_ok(hipEventRecord(d->ev_size[g], d->ss));
  d->t_lengths += seconds_since(tr);
  if (rc != SDF_OK) return fail(d, rc);
  d->pending.push_back({first, n, b0, g});
  return SDF_OK;
}

// A decode found a malformed stream (a truncated or mismatched receive):
// the ranks no longer agree on what was sent, so the communicators are
// aborted and the driver fails with SDF_E_COMM.
int check_streams(sdf_driver* d) {
  if (!d->bad_host) return SDF_OK;
  const volatile uint32_t* bad = d->bad_host;
  for (int r = 0; r < d->world; ++r)
    if (bad[r] != 0u) {
      if (debug_on())
        std::fprintf(stderr, "sdf driver: rank %d's stream was malformed (code %u)\n", r, bad[r]);
      abort_comms(d);
      return fail(d, SDF_E_COMM);
    }
  return SDF_OK;
}

void release(sdf_driver* d) {
  (void)hipSetDevice(d->dev);
  for (auto* v : {&d->local, &d->frames, &d->gathered})
    for (void* p : *v)
      if (p) (void)hipFree(p);
  if (d->sizes_dev) (void)hipFree(d->sizes_dev);
  if (d->zero_dev) (void)hipFree(d->zero_dev);
  if (d->lens_dev) (void)hipFree(d->lens_dev);
  if (d->sizes_host) (void)hipHostFree(d->sizes_host);
  if (d->bad_host) (void)hipHostFree(d->bad_host);
  for (hipStream_t s : d->streams)
    if (s) (void)hipStreamDestroy(s);
  if (d->ss) (void)hipStreamDestroy(d->ss);
  if (d->ds) (void)hipStreamDestroy(d->ds);
  for (auto* v : {&d->ev_render, &d->ev_size, &d->ev_gather})
    for (hipEvent_t e : *v)
      if (e) (void)hipEventDestroy(e);
  delete d;
}

}  // namespace

extern "C" {

int sdf_comm_unique_id(const char* rccl_path, void* id) {
  if (!id) return SDF_E_INVALID_ARG;
  Rccl* R = load_rccl(rccl_path);
  if (!R) return SDF_E_COMM;
  ncclUniqueId uid;
  if (R->GetUniqueId(&uid) != ncclSuccess) return SDF_E_COMM;
  std::memcpy(id, &uid, sizeof(uid));
  return SDF_OK;
}

// Creation waits until every rank has joined, at most `timeout_ms`: a peer
// that never joins (it failed, or the id is from an earlier run) gives
// SDF_E_TIMEOUT.  With ncclCommInitRankConfig the communicator is created
// non-blocking (config.blocking = 0) and polled with ncclCommGetAsyncError;
// on the limit it is aborted (ncclCommAbort), so nothing of it is left
// running in the process.  An RCCL without that entry point gets the blocking
// ncclCommInitRank on a helper thread, which on a timeout is left blocked
// (it aborts the communicator if it ever returns).
int sdf_comm_create(const char* rccl_path, const void* id, int32_t nranks, int32_t rank,
                    int32_t timeout_ms, sdf_comm** comm) {
  if (!id || !comm || nranks < 1 || rank < 0 || rank >= nranks) return SDF_E_INVALID_ARG;
  *comm = nullptr;
  Rccl* R = load_rccl(rccl_path);
  if (!R) return SDF_E_COMM;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return SDF_E_NO_DEVICE;
  if (R->CommInitRankConfig) {
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclConfig_t config = NCCL_CONFIG_INITIALIZER;
    config.blocking = 0;
    ncclComm_t c = nullptr;
    ncclResult_t rc = R->CommInitRankConfig(&c, nranks, uid, rank, &config);
    if (rc != ncclSuccess && rc != ncclInProgress) {
      if (c) R->CommAbort(c);
      return SDF_E_COMM;
    }
    const int limit = timeout_ms > 0 ? timeout_ms : 120000;
    sdf_comm probe{R, c, nranks, rank, dev, true, limit};
    rc = c ? settle(&probe, ncclInProgress, limit) : ncclSystemError;
    if (rc != ncclSuccess) {
      if (c) R->CommAbort(c);
      return rc == ncclInProgress ? SDF_E_TIMEOUT : SDF_E_COMM;
    }
    *comm = new sdf_comm{R, c, nranks, rank, dev, true, limit};
    return SDF_OK;
  }
  struct Init {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    ncclResult_t rc = ncclSuccess;
    ncclComm_t c = nullptr;
  };
  auto st = std::make_shared<Init>();
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  std::thread([st, R, uid, nranks, rank, dev] {
    (void)hipSetDevice(dev);
    ncclComm_t c = nullptr;
    const ncclResult_t rc = R->CommInitRank(&c, nranks, uid, rank);
    std::lock_guard<std::mutex> lock(st->mu);
    if (st->abandoned) {  // the caller gave up: nobody will use it
      if (rc == ncclSuccess && c) R->CommAbort(c);
      return;
    }
    st->rc = rc;
    st->c = c;
    st->done = true;
    st->cv.notify_all();
  }).detach();
  std::unique_lock<std::mutex> lock(st->mu);
  const auto limit = std::chrono::milliseconds(timeout_ms > 0 ? timeout_ms : 120000);
  if (!st->cv.wait_for(lock, limit, [&] { return st->done; })) {
    st->abandoned = true;
    return SDF_E_TIMEOUT;
  }
  if (st->rc != ncclSuccess || !st->c) return SDF_E_COMM;
  *comm = new sdf_comm{R, st->c, nranks, rank, dev, false,
                       timeout_ms > 0 ? timeout_ms : 120000};
  return SDF_OK;
}

// A communicator created non-blocking may answer ncclInProgress while RCCL
// tears it down.  Where RCCL has ncclCommFinalize, such a
// communicator is finalised first and polled to completion (settle, within
// the limit its creation was given; rccl.h: the state becomes ncclSuccess
// once it is globally quiescent), then destroyed, which then only frees local
// resources; a finalise that fails or times out aborts the communicator
// instead.  A blocking communicator (the fallback creation) is not finalised:
// a blocking ncclCommFinalize could wait without limit for a peer that is
// gone.  Without ncclCommFinalize the destroy is the whole
// teardown (an ncclInProgress answer is not an error: the handle is gone, so
// there is nothing left to poll).
int sdf_comm_destroy(sdf_comm* comm) {
  if (!comm) return SDF_OK;
  int rc = SDF_OK;
  if (comm->comm) {
    const int limit = comm->timeout_ms > 0 ? comm->timeout_ms : 60000;
    if (comm->api->CommFinalize && comm->nonblocking) {
      rc = nccl_ok(settle(comm, comm->api->CommFinalize(comm->comm), limit));
      if (rc != SDF_OK) {
        comm->api->CommAbort(comm->comm);
        comm->comm = nullptr;
      }
    }
    if (comm->comm) {
      const ncclResult_t d = comm->api->CommDestroy(comm->comm);
      if (rc == SDF_OK) rc = nccl_ok(d == ncclInProgress ? ncclSuccess : d);
    }
  }
  delete comm;
  return rc;
}

int sdf_driver_create(const sdf_scene* scene, const sdf_camera* camera, const sdf_light* light,
                      const sdf_material* material, const sdf_params* params,
                      const sdf_driver_config* config, sdf_comm* size_comm, sdf_comm* data_comm,
                      sdf_driver** driver) {
  if (!config || !driver || !params) return SDF_E_INVALID_ARG;
  *driver = nullptr;
  const sdf_driver_config& c = *config;
  const int batch = c.batch > 0 ? c.batch : 1;
  if (c.world < 1 || c.world > SDF_MAX_DECODE_PARTS || c.rank < 0 || c.rank >= c.world ||
      c.share_root < 1 || c.share_peer < 1 || c.nbuf < 2 || c.nbuf > 16 || c.lag < 1 ||
      batch > 16 || c.nbuf % batch != 0 || c.lag > c.nbuf - batch ||
      (c.flags & ~SDF_DRIVER_ROOT_AS_PEER) != 0)
    return SDF_E_INVALID_ARG;
  const bool peer_root = (c.flags & SDF_DRIVER_ROOT_AS_PEER) != 0;
  const bool collectives = c.world > 1 || peer_root;
  if (collectives) {
    for (sdf_comm* cm : {size_comm, data_comm})
      if (!cm || !cm->comm || cm->nranks != c.world || cm->rank != c.rank)
        return SDF_E_INVALID_ARG;
    if (size_comm == data_comm) return SDF_E_INVALID_ARG;
    if (params->output_format != SDF_FORMAT_RGBA32F) return SDF_E_UNSUPPORTED;
  } else if (params->output_format == SDF_FORMAT_TILES) {
    return SDF_E_UNSUPPORTED;
  }
  int rc = sdf_validate(scene, camera, light, material, params, nullptr);
  if (rc != SDF_OK) return rc;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return SDF_E_NO_DEVICE;

  sdf_driver* d = new sdf_driver();
  d->dev = dev;
  d->W = params->width;
  d->H = params->height;
  d->rank = c.rank;
  d->world = c.world;
  d->nbuf = c.nbuf;
  d->lag = c.lag;
  d->batch = batch;
  d->ngroups = c.nbuf / batch;
  d->frame_buf.assign(c.nbuf, {-1, 0});
  d->buf_frame.assign(c.nbuf, -1);
  d->flags = c.flags;
  d->timeout_ms = c.timeout_ms > 0 ? c.timeout_ms : 60000;
  d->collectives = collectives;
  d->root = c.rank == 0;
  d->format = params->output_format;
  d->size_comm = size_comm;
  d->data_comm = data_comm;
  d->scene = *scene;
  d->light = *light;
  d->material = *material;
  d->params = *params;
  d->camera = *camera;

  // every rank's share: rank 0 a blocks, the others b, per period a + b (N - 1)
  // (sdf_share_tiling)
  for (int r = 0; r < c.world; ++r) {
    sdf_tiling t;
    const int n = sdf_share_tiling(r, c.world, c.share_root, c.share_peer, &t) == SDF_OK
                      ? sdf::count_rows(d->H, t)
                      : SDF_E_INVALID_ARG;
    if (n < 0) {
      release(d);
      return SDF_E_INVALID_ARG;
    }
    const sdf::TilesLayout L(int64_t((d->W + 7) / 8) * ((n + 7) / 8));
    d->tilings.push_back(t);
    d->rows.push_back(n);
    d->data_off.push_back((long long)L.data);
    d->stream_end.push_back((long long)L.stream_end);
    d->sends.push_back(collectives && (r != 0 || peer_root) && n > 0);
    d->pitch = std::max(d->pitch, (long long)((L.stream_end + 255) / 256 * 256));
  }
  d->sender = d->sends[c.rank] != 0;

  sdf_params pf = *params;  // the frame's own rows / whole frames
  sdf_params pt = *params;  // the wire
  pt.output_format = SDF_FORMAT_TILES;
  const size_t frame_bytes = (size_t)d->W * d->H * (size_t)sdf_format_bytes(pf.output_format);
  const size_t local_bytes = (size_t)sdf_tiles_bytes(d->W, d->rows[c.rank]);
  auto alloc = [&](void** p, size_t n) {
    return rc == SDF_OK ? (rc = hip_ok(hipMalloc(p, n ? n : 16))) : rc;
  };
  // render streams: one per buffer set, at most kRenderStreams distinct
  // (buffer set b on stream b mod kRenderStreams).  Round 6: up to 8 (was
  // 4): a peer's share of the Mandelbulb frame, whose long tiles leave long
  // launch tails, renders as TILES 11 % faster on 8 streams than on 4
  // (tools/tiles_overhead_probe.py, profiles/r06_tiles_overhead.jsonl);
  // bench.py keeps 4 buffer sets by default
  constexpr int kRenderStreams = 8;
  d->streams.assign(std::min(c.nbuf, kRenderStreams), nullptr);
  for (hipStream_t& st : d->streams)
    if (rc == SDF_OK) rc = hip_ok(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  d->rs.assign(c.nbuf, nullptr);
  for (int b = 0; b < c.nbuf; ++b) d->rs[b] = d->streams[b % d->streams.size()];
  d->ev_render.assign(c.nbuf, nullptr);
  d->ev_size.assign(d->ngroups, nullptr);
  d->ev_gather.assign(d->ngroups, nullptr);
  for (auto* v : {&d->ev_render, &d->ev_size, &d->ev_gather})
    for (hipEvent_t& e : *v)
      if (rc == SDF_OK) rc = hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (rc == SDF_OK) rc = hip_ok(hipStreamCreateWithFlags(&d->ss, hipStreamNonBlocking));
  if (rc == SDF_OK) rc = hip_ok(hipStreamCreateWithFlags(&d->ds, hipStreamNonBlocking));
  d->local.assign(c.nbuf, nullptr);
  d->frames.assign(c.nbuf, nullptr);
  d->gathered.assign(c.nbuf, nullptr);
  d->plan_send.resize(c.nbuf);
  d->plan_frame.resize(c.nbuf);
  if (d->sender) {
    // every buffer set's stream length (a rank that owns no rows keeps 0)
    alloc((void**)&d->lens_dev, sizeof(uint32_t) * c.nbuf);
    if (rc == SDF_OK) rc = hip_ok(hipMemset(d->lens_dev, 0, sizeof(uint32_t) * c.nbuf));
  }
  for (int b = 0; b < c.nbuf && rc == SDF_OK; ++b) {
    if (d->sender) {
      alloc(&d->local[b], local_bytes);
      // the header of a stream no render writes (0 rows) must read used = 0
      if (rc == SDF_OK) rc = hip_ok(hipMemset(d->local[b], 0, 64));
      if (rc == SDF_OK)
        rc = sdf::make_render_plan(scene, camera, light, material, &pt, &d->tilings[c.rank],
                                   d->local[b], nullptr, &d->plan_send[b]);
      d->plan_send[b].tiles_used = d->lens_dev + b;
    }
    if (d->root) {
      alloc(&d->frames[b], frame_bytes);
      if (collectives) {
        // part r of gathered[b] at r * pitch; parts nobody sends keep a
        // zero header (ntiles = 0: skipped by the decode)
        alloc(&d->gathered[b], (size_t)d->pitch * c.world);
        if (rc == SDF_OK)
          rc = hip_ok(hipMemset(d->gathered[b], 0, (size_t)d->pitch * c.world));
      }
      if (rc == SDF_OK && !d->sender) {
        // rank 0's own rows straight into the frame (whole frames at world 1)
        sdf_tiling t = d->tilings[0];
        if (collectives) t.flags = SDF_TILING_FRAME_ROWS;
        rc = sdf::make_render_plan(scene, camera, light, material, &pf, &t, d->frames[b],
                                   nullptr, &d->plan_frame[b]);
      }
    }
  }
  if (collectives && rc == SDF_OK) {
    // batch slots x batch frames x world ranks (= nbuf x world)
    alloc((void**)&d->sizes_dev, sizeof(int32_t) * c.nbuf * c.world);
    alloc((void**)&d->zero_dev, 64);   // a non-sending rank's lengths (batch <= 16)
    if (rc == SDF_OK) rc = hip_ok(hipMemset(d->zero_dev, 0, 64));
    if (rc == SDF_OK)
      rc = hip_ok(hipHostMalloc((void**)&d->sizes_host, sizeof(int32_t) * c.nbuf * c.world,
                                hipHostMallocDefault));
    if (d->root && rc == SDF_OK) {
      rc = hip_ok(hipHostMalloc((void**)&d->bad_host, sizeof(uint32_t) * c.world,
                                hipHostMallocDefault));
      if (rc == SDF_OK) std::memset(d->bad_host, 0, sizeof(uint32_t) * c.world);
      d->decode.status = d->bad_host;
    }
    d->decode.nparts = c.world;
    d->decode.width = d->W;
    d->decode.height = d->H;
    d->decode.part_stride = d->pitch;
    for (int r = 0; r < c.world; ++r) {
      const sdf_tiling& t = d->tilings[r];
      d->decode.rows[r] = d->rows[r];
      d->decode.first_block[r] = t.first_block;
      d->decode.block_stride[r] = t.block_stride;
      d->decode.block_rows[r] = t.block_rows;
      d->decode.chunk_rows[r] = t.block_rows * sdf::tiling_run(t);
      d->decode.run_gap_rows[r] = sdf::tiling_gap_rows(t);
    }
  }
  if (rc == SDF_OK) rc = hip_ok(hipDeviceSynchronize());  // memsets done
  if (rc != SDF_OK) {
    release(d);
    return rc;
  }
  *driver = d;
  return SDF_OK;
}

int sdf_driver_set_camera(sdf_driver* d, const sdf_camera* camera) {
  if (!d) return SDF_E_INVALID_ARG;
  const int rc = sdf_validate(&d->scene, camera, &d->light, &d->material, &d->params, nullptr);
  if (rc != SDF_OK) return rc;
  d->camera = *camera;
  for (auto* v : {&d->plan_send, &d->plan_frame})
    for (sdf::RenderPlan& p : *v)
      if (p.rows > 0) sdf::plan_set_camera(&p, camera);
  return SDF_OK;
}

static int driver_step(sdf_driver* d, int64_t* frame_index);

int sdf_driver_step(sdf_driver* d, int64_t* frame_index) {
  if (!d) return SDF_E_INVALID_ARG;
  const auto t0 = Clock::now();
  const int rc = driver_step(d, frame_index);
  d->t_calls += seconds_since(t0);
  d->n_steps++;
  return rc;
}

static int driver_step(sdf_driver* d, int64_t* frame_index) {
  if (d->error != SDF_OK) return d->error;
  if (check_streams(d) != SDF_OK) return d->error;
  if (hipSetDevice(d->dev) != hipSuccess) return fail(d, SDF_E_HIP);
  const long long i = d->next;
  const int b = d->buf_next;
  hipStream_t s = d->rs[b];
  int rc = SDF_OK;
  auto tr = Clock::now();
  if (d->sender) rc = sdf::launch_render_plan(d->plan_send[b], s);
  if (rc == SDF_OK && d->root && !d->sender) rc = sdf::launch_render_plan(d->plan_frame[b], s);
  d->t_render += seconds_since(tr);
  if (rc != SDF_OK && debug_on())
    std::fprintf(stderr, "sdf driver: render launch failed (%d): %s\n", rc,
                 hipGetErrorString(hipGetLastError()));
  if (rc != SDF_OK) return fail(d, rc);
  if (frame_index) *frame_index = i;
  d->next = i + 1;
  d->frame_buf[i % d->nbuf] = {i, b};
  d->buf_frame[b] = i;
  d->buf_next = (b + 1) % d->nbuf;
  if (!d->collectives) return SDF_OK;
  rc = hip_ok(hipEventRecord(d->ev_render[b], s));
  if (rc != SDF_OK) return fail(d, rc);
  // batches whose last frame is at least `lag` frames old: their lengths are
  // on the host by now (lag >= 2: long since)
  while (!d->pending.empty() &&
         d->pending.front().first + d->pending.front().n - 1 <= i - d->lag) {
    const sdf_driver::Batch bt = d->pending.front();
    d->pending.pop_front();
    rc = ship(d, bt);
    if (rc != SDF_OK) return rc;
  }
  // frame i ends a batch: its lengths to every rank
  if (i + 1 - d->batch_first == d->batch) {
    const long long first = d->batch_first;
    d->batch_first = i + 1;
    return gather_lengths(d, first, d->batch, b + 1 - d->batch);
  }
  return SDF_OK;
}

static int driver_drain(sdf_driver* d);

int sdf_driver_drain(sdf_driver* d) {
  if (!d) return SDF_E_INVALID_ARG;
  const auto t0 = Clock::now();
  const int rc = driver_drain(d);
  d->t_calls += seconds_since(t0);
  return rc;
}

static int driver_drain(sdf_driver* d) {
  if (d->error != SDF_OK) return d->error;
  if (hipSetDevice(d->dev) != hipSuccess) return fail(d, SDF_E_HIP);
  // a batch the last steps began but did not complete goes as it is (every
  // rank has stepped the same frames)
  if (d->collectives && d->next > d->batch_first) {
    const long long first = d->batch_first;
    const int n = (int)(d->next - first);
    const int b0 = (d->buf_next - n + d->nbuf) % d->nbuf;
    d->batch_first = d->next;
    // the next batch starts on a multiple of `batch` (contiguous buffer sets)
    d->buf_next = (d->buf_next + d->batch - 1) / d->batch * d->batch % d->nbuf;
    const int rc = gather_lengths(d, first, n, b0);
    if (rc != SDF_OK) return rc;
  }
  while (!d->pending.empty()) {
    const sdf_driver::Batch bt = d->pending.front();
    d->pending.pop_front();
    const int rc = ship(d, bt);
    if (rc != SDF_OK) return rc;
  }
  std::vector<hipStream_t> all = d->streams;
  all.push_back(d->ss);
  all.push_back(d->ds);
  for (hipStream_t s : all) {
    const int rc = host_wait(d, [s] { return hipStreamQuery(s); });
    if (rc != SDF_OK) return rc;
  }
  return check_streams(d);   // every decode has completed
}

int sdf_driver_frame(sdf_driver* d, int64_t index, void** rgba) {
  if (!d || !rgba) return SDF_E_INVALID_ARG;
  *rgba = nullptr;
  // a driver that has failed hands out no frame: a malformed peer stream
  // leaves its tiles holding an older frame's pixels; the
  // status words of decodes already completed are polled here too
  if (!debug_read_failed()) {
    if (d->error != SDF_OK) return d->error;
    if (check_streams(d) != SDF_OK) return d->error;
  }
  if (!d->root || index < 0 || index >= d->next || index < d->next - d->nbuf)
    return SDF_E_INVALID_ARG;
  // with collectives a frame holds the peers' rows only once it has been
  // shipped (the last `lag` frames stepped: after sdf_driver_drain)
  if (d->collectives && index > d->shipped) return SDF_E_INVALID_ARG;
  const auto& fb = d->frame_buf[index % d->nbuf];
  if (fb.first != index || d->buf_frame[fb.second] != index) return SDF_E_INVALID_ARG;
  *rgba = d->frames[fb.second];
  return SDF_OK;
}

int sdf_driver_read_frame(sdf_driver* d, int64_t index, void* dst, int64_t bytes, void* stream) {
  void* src = nullptr;
  int rc = sdf_driver_frame(d, index, &src);
  if (rc != SDF_OK) return rc;
  const size_t n = (size_t)d->W * d->H * (size_t)sdf_format_bytes(d->format);
  if (!dst || bytes < (int64_t)n) return SDF_E_INVALID_ARG;
  if (hipSetDevice(d->dev) != hipSuccess) return SDF_E_HIP;
  // after everything queued for the frame's buffer set (render, decode)
  const int b = d->frame_buf[index % d->nbuf].second;
  hipEvent_t e = nullptr;
  rc = hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (rc == SDF_OK) rc = hip_ok(hipEventRecord(e, d->rs[b]));
  if (rc == SDF_OK) rc = hip_ok(hipStreamWaitEvent((hipStream_t)stream, e, 0));
  if (rc == SDF_OK)
    rc = hip_ok(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, (hipStream_t)stream));
  if (e) (void)hipEventDestroy(e);
  return rc;
}

int sdf_driver_stats(sdf_driver* d, double* out, int32_t n) {
  if (!d || !out || n < 3) return SDF_E_INVALID_ARG;
  const double v[7] = {(double)d->n_steps, d->t_calls, d->t_wait, d->t_render,
                       d->t_lengths, d->t_group, d->t_decode};
  for (int i = 0; i < n && i < 7; ++i) out[i] = v[i];
  return SDF_OK;
}

int sdf_driver_destroy(sdf_driver* d) {
  if (!d) return SDF_OK;
  int rc = SDF_OK;
  if (d->error == SDF_OK) rc = sdf_driver_drain(d);
  release(d);
  return rc;
}

}  // extern "C"

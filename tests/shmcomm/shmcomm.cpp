// shmcomm.cpp -- TEST INFRASTRUCTURE ONLY: a stand-in for the RCCL symbols the
// native frame driver loads at run time (sdf3d_amd/csrc/driver.cpp load_rccl:
// ncclGetUniqueId, ncclCommInitRank(Config), ncclCommDestroy, ncclCommAbort,
// ncclCommGetAsyncError, ncclAllGather, ncclSend, ncclRecv, ncclGroupStart,
// ncclGroupEnd), so that the driver's multi-rank sequence can run with
// several ranks on ONE GPU, which RCCL refuses ("Duplicate GPU detected").
//
// Every rank is a process; a communicator is one POSIX shared-memory segment
// named by the unique id.  Data moves through host memory.
//
// ASYNCHRONOUS, like RCCL (round 3; VERDICT r02: the round-2 stand-in
// completed every call before returning, so it could not show a missing
// stream dependency or a cross-communicator ordering hazard).  A call returns
// as soon as it is enqueued:
//   * it records an event on the caller's stream (the work the collective is
//     ordered after) and makes the stream wait, on the GPU, for the call's
//     completion flag (hipStreamWaitValue32 on coherent host memory);
//   * ONE progress engine per process runs the calls of ALL its
//     communicators in the order they were issued: it waits for the call's
//     event, moves the data (device -> shared memory -> device, on a private
//     stream), then writes the flag (a host store to coherent memory),
//     releasing the caller's stream.
// So the driver's streams see RCCL's ordering (nothing after a collective on
// its stream runs before the collective's data is in place; nothing else is
// ordered), and the single FIFO engine is STRICTER than RCCL across
// communicators: ranks that issue calls on two communicators in different
// orders deadlock here and hit the time limit, so every rank must issue its
// calls in one global order.  Sends and receives inside a group are
// progressed together, chunk by chunk, so any pattern (rank 0 receiving from
// 7 peers, a rank sending to itself) completes.  Every wait polls with a
// limit (SHMCOMM_TIMEOUT_MS, default 60 s) and then sets the communicator's
// asynchronous error, as a failed RCCL would -- and still writes the flag, so
// no GPU stream is left waiting.  A stream held by a wait packet holds the
// hardware queue it sits on, so every stream of a test process needs a queue
// of its own, as on real hardware for RCCL's spinning kernels: the tests run
// with GPU_MAX_HW_QUEUES=8 (as bench.py's N > 1 runs) or 16; a rank holds
// the default stream, its render streams, the driver's two communication
// streams and this library's one copy stream.  SHMCOMM_SYNC=1 (or a device without
// stream wait-value support) selects the round-2 behaviour: each call waits
// for its stream and completes before returning.
//
// SHMCOMM_NONBLOCKING=1 (round 4) mimics RCCL's non-blocking
// communicators (ncclConfig_t.blocking = 0), whose calls may answer
// ncclInProgress while they are still being set up: ncclCommInitRankConfig
// returns at once with the join running on a helper thread; ncclAllGather,
// ncclGroupEnd and ncclCommFinalize return ncclInProgress and are enqueued
// (their stream event and wait recorded) a little later by a helper thread,
// in issue order; ncclCommGetAsyncError reports ncclInProgress until that is
// done.  A caller that records stream work behind such a call without
// settling it first (polling ncclCommGetAsyncError) orders that work before
// the collective -- the tests catch it as wrong data.  ncclCommAbort during
// the join stops it.  SHMCOMM_STATS=1 prints the counts of ncclInProgress
// answers and aborts to stderr at exit.  Never linked into the product
// library; tests load it through the driver's rccl_path.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types and signatures only
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr uint64_t kMagic = 0x53444633444d4d43ull;  // "SDF3DMMC"
constexpr int kAgSlots = 4;                           // all-gather ops in flight
constexpr size_t kAgBytes = 64 << 10;                 // per rank per all-gather
constexpr int kChSlots = 4;                           // chunks in flight per channel
constexpr size_t kChunk = 256 << 10;                  // bytes per chunk

struct Header {
  uint64_t magic;
  int32_t nranks;
  std::atomic<int32_t> joined;
  std::atomic<int32_t> aborted;
};
struct AgState {
  std::atomic<uint64_t> seq[kAgSlots];  // per rank: op index + 1 deposited in slot
  std::atomic<uint64_t> done;           // per rank: all-gathers completed
};
struct Channel {                         // one ordered pair src -> dst
  std::atomic<uint64_t> sent;            // chunks deposited
  std::atomic<uint64_t> taken;           // chunks consumed
};

size_t align(size_t x) { return (x + 63) & ~size_t(63); }

struct Layout {
  size_t ag_state, ag_data, channels, ch_data, total;
  explicit Layout(int n) {
    ag_state = align(sizeof(Header));
    ag_data = align(ag_state + sizeof(AgState) * n);
    channels = align(ag_data + kAgSlots * kAgBytes * n);
    ch_data = align(channels + sizeof(Channel) * n * n);
    total = ch_data + kChSlots * kChunk * n * n;
  }
};

struct Op {  // one send or receive of a group, progressed chunk by chunk
  bool send;
  char* dev;
  size_t bytes;
  int peer;
  size_t chunk = 0, nchunks = 0;
  int ordinal = 0;   // receives: 1, 2, ... in issue order (fault injection)
};

// Fault injection (tests only): SHMCOMM_CORRUPT_RECV=k overwrites bytes
// 64..127 of the k-th receive of this process with 0xFF once its first chunk
// has landed -- a TILES stream's offset table, i.e. a receive whose content
// no longer matches its header (tests/test_gpu_driver.py).
int corrupt_recv_ordinal() {
  static const int k = [] {
    const char* e = std::getenv("SHMCOMM_CORRUPT_RECV");
    return e ? std::atoi(e) : 0;
  }();
  return k;
}
std::atomic<int> g_recv_ops{0};

}  // namespace

struct ncclComm {
  int rank = 0, nranks = 1;
  // non-blocking mode: creation and enqueueing state (ncclCommGetAsyncError)
  std::atomic<int> init{ncclSuccess};     // ncclInProgress while joining
  std::atomic<int> enqueueing{0};         // calls returned ncclInProgress, not yet enqueued
  std::atomic<bool> abort_req{false};
  std::thread joiner;
  std::string name;
  char* base = nullptr;
  size_t size = 0;
  Layout* L = nullptr;
  uint64_t ag_ops = 0;
  std::vector<uint64_t> sent, taken;  // my view: chunks I sent to / took from each peer
  hipStream_t copy = nullptr;
  std::atomic<int> async{ncclSuccess};
  long timeout_ms = 60000;

  Header* hdr() { return reinterpret_cast<Header*>(base); }
  AgState* ag(int r) { return reinterpret_cast<AgState*>(base + L->ag_state) + r; }
  char* ag_buf(int slot, int r) { return base + L->ag_data + (size_t(slot) * nranks + r) * kAgBytes; }
  Channel* ch(int src, int dst) {
    return reinterpret_cast<Channel*>(base + L->channels) + (size_t(src) * nranks + dst);
  }
  char* ch_buf(int src, int dst, uint64_t k) {
    return base + L->ch_data + ((size_t(src) * nranks + dst) * kChSlots + k % kChSlots) * kChunk;
  }
};

namespace {

thread_local int g_group_depth = 0;

using Clock = std::chrono::steady_clock;

template <class Pred>
bool wait_for(ncclComm* c, Pred ready) {
  if (ready()) return true;
  const auto t0 = Clock::now();
  for (unsigned n = 0;; ++n) {
    if (ready()) return true;
    if ((n & 255) == 255) {
      if (c->abort_req.load() || (c->base && c->hdr()->aborted.load())) break;
      if (std::chrono::duration_cast<std::chrono::milliseconds>(Clock::now() - t0).count() >
          c->timeout_ms)
        break;
    }
    sched_yield();
  }
  c->async.store(ncclSystemError);
  return false;
}

// ONE copy stream per process, shared by all communicators (only the engine
// thread, or in synchronous mode the calling thread, uses it): the fewer
// streams a rank holds, the fewer hardware queues it needs
hipStream_t copy_stream() {
  static std::mutex mu;
  static hipStream_t s = nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (!s) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  return s;
}

bool copy(ncclComm* c, void* dst, const void* src, size_t n, hipMemcpyKind kind) {
  if (n == 0) return true;
  if (hipMemcpyAsync(dst, src, n, kind, c->copy) != hipSuccess) {
    c->async.store(ncclUnhandledCudaError);
    return false;
  }
  // polled with the limit: a copy stream that shares a hardware queue with a
  // stream held by a wait-value packet would otherwise block forever
  const auto t0 = Clock::now();
  for (unsigned k = 0;; ++k) {
    const hipError_t q = hipStreamQuery(c->copy);
    if (q == hipSuccess) return true;
    if (q != hipErrorNotReady ||
        std::chrono::duration_cast<std::chrono::milliseconds>(Clock::now() - t0).count() >
            c->timeout_ms) {
      c->async.store(ncclUnhandledCudaError);
      return false;
    }
    if ((k & 63) == 63) sched_yield();
  }
}

size_t dtype_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 1;
  }
}

// Progress one op by as many chunks as are possible without waiting; true
// when it made progress.
bool progress(ncclComm* c, Op& op) {
  bool moved = false;
  while (op.chunk < op.nchunks) {
    const size_t off = op.chunk * kChunk;
    const size_t n = std::min(kChunk, op.bytes - off);
    if (op.send) {
      Channel* ch = c->ch(c->rank, op.peer);
      const uint64_t k = c->sent[op.peer];
      if (k >= kChSlots && ch->taken.load(std::memory_order_acquire) < k - kChSlots + 1) break;
      if (!copy(c, c->ch_buf(c->rank, op.peer, k), op.dev + off, n, hipMemcpyDeviceToHost))
        return false;
      c->sent[op.peer] = k + 1;
      ch->sent.store(k + 1, std::memory_order_release);
    } else {
      Channel* ch = c->ch(op.peer, c->rank);
      const uint64_t k = c->taken[op.peer];
      if (ch->sent.load(std::memory_order_acquire) < k + 1) break;
      if (!copy(c, op.dev + off, c->ch_buf(op.peer, c->rank, k), n, hipMemcpyHostToDevice))
        return false;
      if (op.chunk == 0 && n >= 128 && op.ordinal == corrupt_recv_ordinal()) {
        static const unsigned char ff[64] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                             0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                             0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                             0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                             0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                             0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                             0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                                             0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF};
        if (!copy(c, op.dev + 64, ff, sizeof(ff), hipMemcpyHostToDevice)) return false;
      }
      c->taken[op.peer] = k + 1;
      ch->taken.store(k + 1, std::memory_order_release);
    }
    ++op.chunk;
    moved = true;
  }
  return moved;
}

// Several ops of a group between the same pair of ranks in the same
// direction share one channel, so they are matched in issue order (as RCCL
// matches point-to-point calls): an op moves only after every earlier op of
// its channel has finished.  (Progressing them independently let a later
// receive take a chunk an earlier one had just missed -- a data race that
// batched ships, several frames per peer in one group, turned into a decode
// of a mixed-up stream.)
ncclResult_t run_ops(ncclComm* c, std::vector<Op>& ops) {
  for (Op& op : ops) op.nchunks = (op.bytes + kChunk - 1) / kChunk;
  bool all = false;
  std::vector<char> busy(2 * size_t(c->nranks));   // (peer, direction) has an unfinished earlier op
  auto finished = [&] {
    all = true;
    std::fill(busy.begin(), busy.end(), 0);
    for (Op& op : ops) {
      if (op.chunk == op.nchunks) continue;
      char& b = busy[2 * size_t(op.peer) + (op.send ? 1 : 0)];
      if (!b) progress(c, op);
      if (c->async.load() != ncclSuccess) return true;
      if (op.chunk != op.nchunks) {
        b = 1;
        all = false;
      }
    }
    return all;
  };
  if (!wait_for(c, finished) || c->async.load() != ncclSuccess) return ncclSystemError;
  return ncclSuccess;
}

// ---- the progress engine (one per process) ---------------------------------
constexpr uint32_t kFlags = 4096;   // completion flags, slot seq % kFlags

struct Task {
  std::vector<hipEvent_t> ready;   // the callers' streams up to the call
  std::function<ncclResult_t()> run;
  std::vector<ncclComm*> comms;
  uint32_t seq = 0;
};

struct Engine {
  std::mutex mu;
  std::condition_variable cv, idle;
  std::deque<Task> q;
  bool busy = false;
  int dev = 0;
  uint32_t* flags = nullptr;   // coherent pinned host memory
  uint32_t seq = 0;
  long timeout_ms = 60000;
};

Engine* g_engine = nullptr;   // never destroyed: its thread may outlive main's locals
int g_engine_state = 0;       // 1 engine, -1 SHMCOMM_SYNC, -2 no wait-value support, -3 setup
std::mutex g_engine_mu;

bool async_mode() {
  const char* e = std::getenv("SHMCOMM_SYNC");
  return !(e && *e && *e != '0');
}

void engine_loop(Engine* E) {
  (void)hipSetDevice(E->dev);
  for (;;) {
    Task t;
    {
      std::unique_lock<std::mutex> lock(E->mu);
      E->cv.wait(lock, [&] { return !E->q.empty(); });
      t = std::move(E->q.front());
      E->q.pop_front();
      E->busy = true;
    }
    // the work the call is ordered after, with the communicators' limit
    bool ok = true;
    const auto t0 = Clock::now();
    for (hipEvent_t ev : t.ready) {
      for (unsigned n = 0;; ++n) {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady ||
            std::chrono::duration_cast<std::chrono::milliseconds>(Clock::now() - t0).count() >
                E->timeout_ms) {
          ok = false;
          break;
        }
        if ((n & 63) == 63) sched_yield();
      }
      (void)hipEventDestroy(ev);
    }
    const ncclResult_t rc = ok ? t.run() : ncclSystemError;
    if (rc != ncclSuccess)
      for (ncclComm* c : t.comms) {
        int expect = ncclSuccess;
        c->async.compare_exchange_strong(expect, rc == ncclInProgress ? ncclSystemError : rc);
      }
    // release the callers' streams whatever happened (no stream left waiting):
    // a host store to the coherent flag the GPU's wait packet polls, so the
    // release needs no queue of its own
    __atomic_store_n(E->flags + t.seq % kFlags, t.seq, __ATOMIC_RELEASE);
    {
      std::lock_guard<std::mutex> lock(E->mu);
      E->busy = false;
      if (E->q.empty()) E->idle.notify_all();
    }
  }
}

// The process's engine, created on the calling thread's device; null when
// the device cannot wait on a value (then calls run synchronously).
Engine* engine(long timeout_ms) {
  if (!async_mode()) {
    g_engine_state = -1;
    return nullptr;
  }
  std::lock_guard<std::mutex> lock(g_engine_mu);
  if (g_engine) return g_engine;
  int dev = 0, can = 0;
  const bool dbg = std::getenv("SHMCOMM_DEBUG") != nullptr;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, dev) != hipSuccess ||
      !can) {
    if (dbg) std::fprintf(stderr, "shmcomm: no stream wait-value support (%d): synchronous\n", can);
    g_engine_state = -2;
    return nullptr;
  }
  auto* E = new Engine;
  E->dev = dev;
  E->timeout_ms = timeout_ms;
  // coherent pinned host memory: the GPU's wait-value and write-value packets
  // both work on it (hipMallocSignalMemory takes single 8-byte signals only)
  if (hipHostMalloc(reinterpret_cast<void**>(&E->flags), kFlags * sizeof(uint32_t),
                    hipHostMallocCoherent) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess) {
    if (dbg) std::fprintf(stderr, "shmcomm: engine setup failed: synchronous\n");
    g_engine_state = -3;
    delete E;
    return nullptr;
  }
  std::memset(E->flags, 0, kFlags * sizeof(uint32_t));
  std::thread(engine_loop, E).detach();
  g_engine = E;
  g_engine_state = 1;
  return E;
}

// Enqueue `run` after the work already on `streams`; the streams wait (on the
// GPU) for its completion.  Without an engine: wait for the streams, run now.
ncclResult_t submit(std::vector<hipStream_t> streams, std::vector<ncclComm*> comms,
                    std::function<ncclResult_t()> run) {
  Engine* E = engine(comms.empty() ? 60000 : comms[0]->timeout_ms);
  if (!E) {
    for (hipStream_t s : streams)
      if (hipStreamSynchronize(s) != hipSuccess) return ncclUnhandledCudaError;
    return run();
  }
  Task t;
  t.run = std::move(run);
  t.comms = std::move(comms);
  for (hipStream_t s : streams) {
    hipEvent_t ev;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(ev, s) != hipSuccess)
      return ncclUnhandledCudaError;
    t.ready.push_back(ev);
  }
  std::lock_guard<std::mutex> lock(E->mu);
  t.seq = ++E->seq;
  for (hipStream_t s : streams)
    if (hipStreamWaitValue32(s, E->flags + t.seq % kFlags, t.seq, hipStreamWaitValueGte) !=
        hipSuccess)
      return ncclUnhandledCudaError;
  E->q.push_back(std::move(t));
  E->cv.notify_one();
  return ncclSuccess;
}

// Wait until the engine has run every call enqueued so far (communicator
// teardown: nothing of it may still be in use).
void engine_drain(long timeout_ms) {
  Engine* E = g_engine;
  if (!E) return;
  std::unique_lock<std::mutex> lock(E->mu);
  E->idle.wait_for(lock, std::chrono::milliseconds(timeout_ms + 1000),
                   [&] { return E->q.empty() && !E->busy; });
}

// ---- non-blocking mode (SHMCOMM_NONBLOCKING=1) -----------------------------
bool nonblocking_mode() {
  const char* e = std::getenv("SHMCOMM_NONBLOCKING");
  return e && *e && *e != '0';
}
std::atomic<unsigned long long> g_inprogress{0}, g_aborts{0};

// One thread enqueues deferred calls in issue order, each a little later
// (the window in which an unsettled caller would misorder its stream work).
struct Deferred {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::function<void()>> q;
};
Deferred* deferred() {
  static Deferred* D = [] {
    auto* d = new Deferred;
    std::thread([d] {
      for (;;) {
        std::function<void()> f;
        {
          std::unique_lock<std::mutex> lock(d->mu);
          d->cv.wait(lock, [&] { return !d->q.empty(); });
          f = std::move(d->q.front());
          d->q.pop_front();
        }
        std::this_thread::sleep_for(std::chrono::microseconds(300));
        f();
      }
    }).detach();
    return d;
  }();
  return D;
}

// Run `enq` (which enqueues a call and returns its result) now, or -- in
// non-blocking mode -- later on the deferred thread, answering ncclInProgress
// until it has run (a failure then becomes the communicators' async error).
ncclResult_t maybe_defer(const std::vector<ncclComm*>& comms, std::function<ncclResult_t()> enq) {
  if (!nonblocking_mode()) return enq();
  for (ncclComm* c : comms) c->enqueueing.fetch_add(1);
  g_inprogress.fetch_add(1);
  Deferred* D = deferred();
  std::lock_guard<std::mutex> lock(D->mu);
  D->q.push_back([comms, enq = std::move(enq)] {
    const ncclResult_t rc = enq();
    for (ncclComm* c : comms) {
      if (rc != ncclSuccess) {
        int expect = ncclSuccess;
        c->async.compare_exchange_strong(expect, rc);
      }
      c->enqueueing.fetch_sub(1);
    }
  });
  D->cv.notify_one();
  return ncclInProgress;
}

struct StatsAtExit {
  ~StatsAtExit() {
    if (std::getenv("SHMCOMM_STATS"))
      std::fprintf(stderr, "shmcomm: inprogress_returns=%llu aborts=%llu\n",
                   (unsigned long long)g_inprogress.load(), (unsigned long long)g_aborts.load());
  }
} g_stats_at_exit;

struct GroupEntry {
  ncclComm* comm;
  std::vector<Op> ops;
  std::vector<hipStream_t> streams;
};
thread_local std::vector<GroupEntry> g_pending;

ncclResult_t enqueue(ncclComm* c, Op op, hipStream_t stream) {
  if (!c || c->async.load() != ncclSuccess) return ncclInvalidUsage;
  if (op.peer < 0 || op.peer >= c->nranks) return ncclInvalidArgument;
  if (g_group_depth > 0) {
    for (auto& g : g_pending)
      if (g.comm == c) {
        g.ops.push_back(op);
        bool have = false;
        for (hipStream_t s : g.streams) have = have || s == stream;
        if (!have) g.streams.push_back(stream);
        return ncclSuccess;
      }
    g_pending.push_back({c, {op}, {stream}});
    return ncclSuccess;
  }
  return submit({stream}, {c}, [c, op]() mutable {
    std::vector<Op> ops{op};
    return run_ops(c, ops);
  });
}

}  // namespace

extern "C" {

// 1 when calls run on the asynchronous engine, 0 when synchronously (tests)
int shmcomm_async_engine(void) { return g_engine_state; }
// tests: 0 ncclInProgress answers, 1 ncclCommAbort calls (this process)
unsigned long long shmcomm_counts(int which) {
  return which == 0 ? g_inprogress.load() : g_aborts.load();
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  if (!id) return ncclInvalidArgument;
  std::memset(id, 0, sizeof(*id));
  std::random_device rd;
  std::snprintf(id->internal, sizeof(id->internal), "/sdf3d_shmcomm_%d_%08x%08x", (int)getpid(),
                rd(), rd());
  return ncclSuccess;
}

namespace {
// Map the segment and wait until all ranks have joined; the communicator's
// `init` state becomes ncclSuccess or an error.  (Blocking creation runs it
// on the caller's thread, non-blocking creation on c->joiner.)
ncclResult_t join(ncclComm* c, int dev) {
  (void)hipSetDevice(dev);
  int fd = shm_open(c->name.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0 || ftruncate(fd, (off_t)c->size) != 0) {
    if (fd >= 0) close(fd);
    return ncclSystemError;
  }
  void* p = mmap(nullptr, c->size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return ncclSystemError;
  c->base = static_cast<char*>(p);
  // a new segment is zero-filled; the first rank to see no magic sets it
  uint64_t expect = 0;
  reinterpret_cast<std::atomic<uint64_t>*>(&c->hdr()->magic)
      ->compare_exchange_strong(expect, kMagic);
  c->hdr()->nranks = c->nranks;
  c->copy = copy_stream();
  // created now (its setup synchronises the device); SHMCOMM_REQUIRE_ASYNC=1
  // makes a missing engine an error, so a test cannot pass synchronously
  if (!engine(c->timeout_ms) && std::getenv("SHMCOMM_REQUIRE_ASYNC")) return ncclSystemError;
  c->hdr()->joined.fetch_add(1);
  if (!wait_for(c, [&] { return c->hdr()->joined.load() >= c->nranks; }))
    return ncclSystemError;
  if (c->rank == 0) shm_unlink(c->name.c_str());  // every rank has it mapped
  return ncclSuccess;
}

ncclComm* new_comm(int nranks, const ncclUniqueId& id, int rank) {
  auto* c = new ncclComm();
  c->rank = rank;
  c->nranks = nranks;
  c->name.assign(id.internal, strnlen(id.internal, sizeof(id.internal)));
  if (const char* t = std::getenv("SHMCOMM_TIMEOUT_MS")) c->timeout_ms = std::atol(t);
  c->L = new Layout(nranks);
  c->size = c->L->total;
  c->sent.assign(nranks, 0);
  c->taken.assign(nranks, 0);
  return c;
}

void free_comm(ncclComm* c) {
  if (c->joiner.joinable()) c->joiner.join();
  if (c->base) munmap(c->base, c->size);
  delete c->L;
  delete c;
}
}  // namespace

ncclResult_t ncclCommInitRank(ncclComm_t* out, int nranks, ncclUniqueId id, int rank) {
  if (!out || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  *out = nullptr;
  ncclComm* c = new_comm(nranks, id, rank);
  int dev = 0;
  (void)hipGetDevice(&dev);
  const ncclResult_t rc = join(c, dev);
  if (rc != ncclSuccess) {
    free_comm(c);
    return rc;
  }
  *out = c;
  return ncclSuccess;
}

// The driver creates communicators through this entry point when it exists,
// non-blocking (config->blocking = 0), and polls ncclCommGetAsyncError.  By
// default creation completes before returning, so the state it polls is
// ncclSuccess at once; with SHMCOMM_NONBLOCKING=1 the join runs on a helper
// thread and the call answers ncclInProgress, as RCCL does.
ncclResult_t ncclCommInitRankConfig(ncclComm_t* out, int nranks, ncclUniqueId id, int rank,
                                    ncclConfig_t* config) {
  if (!(nonblocking_mode() && config && config->blocking == 0))
    return ncclCommInitRank(out, nranks, id, rank);
  if (!out || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  ncclComm* c = new_comm(nranks, id, rank);
  int dev = 0;
  (void)hipGetDevice(&dev);
  c->init.store(ncclInProgress);
  c->joiner = std::thread([c, dev] { c->init.store(join(c, dev)); });
  *out = c;
  g_inprogress.fetch_add(1);
  return ncclInProgress;
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
  if (!c) return ncclSuccess;
  if (c->joiner.joinable()) {   // a non-blocking creation still joining: stop it
    c->abort_req.store(true);
    c->joiner.join();
  }
  if (c->init.load() == ncclSuccess) engine_drain(c->timeout_ms);   // no call of it still running
  // (the copy stream is the process's, shared by its communicators)
  free_comm(c);
  return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t c) {
  if (!c) return ncclSuccess;
  g_aborts.fetch_add(1);
  c->abort_req.store(true);
  if (c->joiner.joinable()) c->joiner.join();
  if (c->base) c->hdr()->aborted.store(1);   // peers' waits end with an error
  if (c->init.load() != ncclSuccess) shm_unlink(c->name.c_str());   // nobody else will
  return ncclCommDestroy(c);
}

// Non-blocking mode: flushes the communicator's calls (engine drain) on the
// deferred thread, answering ncclInProgress meanwhile.
ncclResult_t ncclCommFinalize(ncclComm_t c) {
  if (!c) return ncclInvalidArgument;
  if (!nonblocking_mode()) return ncclSuccess;
  const long t = c->timeout_ms;
  return maybe_defer({c}, [t] {
    engine_drain(t);
    return ncclSuccess;
  });
}

ncclResult_t ncclCommGetAsyncError(ncclComm_t c, ncclResult_t* e) {
  if (!c || !e) return ncclInvalidArgument;
  const int init = c->init.load();
  if (init != ncclSuccess) {
    *e = (ncclResult_t)init;
    return ncclSuccess;
  }
  if (c->hdr()->aborted.load()) *e = ncclRemoteError;
  else if (c->async.load() != ncclSuccess) *e = (ncclResult_t)c->async.load();
  else *e = c->enqueueing.load() > 0 ? ncclInProgress : ncclSuccess;
  return ncclSuccess;
}

ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t count,
                           ncclDataType_t datatype, ncclComm_t c, hipStream_t stream) {
  if (!c || c->async.load() != ncclSuccess) return ncclInvalidUsage;
  const size_t bytes = count * dtype_size(datatype);
  if (bytes > kAgBytes) return ncclInvalidArgument;
  const uint64_t k = c->ag_ops++;   // issue order = the engine's order
  return maybe_defer({c}, [=] { return submit({stream}, {c}, [c, k, bytes, sendbuff, recvbuff]() -> ncclResult_t {
    const int slot = int(k % kAgSlots);
    // the slot is free once every rank has finished all-gather k - kAgSlots
    if (!wait_for(c, [&] {
          for (int r = 0; r < c->nranks; ++r)
            if (k >= kAgSlots && c->ag(r)->done.load(std::memory_order_acquire) < k - kAgSlots + 1)
              return false;
          return true;
        }))
      return ncclSystemError;
    if (!copy(c, c->ag_buf(slot, c->rank), sendbuff, bytes, hipMemcpyDeviceToHost))
      return ncclUnhandledCudaError;
    c->ag(c->rank)->seq[slot].store(k + 1, std::memory_order_release);
    for (int r = 0; r < c->nranks; ++r) {
      if (!wait_for(c, [&] { return c->ag(r)->seq[slot].load(std::memory_order_acquire) == k + 1; }))
        return ncclSystemError;
      if (!copy(c, static_cast<char*>(recvbuff) + r * bytes, c->ag_buf(slot, r), bytes,
                hipMemcpyHostToDevice))
        return ncclUnhandledCudaError;
    }
    c->ag(c->rank)->done.store(k + 1, std::memory_order_release);
    return ncclSuccess;
  }); });
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer,
                      ncclComm_t c, hipStream_t stream) {
  Op op{true, static_cast<char*>(const_cast<void*>(sendbuff)), count * dtype_size(datatype), peer};
  return enqueue(c, op, stream);
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer,
                      ncclComm_t c, hipStream_t stream) {
  Op op{false, static_cast<char*>(recvbuff), count * dtype_size(datatype), peer};
  op.ordinal = ++g_recv_ops;
  return enqueue(c, op, stream);
}

ncclResult_t ncclGroupStart() {
  ++g_group_depth;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (g_group_depth <= 0) return ncclInvalidUsage;
  if (--g_group_depth > 0) return ncclSuccess;
  auto groups = std::move(g_pending);
  g_pending.clear();
  if (groups.empty()) return ncclSuccess;
  // one call for the whole group: every stream in it waits for all of it
  std::vector<hipStream_t> streams;
  std::vector<ncclComm*> comms;
  for (auto& g : groups) {
    comms.push_back(g.comm);
    for (hipStream_t s : g.streams) {
      bool have = false;
      for (hipStream_t t : streams) have = have || t == s;
      if (!have) streams.push_back(s);
    }
  }
  auto shared = std::make_shared<std::vector<GroupEntry>>(std::move(groups));
  return maybe_defer(comms, [=] {
    return submit(streams, comms, [shared]() {
      ncclResult_t rc = ncclSuccess;
      for (auto& g : *shared) {
        const ncclResult_t r = run_ops(g.comm, g.ops);
        if (rc == ncclSuccess) rc = r;
      }
      return rc;
    });
  });
}

}  // extern "C"

// shmcomm.cpp -- TEST INFRASTRUCTURE ONLY: a stand-in for the RCCL symbols the
// native frame driver loads at run time (sdf3d_amd/csrc/driver.cpp load_rccl:
// ncclGetUniqueId, ncclCommInitRank(Config), ncclCommDestroy, ncclCommAbort,
// ncclCommGetAsyncError, ncclAllGather, ncclSend, ncclRecv, ncclGroupStart,
// ncclGroupEnd), so that the driver's multi-rank sequence can run with
// several ranks on ONE GPU, which RCCL refuses ("Duplicate GPU detected").
//
// Every rank is a process; a communicator is one POSIX shared-memory segment
// named by the unique id.  Data moves through host memory:
//   * a call first waits for the work already enqueued on its stream
//     (hipStreamSynchronize), as the collective would be ordered after it,
//   * then copies device -> shared memory -> device on a private stream and
//     returns with the data in place, so later work on the stream sees it.
// So every call completes on the host before it returns (stricter than
// RCCL's asynchronous enqueue, never weaker): a dependency the driver forgets
// on ANOTHER stream (a render on rs[b] not waited for before a send on ds)
// still shows as a wrong frame.  Sends and receives inside a group are
// progressed together, chunk by chunk, so any pattern (rank 0 receiving from
// 7 peers, a rank sending to itself) completes.  Every wait polls with a
// limit (SHMCOMM_TIMEOUT_MS, default 60 s) and then sets the communicator's
// asynchronous error, as a failed RCCL would.  Never linked into the product
// library; tests load it through the driver's rccl_path.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types and signatures only
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
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
};

}  // namespace

struct ncclComm {
  int rank = 0, nranks = 1;
  std::string name;
  char* base = nullptr;
  size_t size = 0;
  Layout* L = nullptr;
  uint64_t ag_ops = 0;
  std::vector<uint64_t> sent, taken;  // my view: chunks I sent to / took from each peer
  hipStream_t copy = nullptr;
  ncclResult_t async = ncclSuccess;
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
thread_local std::vector<std::pair<ncclComm*, std::vector<Op>>> g_group;

using Clock = std::chrono::steady_clock;

template <class Pred>
bool wait_for(ncclComm* c, Pred ready) {
  if (ready()) return true;
  const auto t0 = Clock::now();
  for (unsigned n = 0;; ++n) {
    if (ready()) return true;
    if ((n & 255) == 255) {
      if (c->hdr()->aborted.load()) break;
      if (std::chrono::duration_cast<std::chrono::milliseconds>(Clock::now() - t0).count() >
          c->timeout_ms)
        break;
    }
    sched_yield();
  }
  c->async = ncclSystemError;
  return false;
}

bool copy(ncclComm* c, void* dst, const void* src, size_t n, hipMemcpyKind kind) {
  if (n == 0) return true;
  if (hipMemcpyAsync(dst, src, n, kind, c->copy) != hipSuccess ||
      hipStreamSynchronize(c->copy) != hipSuccess) {
    c->async = ncclUnhandledCudaError;
    return false;
  }
  return true;
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
      c->taken[op.peer] = k + 1;
      ch->taken.store(k + 1, std::memory_order_release);
    }
    ++op.chunk;
    moved = true;
  }
  return moved;
}

ncclResult_t run_ops(ncclComm* c, std::vector<Op>& ops) {
  for (Op& op : ops) op.nchunks = (op.bytes + kChunk - 1) / kChunk;
  bool all = false;
  auto finished = [&] {
    all = true;
    for (Op& op : ops) {
      progress(c, op);
      if (c->async != ncclSuccess) return true;
      all = all && op.chunk == op.nchunks;
    }
    return all;
  };
  if (!wait_for(c, finished) || c->async != ncclSuccess) return ncclSystemError;
  return ncclSuccess;
}

ncclResult_t enqueue(ncclComm* c, Op op, hipStream_t stream) {
  if (!c || c->async != ncclSuccess) return ncclInvalidUsage;
  if (op.peer < 0 || op.peer >= c->nranks) return ncclInvalidArgument;
  // ordered after the work already on `stream`
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
  if (g_group_depth > 0) {
    for (auto& g : g_group)
      if (g.first == c) {
        g.second.push_back(op);
        return ncclSuccess;
      }
    g_group.push_back({c, {op}});
    return ncclSuccess;
  }
  std::vector<Op> ops{op};
  return run_ops(c, ops);
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  if (!id) return ncclInvalidArgument;
  std::memset(id, 0, sizeof(*id));
  std::random_device rd;
  std::snprintf(id->internal, sizeof(id->internal), "/sdf3d_shmcomm_%d_%08x%08x", (int)getpid(),
                rd(), rd());
  return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* out, int nranks, ncclUniqueId id, int rank) {
  if (!out || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
  *out = nullptr;
  auto* c = new ncclComm();
  c->rank = rank;
  c->nranks = nranks;
  c->name.assign(id.internal, strnlen(id.internal, sizeof(id.internal)));
  if (const char* t = std::getenv("SHMCOMM_TIMEOUT_MS")) c->timeout_ms = std::atol(t);
  c->L = new Layout(nranks);
  c->size = c->L->total;
  int fd = shm_open(c->name.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0 || ftruncate(fd, (off_t)c->size) != 0) {
    if (fd >= 0) close(fd);
    delete c->L;
    delete c;
    return ncclSystemError;
  }
  void* p = mmap(nullptr, c->size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    delete c->L;
    delete c;
    return ncclSystemError;
  }
  c->base = static_cast<char*>(p);
  // a new segment is zero-filled; the first rank to see no magic sets it
  uint64_t expect = 0;
  reinterpret_cast<std::atomic<uint64_t>*>(&c->hdr()->magic)
      ->compare_exchange_strong(expect, kMagic);
  c->hdr()->nranks = nranks;
  c->sent.assign(nranks, 0);
  c->taken.assign(nranks, 0);
  (void)hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking);
  c->hdr()->joined.fetch_add(1);
  if (!wait_for(c, [&] { return c->hdr()->joined.load() >= nranks; })) {
    munmap(c->base, c->size);
    delete c->L;
    delete c;
    return ncclSystemError;
  }
  if (rank == 0) shm_unlink(c->name.c_str());  // every rank has it mapped
  *out = c;
  return ncclSuccess;
}

// The driver creates communicators through this entry point when it exists
// (non-blocking, polled with ncclCommGetAsyncError): here creation completes
// before returning, so the state it polls is ncclSuccess at once.
ncclResult_t ncclCommInitRankConfig(ncclComm_t* out, int nranks, ncclUniqueId id, int rank,
                                    ncclConfig_t*) {
  return ncclCommInitRank(out, nranks, id, rank);
}

ncclResult_t ncclCommDestroy(ncclComm_t c) {
  if (!c) return ncclSuccess;
  if (c->copy) (void)hipStreamDestroy(c->copy);
  munmap(c->base, c->size);
  delete c->L;
  delete c;
  return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t c) {
  if (!c) return ncclSuccess;
  c->hdr()->aborted.store(1);  // peers' waits end with an error
  return ncclCommDestroy(c);
}

ncclResult_t ncclCommGetAsyncError(ncclComm_t c, ncclResult_t* e) {
  if (!c || !e) return ncclInvalidArgument;
  *e = c->hdr()->aborted.load() ? ncclRemoteError : c->async;
  return ncclSuccess;
}

ncclResult_t ncclAllGather(const void* sendbuff, void* recvbuff, size_t count,
                           ncclDataType_t datatype, ncclComm_t c, hipStream_t stream) {
  if (!c || c->async != ncclSuccess) return ncclInvalidUsage;
  const size_t bytes = count * dtype_size(datatype);
  if (bytes > kAgBytes) return ncclInvalidArgument;
  if (hipStreamSynchronize(stream) != hipSuccess) return ncclUnhandledCudaError;
  const uint64_t k = c->ag_ops++;
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
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer,
                      ncclComm_t c, hipStream_t stream) {
  Op op{true, static_cast<char*>(const_cast<void*>(sendbuff)), count * dtype_size(datatype), peer};
  return enqueue(c, op, stream);
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer,
                      ncclComm_t c, hipStream_t stream) {
  Op op{false, static_cast<char*>(recvbuff), count * dtype_size(datatype), peer};
  return enqueue(c, op, stream);
}

ncclResult_t ncclGroupStart() {
  ++g_group_depth;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  if (g_group_depth <= 0) return ncclInvalidUsage;
  if (--g_group_depth > 0) return ncclSuccess;
  ncclResult_t rc = ncclSuccess;
  auto groups = std::move(g_group);
  g_group.clear();
  for (auto& g : groups) {
    const ncclResult_t r = run_ops(g.first, g.second);
    if (rc == ncclSuccess) rc = r;
  }
  return rc;
}

}  // extern "C"

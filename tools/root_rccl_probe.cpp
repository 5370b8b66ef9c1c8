// root_rccl_probe.cpp -- rank 0's frame loop at N ranks on ONE MI355X, with
// the streams moved by REAL RCCL (the N = 8 bound measured
// with the transfer load, not only the decode of cache-warm buffers).
//
// The N - 1 peers' TILES streams of `nsets` distinct frames (different
// cameras) are rendered up front; then every frame i, exactly as the frame
// driver's rank 0 (sdf3d_amd/csrc/driver.cpp) does it:
//   rs[b]  render rank 0's own rows in place into frame[b]
//   batch of `batch` frames complete:
//     ss   RCCL all-gather of the batch's lengths (world 1: the real call)
//     ds   RCCL group: rank 0 sends set (i mod nsets)'s N - 1 streams to
//          itself and receives them into gathered[b] (fresh receive buffers,
//          a set the previous frames did not read) -- the bytes and the
//          receives of an N-rank ship, over RCCL's own path
//     rs[b] wait for the group, decode gathered[b] into frame[b]
//          (sdf_tiles_decode_checked: the length check and status words
//          of the product decode)
// It reports the frame period (wall time of K frames, the GPU busy with
// renders, RCCL kernels and decodes) and the host microseconds per frame of
// these calls (sdf_render builds its plan per call: a few microseconds more
// than the driver's prepared plans), and checks the last frame against a
// one-device render bit for bit.  TEST / MEASUREMENT TOOL: not product code.
//
//   tools/root_rccl_probe.bin frame.bin librccl.so frames warmup batch [nbuf [mode]]
// (frame.bin from tools/root_rccl_probe.py: the C4 frame's structs, the
// set cameras, world and shares).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/sdf_abi.h"
#include "../sdf3d_amd/csrc/kernel_args.h"

namespace {

// recvcopy's receive: ONE kernel per batch moves every stream of it (as an
// RCCL group of receives is one kernel), 16 bytes per lane, grid-stride
struct CopyList {
  const uint4* src[32];
  uint4* dst[32];
  unsigned long long n16[32];   // 16-byte units (streams rounded up: parts are 256-B pitched)
  int count;
};
__global__ void copy_streams(CopyList L) {
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (int j = 0; j < L.count; ++j)
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
         i < L.n16[j]; i += stride)
      L.dst[j][i] = L.src[j][i];
}

struct Api {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*);
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*CommDestroy)(ncclComm_t);
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*GroupStart)();
  ncclResult_t (*GroupEnd)();
};

void die(const char* what, int rc) {
  std::fprintf(stderr, "root_rccl_probe: %s failed (%d)\n", what, rc);
  std::exit(2);
}
void hip(hipError_t e, const char* what) {
  if (e != hipSuccess) die(what, (int)e);
}
void ok(int rc, const char* what) {
  if (rc != SDF_OK) die(what, rc);
}
void nccl(ncclResult_t rc, const char* what) {
  if (rc != ncclSuccess) die(what, (int)rc);
}

using Clock = std::chrono::steady_clock;
double since(Clock::time_point t) { return std::chrono::duration<double>(Clock::now() - t).count(); }

}  // namespace

int main(int argc, char** argv) {
  if (argc < 6) {
    std::fprintf(stderr, "usage: %s frame.bin librccl.so frames warmup batch [nbuf]\n", argv[0]);
    return 2;
  }
  const int K = std::atoi(argv[3]), WARM = std::atoi(argv[4]), B = std::atoi(argv[5]);
  const int NB = argc > 6 ? std::atoi(argv[6]) : 4;
  // what runs per frame: full (render + RCCL + decode), norccl (the decode
  // reads the set's streams where they were rendered: no transfer), rccl
  // (the transfers only), decode (the decode only, from the rotated sets),
  // render (rank 0's rows only), recvcopy (round 6, VERDICT r05 #3: the
  // RECEIVING side only -- render + decode, with the N - 1 streams of every
  // frame arriving in fresh receive buffers by hipMemcpyAsync on the data
  // stream, one device-to-device copy per stream, as rank 0's memory sees
  // the peers' writes over xGMI; no RCCL send on this GPU), recvkernel (the
  // same bytes moved by ONE copy kernel per batch, as an RCCL group of
  // receives is one kernel)
  const std::string mode = argc > 7 ? argv[7] : "full";
  const bool do_copy = mode == "recvcopy" || mode == "recvkernel";
  const bool one_kernel = mode == "recvkernel";
  const bool do_render = mode == "full" || mode == "norccl" || mode == "render" || do_copy;
  const bool do_rccl = mode == "full" || mode == "rccl";
  const bool do_decode = mode == "full" || mode == "norccl" || mode == "decode" || do_copy;
  if (K <= 0 || WARM < 0 || B < 1 || NB < B || NB % B) die("arguments", -1);
  // ---- the frame description ----
  sdf_scene scene;
  sdf_light light;
  sdf_material material;
  sdf_params params;
  int32_t hdr[4];   // world, share a, share b, nsets
  FILE* fp = std::fopen(argv[1], "rb");
  if (!fp || std::fread(&scene, sizeof scene, 1, fp) != 1 || std::fread(&light, sizeof light, 1, fp) != 1 ||
      std::fread(&material, sizeof material, 1, fp) != 1 ||
      std::fread(&params, sizeof params, 1, fp) != 1 || std::fread(hdr, sizeof hdr, 1, fp) != 1)
    die("reading frame.bin", -1);
  const int N = hdr[0], SA = hdr[1], SB = hdr[2], NS = hdr[3];
  if (N < 2 || N > SDF_MAX_DECODE_PARTS || NS < 1 || NS > 64) die("frame.bin header", -1);
  std::vector<sdf_camera> cams(NS);
  if (std::fread(cams.data(), sizeof(sdf_camera), NS, fp) != (size_t)NS) die("cameras", -1);
  std::fclose(fp);
  const int W = params.width, H = params.height;
  hip(hipSetDevice(0), "hipSetDevice");
  // ---- RCCL, one rank ----
  void* h = dlopen(argv[2], RTLD_NOW | RTLD_LOCAL);
  if (!h) die("dlopen librccl", -1);
  Api R;
  auto sym = [&](auto& fn, const char* name) {
    fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
    if (!fn) die(name, -1);
  };
  sym(R.GetUniqueId, "ncclGetUniqueId");
  sym(R.CommInitRank, "ncclCommInitRank");
  sym(R.CommDestroy, "ncclCommDestroy");
  sym(R.AllGather, "ncclAllGather");
  sym(R.Send, "ncclSend");
  sym(R.Recv, "ncclRecv");
  sym(R.GroupStart, "ncclGroupStart");
  sym(R.GroupEnd, "ncclGroupEnd");
  ncclUniqueId id;
  ncclComm_t data_comm, size_comm;
  nccl(R.GetUniqueId(&id), "ncclGetUniqueId");
  nccl(R.CommInitRank(&data_comm, 1, id, 0), "ncclCommInitRank");
  nccl(R.GetUniqueId(&id), "ncclGetUniqueId");
  nccl(R.CommInitRank(&size_comm, 1, id, 0), "ncclCommInitRank");
  // ---- tilings and the peers' streams of every set ----
  std::vector<sdf_tiling> til(N);
  std::vector<int> rows(N);
  std::vector<long long> data_off(N);
  long long pitch = 0;
  for (int r = 0; r < N; ++r) {
    ok(sdf_share_tiling(r, N, SA, SB, &til[r]), "sdf_share_tiling");
    rows[r] = sdf_owned_rows(H, &til[r]);
    const sdf::TilesLayout L(int64_t((W + 7) / 8) * ((rows[r] + 7) / 8));
    data_off[r] = (long long)L.data;
    pitch = std::max(pitch, (long long)((L.stream_end + 255) / 256 * 256));
  }
  sdf_params pt = params;
  pt.output_format = SDF_FORMAT_TILES;
  // set s: one buffer of N parts at `pitch` (part 0 empty: its zero header
  // says no stream), as a gathered buffer is laid out
  std::vector<void*> setbuf(NS);
  std::vector<std::vector<void*>> part(NS, std::vector<void*>(N, nullptr));
  std::vector<std::vector<int64_t>> used(NS, std::vector<int64_t>(N, -1));
  size_t set_bytes = 0;
  for (int s = 0; s < NS; ++s) {
    hip(hipMalloc(&setbuf[s], (size_t)pitch * N), "hipMalloc set");
    hip(hipMemset(setbuf[s], 0, (size_t)pitch * N), "hipMemset");
  }
  // a TILES render needs sdf_tiles_bytes (the stream's worst case plus the
  // encoder's scratch), more than a part's pitch: render into a scratch
  // buffer, then copy the stream itself into its part
  int64_t scratch_bytes = 0;
  for (int r = 1; r < N; ++r) scratch_bytes = std::max(scratch_bytes, sdf_tiles_bytes(W, rows[r]));
  void* scratch = nullptr;
  hip(hipMalloc(&scratch, (size_t)scratch_bytes), "hipMalloc scratch");
  for (int s = 0; s < NS; ++s)
    for (int r = 1; r < N; ++r) {
      part[s][r] = static_cast<char*>(setbuf[s]) + (size_t)r * pitch;
      ok(sdf_render(&scene, &cams[s], &light, &material, &pt, &til[r], scratch, nullptr, nullptr),
         "sdf_render peer");
      uint32_t u = 0;
      hip(hipMemcpy(&u, scratch, 4, hipMemcpyDeviceToHost), "read used");
      used[s][r] = u;
      if (data_off[r] + (long long)u > pitch) die("stream longer than its pitch", (int)u);
      hip(hipMemcpy(part[s][r], scratch, (size_t)(data_off[r] + u), hipMemcpyDeviceToDevice),
          "copy stream");
      set_bytes += (size_t)(data_off[r] + u);
    }
  hip(hipFree(scratch), "hipFree");
  // ---- rank 0's buffers ----
  std::vector<void*> frame(NB), gathered(NB);
  const size_t frame_bytes = (size_t)W * H * 16;
  for (int b = 0; b < NB; ++b) {
    hip(hipMalloc(&frame[b], frame_bytes), "hipMalloc frame");
    hip(hipMalloc(&gathered[b], (size_t)pitch * N), "hipMalloc gathered");
    hip(hipMemset(gathered[b], 0, (size_t)pitch * N), "hipMemset");
  }
  const int NR = std::min(NB, 4);
  std::vector<hipStream_t> rs(NR);
  for (auto& s : rs) hip(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "stream");
  hipStream_t ss, ds;
  hip(hipStreamCreateWithFlags(&ss, hipStreamNonBlocking), "stream");
  hip(hipStreamCreateWithFlags(&ds, hipStreamNonBlocking), "stream");
  std::vector<hipEvent_t> ev_render(NB), ev_dec(NB), ev_recv(NB), ev_size(NB);
  for (auto* v : {&ev_render, &ev_dec, &ev_recv, &ev_size})
    for (auto& e : *v) hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
  int32_t *lens_dev, *sizes_dev;
  hip(hipMalloc((void**)&lens_dev, 64), "hipMalloc");
  hip(hipMalloc((void**)&sizes_dev, 64 * 4), "hipMalloc");
  hip(hipMemset(lens_dev, 0, 64), "hipMemset");
  int32_t* sizes_host;
  hip(hipHostMalloc((void**)&sizes_host, 64 * 4, hipHostMallocDefault), "hipHostMalloc");
  uint32_t* status;   // the checked decode's status words, one per part per buffer set
  hip(hipMalloc((void**)&status, sizeof(uint32_t) * N * NB), "hipMalloc");
  hip(hipMemset(status, 0, sizeof(uint32_t) * N * NB), "hipMemset");
  sdf_tiling t0 = til[0];
  t0.flags = SDF_TILING_FRAME_ROWS;
  hip(hipDeviceSynchronize(), "sync");

  double host = 0.0, h_render = 0.0, h_rccl = 0.0, h_decode = 0.0;
  auto frame_loop = [&](int count, long long base) {
    for (int k = 0; k < count; ++k) {
      const long long i = base + k;
      const int b = (int)(i % NB), s = (int)(i % NS);
      hipStream_t st = rs[b % NR];
      const auto t = Clock::now();
      if (do_render)
        ok(sdf_render(&scene, &cams[s], &light, &material, &params, &t0, frame[b], nullptr, st),
           "sdf_render root");
      h_render += since(t);
      const auto tc = Clock::now();
      hip(hipEventRecord(ev_render[b], st), "event");
      if ((i + 1) % B == 0 && (do_rccl || do_decode)) {
        const int b0 = b + 1 - B;
        if (do_rccl) {
        // the lengths of the batch (world 1: the real all-gather of batch int32)
        for (int f = 0; f < B; ++f) hip(hipStreamWaitEvent(ss, ev_render[b0 + f], 0), "wait");
        nccl(R.AllGather(lens_dev, sizes_dev, (size_t)B, ncclInt32, size_comm, ss), "allgather");
        hip(hipMemcpyAsync(sizes_host, sizes_dev, B * 4, hipMemcpyDeviceToHost, ss), "copy");
        hip(hipEventRecord(ev_size[b0], ss), "event");
        // the group: N - 1 streams per frame to rank 0 (itself), fresh buffers
        for (int f = 0; f < B; ++f) hip(hipStreamWaitEvent(ds, ev_dec[b0 + f], 0), "wait");
        nccl(R.GroupStart(), "group");
        for (int f = 0; f < B; ++f) {
          const int sf = (int)((i - B + 1 + f) % NS);
          for (int r = 1; r < N; ++r) {
            const size_t n = (size_t)(data_off[r] + used[sf][r]);
            nccl(R.Send(part[sf][r], n, ncclUint8, 0, data_comm, ds), "send");
            nccl(R.Recv(static_cast<char*>(gathered[b0 + f]) + (size_t)r * pitch, n, ncclUint8, 0,
                        data_comm, ds),
                 "recv");
          }
        }
        nccl(R.GroupEnd(), "group end");
        hip(hipEventRecord(ev_recv[b0], ds), "event");
        }
        if (do_copy) {
          for (int f = 0; f < B; ++f) hip(hipStreamWaitEvent(ds, ev_dec[b0 + f], 0), "wait");
          CopyList L{};
          for (int f = 0; f < B; ++f) {
            const int sf = (int)((i - B + 1 + f) % NS);
            for (int r = 1; r < N; ++r) {
              char* dst = static_cast<char*>(gathered[b0 + f]) + (size_t)r * pitch;
              const size_t n = (size_t)(data_off[r] + used[sf][r]);
              if (one_kernel && L.count < 32) {
                L.src[L.count] = static_cast<const uint4*>(part[sf][r]);
                L.dst[L.count] = reinterpret_cast<uint4*>(dst);
                L.n16[L.count++] = (n + 15) / 16;
              } else {
                hip(hipMemcpyAsync(dst, part[sf][r], n, hipMemcpyDeviceToDevice, ds), "copy-in");
              }
            }
          }
          if (one_kernel) hipLaunchKernelGGL(copy_streams, dim3(512), dim3(256), 0, ds, L);
          hip(hipEventRecord(ev_recv[b0], ds), "event");
        }
        h_rccl += since(tc);
        const auto td = Clock::now();
        for (int f = 0; f < B && do_decode; ++f) {
          const int bf = b0 + f, sf = (int)((i - B + 1 + f) % NS);
          hipStream_t sb = rs[bf % NR];
          if (do_rccl || do_copy) hip(hipStreamWaitEvent(sb, ev_recv[b0], 0), "wait");
          ok(sdf_tiles_decode_checked(do_rccl || do_copy ? gathered[bf] : setbuf[sf], N, pitch,
                                      til.data(),
                                      used[sf].data(), W, H, frame[bf],
                                      status + (size_t)N * bf, sb),
             "decode");
          hip(hipEventRecord(ev_dec[bf], sb), "event");
        }
        h_decode += since(td);
      }
      host += since(t);
    }
  };
  frame_loop(WARM, 0);
  hip(hipDeviceSynchronize(), "sync");
  host = h_render = h_rccl = h_decode = 0.0;
  const auto t_run = Clock::now();
  frame_loop(K, WARM);
  hip(hipDeviceSynchronize(), "sync");
  const double wall = since(t_run);
  // ---- checks ----
  std::vector<uint32_t> st(N * NB);
  hip(hipMemcpy(st.data(), status, st.size() * 4, hipMemcpyDeviceToHost), "status");
  unsigned bad = 0;
  for (uint32_t v : st) bad |= v;
  const long long last = WARM + K - 1;
  const int bl = (int)(last % NB), sl = (int)(last % NS);
  void* ref;
  hip(hipMalloc(&ref, frame_bytes), "hipMalloc ref");
  ok(sdf_render(&scene, &cams[sl], &light, &material, &params, nullptr, ref, nullptr, nullptr),
      "sdf_render ref");
  std::vector<unsigned char> a(frame_bytes), c(frame_bytes);
  hip(hipMemcpy(a.data(), frame[bl], frame_bytes, hipMemcpyDeviceToHost), "copy");
  hip(hipMemcpy(c.data(), ref, frame_bytes, hipMemcpyDeviceToHost), "copy");
  const bool exact = mode != "full" && mode != "norccl" && !do_copy
                         ? true   // no whole frame is assembled
                         : std::memcmp(a.data(), c.data(), frame_bytes) == 0;
  std::printf("{\"mode\": \"%s\", \"world\": %d, \"shares\": \"%d:%d\", \"batch\": %d, \"nbuf\": %d, \"sets\": %d, "
              "\"frames\": %d, \"ms_per_frame\": %.4f, \"host_us_per_frame\": %.2f, "
              "\"host_us_split\": {\"render\": %.2f, \"rccl\": %.2f, \"decode\": %.2f}, "
              "\"set_mbytes\": %.2f, \"peer_stream_mbytes\": %.3f, \"status_bits\": %u, "
              "\"last_frame_bit_exact\": %s}\n",
              mode.c_str(), N, SA, SB, B, NB, NS, K, wall / K * 1e3, host / K * 1e6,
              h_render / K * 1e6, h_rccl / K * 1e6, h_decode / K * 1e6, set_bytes / 1e6,
              set_bytes / 1e6 / NS / (N - 1), bad, exact ? "true" : "false");
  (void)R.CommDestroy(data_comm);
  (void)R.CommDestroy(size_comm);
  return exact && bad == 0 ? 0 : 1;
}

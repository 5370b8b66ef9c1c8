// valu_rates.hip -- issue-rate microbenchmark for the instruction classes the
// render kernel is made of, at full occupancy (8 waves per SIMD) on every CU.
//
// Each lane runs ITERS iterations of 8 independent chains of one instruction
// class (inline asm with per-chain operands, so the compiler cannot fuse or
// drop them and no two chains share a source register).  Every wave reads the
// shader clock (s_memtime) and the 100 MHz real-time counter (s_memrealtime)
// around its loop, so the result is in measured shader cycles:
//   cycles per wave-instruction on one SIMD
//     = wave loop cycles / (instructions per wave x waves per SIMD).
//
//   hipcc -O3 --offload-arch=gfx950 tools/valu_rates.hip -o tools/valu_rates.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int ITERS = 4096;
constexpr int WAVES_PER_SIMD = 8;

#define CHAIN8(op) op(0) op(1) op(2) op(3) op(4) op(5) op(6) op(7)

__device__ __forceinline__ unsigned long long memtime() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}
__device__ __forceinline__ unsigned long long realtime() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t));
  return t;
}

template <int KIND>
__global__ __launch_bounds__(256) void bench(float* out, unsigned long long* tm, float s) {
  float a[8], b[8], c[8];
  f2 pa[8], pb[8];
  for (int i = 0; i < 8; i++) {
    a[i] = threadIdx.x * 0.001f + i + s;
    b[i] = 1.0f + i * 1e-3f;
    c[i] = 0.5f * i;
    pa[i] = f2{a[i], a[i] + 1.0f};
    pb[i] = f2{b[i], c[i]};
  }
  __builtin_amdgcn_s_barrier();
  const unsigned long long t0 = memtime(), r0 = realtime();
  for (int it = 0; it < ITERS; it++) {
    if constexpr (KIND == 0) {
#define OP(i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b[i]), "v"(c[i]));
      CHAIN8(OP)
#undef OP
    } else if constexpr (KIND == 1) {
#define OP(i) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(pa[i]) : "v"(pb[i]));
      CHAIN8(OP)
#undef OP
    } else if constexpr (KIND == 2) {
#define OP(i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
      CHAIN8(OP)
#undef OP
    } else if constexpr (KIND == 3) {
#define OP(i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(pa[i]) : "v"(pb[i]));
      CHAIN8(OP)
#undef OP
    } else if constexpr (KIND == 4) {
#define OP(i) asm volatile("v_sqrt_f32 %0, %0" : "+v"(a[i]));
      CHAIN8(OP)
#undef OP
    } else if constexpr (KIND == 5) {
#define OP(i) asm volatile("v_min_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
      CHAIN8(OP)
#undef OP
    } else if constexpr (KIND == 6) {
#define OP(i) \
  asm volatile("v_cmp_gt_f32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b[i]) : "vcc");
      CHAIN8(OP)
#undef OP
    } else if constexpr (KIND == 7) {
#define OP(i)                                                                  \
  asm volatile("v_sqrt_f32 %0, %0\n\tv_fma_f32 %1, %1, %2, %2\n\t"             \
               "v_fma_f32 %1, %1, %2, %2\n\tv_fma_f32 %1, %1, %2, %2"           \
               : "+v"(a[i]), "+v"(c[i]) : "v"(b[i]));
      CHAIN8(OP)
#undef OP
    } else if constexpr (KIND == 8) {
#define OP(i) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b[i]));
      CHAIN8(OP)
#undef OP
    } else {
      // dependent chain: one accumulator (latency-bound for a single wave)
#define OP(i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[0]) : "v"(b[i]), "v"(c[i]));
      CHAIN8(OP)
#undef OP
    }
  }
  const unsigned long long t1 = memtime(), r1 = realtime();
  float r = 0;
  for (int i = 0; i < 8; i++) r += a[i] + c[i] + pa[i].x + pa[i].y;
  out[blockIdx.x * 256 + threadIdx.x] = r;
  if ((threadIdx.x & 63) == 0) {
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    tm[2 * w] = t1 - t0;
    tm[2 * w + 1] = r1 - r0;
  }
}

int main() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int blocks = cus * 4 * WAVES_PER_SIMD / 4;   // 4 waves per block
  const int waves = blocks * 4;
  float* out;
  unsigned long long* tm;
  (void)hipMalloc(&out, (size_t)blocks * 256 * sizeof(float));
  (void)hipMalloc(&tm, (size_t)waves * 2 * sizeof(unsigned long long));
  std::vector<unsigned long long> h(waves * 2);
  struct K { const char* name; void (*fn)(float*, unsigned long long*, float); int insts; };
  K ks[] = {{"v_fma_f32", bench<0>, 8},       {"v_pk_fma_f32", bench<1>, 8},
            {"v_add_f32", bench<2>, 8},       {"v_pk_add_f32", bench<3>, 8},
            {"v_sqrt_f32", bench<4>, 8},      {"v_min_f32", bench<5>, 8},
            {"v_cmp+v_cndmask", bench<6>, 16}, {"sqrt+3fma", bench<7>, 32},
            {"v_mul_f32", bench<8>, 8},       {"fma_dependent_chain", bench<9>, 8}};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  printf("{\"cus\": %d, \"waves_per_simd\": %d, \"rates\": {", cus, WAVES_PER_SIMD);
  const int nk = sizeof(ks) / sizeof(ks[0]);
  for (int k = 0; k < nk; k++) {
    double best = 1e30, mhz = 0;
    float best_ms = 1e30f;
    for (int r = 0; r < 4; r++) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(ks[k].fn, dim3(blocks), dim3(256), 0, 0, out, tm, 1.0001f);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (r > 0) best_ms = std::min(best_ms, ms);
      (void)hipMemcpy(h.data(), tm, h.size() * 8, hipMemcpyDeviceToHost);
      std::vector<double> cyc, rt;
      for (int w = 0; w < waves; w++) cyc.push_back((double)h[2 * w]), rt.push_back((double)h[2 * w + 1]);
      std::sort(cyc.begin(), cyc.end());
      std::sort(rt.begin(), rt.end());
      const double med = cyc[waves / 2], medrt = rt[waves / 2];
      if (r > 0 && med < best) best = med, mhz = med / (medrt / 100.0);   // realtime = 100 MHz
    }
    // per SIMD: WAVES_PER_SIMD waves x ITERS x insts wave-instructions in the
    // kernel time, at the shader clock the waves measured
    const double insts = (double)ITERS * ks[k].insts * WAVES_PER_SIMD;
    printf("%s\"%s\": {\"kernel_ms\": %.4f, \"shader_mhz\": %.0f, "
           "\"cycles_per_wave_inst\": %.3f, \"at_2400\": %.3f}",
           k ? ", " : "", ks[k].name, best_ms, mhz, best_ms * 1e-3 * mhz * 1e6 / insts,
           best_ms * 1e-3 * 2.4e9 / insts);
  }
  printf("}}\n");
  (void)hipFree(out);
  (void)hipFree(tm);
  return 0;
}

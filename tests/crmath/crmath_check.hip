// crmath_check.hip -- TEST INFRASTRUCTURE: exhaustive GPU check of the
// exact-precision kernel's correctly rounded building blocks
// (sdf3d_amd/csrc/cr_math.h) against the generic sequences they replace:
//   sqrt : cr_sqrt(x) vs IEEE sqrtf(x) on all 2^32 bit patterns
//   rcp  : rcp_fast(x) vs IEEE 1.0f / x on its domain [2^-100, 2^100)
//   log  : cr_log(x) vs (float)log((double)x) on all 2^32 bit patterns
//   smin : div_scaled(n, k, sc, ys) vs n / k over the smooth-min domain
//          (every positive finite k, n in [0, k]): bits, and h*h*k*0.25
//          (what the smooth-min uses) -- 2^32 (k, n) pairs, k uniform in
//          bits, n spread over [0, k] including tiny and denormal n
// Prints one JSON line.  Built by sdf3d_amd/build.py (build_crmath_check);
// run by tests/test_gpu_crmath.py.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

#include "../../sdf3d_amd/csrc/cr_math.h"

struct Counts {
  unsigned long long mismatch, fast, effective;
  unsigned first[8];
  unsigned nfirst;
};

__device__ __forceinline__ bool same_bits(float a, float b) {
  return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}

__device__ void tally(Counts* c, bool bad, bool fast, bool eff, unsigned tag) {
  const unsigned long long mb = __builtin_amdgcn_ballot_w64(bad);
  const unsigned long long fb = __builtin_amdgcn_ballot_w64(fast);
  const unsigned long long eb = __builtin_amdgcn_ballot_w64(eff);
  const unsigned lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if (lane == 0) {
    if (mb) atomicAdd(&c->mismatch, (unsigned long long)__builtin_popcountll(mb));
    if (fb) atomicAdd(&c->fast, (unsigned long long)__builtin_popcountll(fb));
    if (eb) atomicAdd(&c->effective, (unsigned long long)__builtin_popcountll(eb));
  }
  if (bad) {
    const unsigned slot = atomicAdd(&c->nfirst, 1u);
    if (slot < 8) c->first[slot] = tag;
  }
}

__global__ void check_sqrt(unsigned base, Counts* c) {
  const unsigned u = base + blockIdx.x * blockDim.x + threadIdx.x;
  const float x = __uint_as_float(u);
  const float a = sdf::crm::cr_sqrt(x), b = __builtin_sqrtf(x);
  const bool bad = !same_bits(a, b);
  tally(c, bad, sdf::crm::sqrt_fast_ok(x), bad, u);
}

__global__ void check_rcp(unsigned base, Counts* c) {
  const unsigned u = base + blockIdx.x * blockDim.x + threadIdx.x;
  const float x = __uint_as_float(u);
  const bool in = sdf::crm::sqrt_fast_ok(x);   // its domain: [2^-100, 2^100)
  const float a = sdf::crm::rcp_fast(x), b = 1.0f / x;
  const bool bad = in && !same_bits(a, b);
  tally(c, bad, in, bad, u);
}

__global__ void check_log(unsigned base, Counts* c) {
  const unsigned u = base + blockIdx.x * blockDim.x + threadIdx.x;
  const float x = __uint_as_float(u);
  const float a = sdf::crm::cr_log(x), b = (float)log((double)x);
  const bool bad = !same_bits(a, b);
  // "fast": lanes whose fast value was safe to round (recomputed here)
  const double v = sdf::crm::log_fast(x);
  const double tol = SDF_CRM_LOG_EPS * __builtin_fabs(v);
  const bool ok = ((float)(v - tol) == (float)v) & ((float)(v + tol) == (float)v) &
                  ((u - 0x00800000u) < (0x7F800000u - 0x00800000u));
  tally(c, bad, ok, bad, u);
}

__device__ __forceinline__ unsigned hash32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

__global__ void check_smin(unsigned base, Counts* c) {
  const unsigned i = base + blockIdx.x * blockDim.x + threadIdx.x;
  // k: 2^20 values, uniform in bits over every positive finite float
  // (denormals included: the host's scaling must cover them); n: 4096 per k
  const unsigned ki = i >> 12, ni = i & 4095u;
  const unsigned kbits = 1u + (unsigned)(((unsigned long long)hash32(ki) * 0x7F7FFFFFull) >> 32);
  const float k = __uint_as_float(kbits);
  // the host's preparation (sdf_abi.cpp prepare_prims): sc = 2^min(1 - e, 127)
  // with k = m 2^e, m in [0.5, 1); ys = RN(1/(k sc))
  const int e = __builtin_amdgcn_frexp_expf(k);
  const float sc = __builtin_ldexpf(1.0f, (1 - e) < 127 ? (1 - e) : 127);
  const float ys = 1.0f / (k * sc);
  float n;
  const unsigned h = hash32(i * 2654435761u + 12345u);
  if (ni < 2048) n = k * (__uint_as_float(0x3F800000u | (h >> 9)) - 1.0f);  // [0, k)
  else if (ni < 3072) n = __uint_as_float(h % kbits);                      // any float below k
  else if (ni < 3584) n = __uint_as_float(h & 0x007FFFFFu) < k
                              ? __uint_as_float(h & 0x007FFFFFu) : 0.0f;   // denormal
  else n = __uint_as_float(kbits - (h & 0xFFFu) < kbits ? kbits - (h & 0xFFFu) : 0u);
  if (!(n <= k)) n = k;
  const float a = sdf::crm::div_scaled(n, k, sc, ys), b = n / k;
  const bool bad = !same_bits(a, b);
  const bool eff = !same_bits(a * a * k * 0.25f, b * b * k * 0.25f);
  tally(c, bad, true, eff, i);
}

static int run(const char* name, void (*kern)(unsigned, Counts*), Counts* d, char* out,
               size_t cap) {
  (void)hipMemset(d, 0, sizeof(Counts));
  const unsigned threads = 256, chunk = 1u << 28;
  for (unsigned long long base = 0; base < (1ull << 32); base += chunk) {
    hipLaunchKernelGGL(kern, dim3(chunk / threads), dim3(threads), 0, 0, (unsigned)base, d);
    if (hipDeviceSynchronize() != hipSuccess) return -1;
  }
  Counts h;
  (void)hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost);
  char firsts[200] = "";
  for (unsigned j = 0; j < (h.nfirst < 8 ? h.nfirst : 8); j++) {
    char tmp[24];
    snprintf(tmp, sizeof tmp, "%s%u", j ? "," : "", h.first[j]);
    strncat(firsts, tmp, sizeof firsts - strlen(firsts) - 1);
  }
  return snprintf(out, cap, "\"%s\": {\"inputs\": %llu, \"mismatch\": %llu, \"effective\": %llu, "
                  "\"fast_path\": %llu, \"first\": [%s]}", name, 1ull << 32, h.mismatch,
                  h.effective, h.fast, firsts);
}

int main(int argc, char** argv) {
  Counts* d;
  if (hipMalloc(&d, sizeof(Counts)) != hipSuccess) return 2;
  char a[400], b[400], c[400], r[400];
  const bool all = argc < 2;
  const bool want_sqrt = all || strstr(argv[1], "sqrt"), want_log = all || strstr(argv[1], "log"),
             want_smin = all || strstr(argv[1], "smin"), want_rcp = all || strstr(argv[1], "rcp");
  a[0] = b[0] = c[0] = r[0] = 0;
  if (want_rcp && run("rcp", check_rcp, d, r, sizeof r) < 0) return 3;
  if (want_sqrt && run("sqrt", check_sqrt, d, a, sizeof a) < 0) return 3;
  if (want_log && run("log", check_log, d, b, sizeof b) < 0) return 3;
  if (want_smin && run("smin", check_smin, d, c, sizeof c) < 0) return 3;
  printf("{%s%s%s%s%s%s%s}\n", r, (r[0] && (a[0] || b[0] || c[0])) ? ", " : "", a,
         (a[0] && (b[0] || c[0])) ? ", " : "", b, (b[0] && c[0]) ? ", " : "", c);
  (void)hipFree(d);
  return 0;
}

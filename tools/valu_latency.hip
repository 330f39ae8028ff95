// Dependent-issue interval of the NTT butterfly's gfx950 VALU forms (round 4): cycles between
// back-to-back dependent instructions of one wave, with W waves per SIMD and C independent chains
// per thread.  valu_rates*.hip measure throughput (8 chains, 8 waves); this asks whether the
// encrypt block passes (3 waves per SIMD, short dependent chains in each butterfly) wait on
// latency: at W = 1, C = 1 the figure is the latency, at W * C >= latency / 4 it is the rate.
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_latency tools/valu_latency.hip && tools/valu_latency
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHK(x)                                                                    \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

constexpr int kIters = 65536;

#define MAD64(r) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(r) : "v"(a), "v"(b) : "s40", "s41");
#define MULHI(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define MULLO(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define ADD32(x) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(x) : "v"(b));
#define LSHLADD64(r) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(r) : "v"(bb));
#define ADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x) : "v"(b));
#define BFI(x) asm volatile("v_bfi_b32 %0, %0, %1, %1" : "+v"(x) : "v"(b));

template <int KIND, int C>
__global__ __launch_bounds__(256) void lat_kernel(uint32_t* out, uint32_t seed, uint64_t* clk) {
  const uint32_t a = seed ^ threadIdx.x, b = seed * 0x9e3779b9u + blockIdx.x;
  const uint64_t bb = (uint64_t)b * 77;
  uint32_t x[C];
  uint64_t r[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    x[c] = a * (2 * c + 3);
    r[c] = (uint64_t)x[c] * 5;
  }
  uint64_t c0 = 0, c1 = 0;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    c0 = __builtin_amdgcn_s_memtime();
    c1 = __builtin_amdgcn_s_memrealtime();
  }
#pragma unroll 1
  for (int i = 0; i < kIters / 8; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        if (KIND == 0) { MAD64(r[c]) }
        if (KIND == 1) { MULHI(x[c]) }
        if (KIND == 2) { MULLO(x[c]) }
        if (KIND == 3) { ADD32(x[c]) }
        if (KIND == 4) { LSHLADD64(r[c]) }
        if (KIND == 5) { ADD3(x[c]) }
        if (KIND == 6) { BFI(x[c]) }
      }
    }
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - c0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - c1;
  }
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < C; ++c) acc ^= x[c] ^ (uint32_t)r[c] ^ (uint32_t)(r[c] >> 32);
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}
static const char* kNames[] = {"v_mad_u64_u32 (acc chain)", "v_mul_hi_u32", "v_mul_lo_u32", "v_add_u32_e32",
                               "v_lshl_add_u64", "v_add3_u32", "v_bfi_b32"};

template <int KIND, int C>
static int run(int cus, int W, uint32_t* out, uint64_t* clk) {
  const int blocks = cus * W;  // one 4-wave block per CU per W: W waves per SIMD
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL((lat_kernel<KIND, C>), dim3(blocks), dim3(256), 0, 0, out, 1u, clk);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((lat_kernel<KIND, C>), dim3(blocks), dim3(256), 0, 0, out, 1u, clk);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  uint64_t c[2];
  CHK(hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost));
  const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
  // cycles per dependent instruction of one chain of one wave (kernel cycles / chain length)
  const double cyc_chain = (ms / 5 * 1e-3) * ghz * 1e9 / kIters;
  // SIMD cycles per wave-instruction issued (all W waves x C chains)
  const double cyc_issue = cyc_chain / (W * C);
  printf("%-26s W=%d C=%d  %8.3f ms  clock %.2f GHz  %6.2f cycles between dependent instrs  %5.2f per issued\n",
         kNames[KIND], W, C, ms / 5, ghz, cyc_chain, cyc_issue);
  return 0;
}

template <int KIND>
static int run_kind(int cus, uint32_t* out, uint64_t* clk) {
  for (int W : {1, 2, 3}) {
    if (run<KIND, 1>(cus, W, out, clk)) return 1;
    if (run<KIND, 2>(cus, W, out, clk)) return 1;
  }
  if constexpr (KIND + 1 < (int)(sizeof(kNames) / sizeof(kNames[0]))) return run_kind<KIND + 1>(cus, out, clk);
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device %s, %d CUs\n", prop.gcnArchName, cus);
  uint32_t* out;
  uint64_t* clk;
  CHK(hipMalloc(&out, (size_t)cus * 3 * 256 * 4));
  CHK(hipMalloc(&clk, 16));
  return run_kind<0>(cus, out, clk);
}

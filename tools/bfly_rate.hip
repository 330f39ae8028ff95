// Issue cost of the encrypt NTT's NORED butterfly (dev_common.h ct_bfly_s<false>) on gfx950 with the
// operands in registers: cycles per wave-butterfly per SIMD at W waves per SIMD and C independent
// butterflies per thread per step.  Against the block pass's measured cost per wave-butterfly this
// separates the butterfly's own issue cost from the pass's LDS exchanges, loads and barriers.
// (Values wrap mod 2^64 over the long loop: only the issue cost is measured, not a transform.)
//   hipcc --offload-arch=gfx950 -O3 -I fhe-fed_amd/csrc -I include -o tools/bfly_rate tools/bfly_rate.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#include "dev_common.h"

#define CHK(x)                                                                    \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

constexpr int kSteps = 4096;

template <int C>
__global__ __launch_bounds__(256) void bfly_kernel(uint64_t* out, uint64_t q, const uint64_t* tw, uint64_t* clk) {
  uint64_t x[2 * C];
#pragma unroll
  for (int c = 0; c < 2 * C; ++c) x[c] = (threadIdx.x * 2654435761ull + c * 40503ull) % q;
  // four twiddle pairs in registers, rotated per step (the pass reads its pairs from LDS)
  uint64_t W[4], Wp[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    W[i] = tw[2 * i];
    Wp[i] = tw[2 * i + 1];
  }
  uint64_t c0 = 0, c1 = 0;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    c0 = __builtin_amdgcn_s_memtime();
    c1 = __builtin_amdgcn_s_memrealtime();
  }
#pragma unroll 1
  for (int s = 0; s < kSteps / 4; ++s) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int c = 0; c < C; ++c) shelfi::ct_bfly_s<false>(x[2 * c], x[2 * c + 1], W[(u + c) & 3], Wp[(u + c) & 3], q, 0);
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - c0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - c1;
  }
  uint64_t acc = 0;
#pragma unroll
  for (int c = 0; c < 2 * C; ++c) acc ^= x[c];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int C>
static int run(int cus, int Wv, uint64_t* out, uint64_t q, const uint64_t* tw, uint64_t* clk) {
  const int blocks = cus * Wv;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL((bfly_kernel<C>), dim3(blocks), dim3(256), 0, 0, out, q, tw, clk);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((bfly_kernel<C>), dim3(blocks), dim3(256), 0, 0, out, q, tw, clk);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  uint64_t c[2];
  CHK(hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost));
  const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
  const double cyc = (ms / 5 * 1e-3) * ghz * 1e9 / ((double)kSteps * C * Wv);  // per wave-butterfly per SIMD
  printf("W=%d C=%d  %8.3f ms  clock %.2f GHz  %6.2f cycles per wave-butterfly per SIMD\n", Wv, C, ms / 5, ghz, cyc);
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device %s, %d CUs; ct_bfly_s<false>, q = 2^52 - 2^20 + 1 class\n", prop.gcnArchName, cus);
  const uint64_t q = (1ull << 52) - (1ull << 20) + 1;
  uint64_t htw[8];
  for (int i = 0; i < 4; ++i) {
    htw[2 * i] = (0x123456789abull * (i + 1)) % q;
    htw[2 * i + 1] = (uint64_t)(((unsigned __int128)htw[2 * i] << 64) / q);
  }
  uint64_t *out, *tw, *clk;
  CHK(hipMalloc(&out, (size_t)cus * 4 * 256 * 8));
  CHK(hipMalloc(&tw, sizeof(htw)));
  CHK(hipMalloc(&clk, 16));
  CHK(hipMemcpy(tw, htw, sizeof(htw), hipMemcpyHostToDevice));
  for (int Wv : {1, 2, 3, 4}) {
    if (run<1>(cus, Wv, out, q, tw, clk) || run<2>(cus, Wv, out, q, tw, clk) || run<4>(cus, Wv, out, q, tw, clk) ||
        run<8>(cus, Wv, out, q, tw, clk))
      return 1;
  }
  return 0;
}

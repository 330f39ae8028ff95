// Issue cost of the VALU instructions the NTT butterflies are built from, on gfx950:
// cycles per wave64 instruction per SIMD at full occupancy (8 independent chains per
// thread, 8 waves per SIMD), from the kernel time and the shader clock the kernel itself
// measures (s_memtime vs s_memrealtime at 100 MHz).
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rates tools/valu_rates.hip && tools/valu_rates
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                             \
    }                                                                       \
  } while (0)

constexpr int kIters = 2048;

#define BODY8(OP) OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)
#define BODY8R(OP) OP(r0) OP(r1) OP(r2) OP(r3) OP(r4) OP(r5) OP(r6) OP(r7)

template <int KIND>
__global__ __launch_bounds__(256) void rate_kernel(uint32_t* out, uint32_t seed, uint64_t* clk) {
  uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,
           a6 = a0 * 17, a7 = a0 * 19;
  uint32_t b = seed * 0x9e3779b9u + blockIdx.x;
  uint64_t c0 = 0, c1 = 0;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    c0 = __builtin_amdgcn_s_memtime();
    c1 = __builtin_amdgcn_s_memrealtime();
  }
  uint64_t r0 = a0, r1 = a1, r2 = a2, r3 = a3, r4 = a4, r5 = a5, r6 = a6, r7 = a7;
  const uint64_t bb = b;
  double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7;
  const double db = b;
  uint32_t h0 = a0, h1 = a1, h2 = a2, h3 = a3;
  uint64_t sc;
#pragma unroll 1
  for (int i = 0; i < kIters / 16; ++i) {
#pragma unroll
   for (int u = 0; u < 16; ++u) {
    if (KIND == 0) {  // v_add_u32 (full-rate reference)
#define OP(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
      BODY8(OP)
#undef OP
    } else if (KIND == 1) {  // v_mul_lo_u32
#define OP(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
      BODY8(OP)
#undef OP
    } else if (KIND == 2) {  // v_mul_hi_u32
#define OP(x) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(x) : "v"(b));
      BODY8(OP)
#undef OP
    } else if (KIND == 3) {  // v_mad_u64_u32 (64-bit result, 64-bit addend), chained on the addend
#define OP(r) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(r), "=s"(sc) : "v"(a1), "v"(b));
      BODY8R(OP)
#undef OP
    } else if (KIND == 4) {  // v_lshl_add_u64
#define OP(r) asm volatile("v_lshl_add_u64 %0, %1, 2, %0" : "+v"(r) : "v"(bb));
      BODY8R(OP)
#undef OP
    } else if (KIND == 5) {  // v_add_co_u32 + v_addc_co_u32 (64-bit add pair)
#define OP2(lo, hi) asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %2, vcc" \
                                 : "+v"(lo), "+v"(hi) : "v"(b) : "vcc");
      OP2(a4, h0) OP2(a5, h1) OP2(a6, h2) OP2(a7, h3)
#undef OP2
    } else if (KIND == 6) {  // v_bfi_b32
#define OP(x) asm volatile("v_bfi_b32 %0, %1, %0, %1" : "+v"(x) : "v"(b));
      BODY8(OP)
#undef OP
    } else if (KIND == 7) {  // v_add3_u32
#define OP(x) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x) : "v"(b));
      BODY8(OP)
#undef OP
    } else if (KIND == 8) {  // v_fma_f64 (for comparison)
#define OP(x) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(x) : "v"(db));
      OP(d0) OP(d1) OP(d2) OP(d3) OP(d4) OP(d5) OP(d6) OP(d7)
#undef OP
    }
   }
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - c0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - c1;
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ h0 ^ h1 ^ h2 ^ h3 ^
                                       (uint32_t)(r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7) ^
                                       (uint32_t)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);
}

static const char* kNames[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32",
                               "v_lshl_add_u64", "v_add_co+v_addc (2 inst)", "v_bfi_b32",
                               "v_add3_u32", "v_fma_f64"};
static const double kInstPerOp[] = {1, 1, 1, 1, 1, 1, 1, 1, 1};  // kind 5: 4 pairs = 8 inst

template <int KIND>
static int run(int cus, uint32_t* out, uint64_t* clk) {
  const int blocks = cus * 8;  // 8 blocks of 4 waves per CU = 8 waves per SIMD
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(rate_kernel<KIND>, dim3(blocks), dim3(256), 0, 0, out, 1u, clk);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(rate_kernel<KIND>, dim3(blocks), dim3(256), 0, 0, out, 1u, clk);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  uint64_t c[2];
  CHK(hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost));
  const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;  // shader clock of block 0
  const double wave_inst = (double)blocks * 4 * kIters * 8 * kInstPerOp[KIND] * 5;
  const double simds = cus * 4.0;
  const double cyc = (ms * 1e-3) * ghz * 1e9 * simds / wave_inst;
  printf("%-26s %7.3f ms  clock %.2f GHz  %.2f cycles per wave64 instruction per SIMD\n",
         kNames[KIND], ms / 5, ghz, cyc);
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device %s, %d CUs\n", prop.gcnArchName, cus);
  uint32_t* out;
  uint64_t* clk;
  CHK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
  CHK(hipMalloc(&clk, 16));
  if (run<0>(cus, out, clk) || run<1>(cus, out, clk) || run<2>(cus, out, clk) || run<3>(cus, out, clk) ||
      run<4>(cus, out, clk) || run<5>(cus, out, clk) || run<6>(cus, out, clk) || run<7>(cus, out, clk) ||
      run<8>(cus, out, clk))
    return 1;
  return 0;
}

// Issue cost of the integer VALU instructions the NTT butterflies are built from, on
// gfx950: each kernel runs 8 independent chains of one instruction per lane (inline asm,
// so the instruction is exactly the one named) and the host reports cycles per
// wave-instruction per SIMD from the wall time and the in-kernel clock
// (s_memtime / s_memrealtime, 100 MHz).
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/valu_rates tools/valu_rates.hip && /tmp/valu_rates
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int kIters = 4096;

#define REP8(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)

template <int OP>
__global__ __launch_bounds__(256) void rate_kernel(uint32_t* out, uint32_t seed, uint64_t* clk) {
  uint32_t a[8], b = seed ^ threadIdx.x;
  uint64_t p[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { a[i] = seed + i * 977 + threadIdx.x; p[i] = a[i] * 3ull; }
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < kIters; ++it) {
#define ADD(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define MULLO(i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define MULHI(i) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
#define MAD64(i) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(p[i]) : "v"(a[i]), "v"(b) : "vcc");
#define LSHLADD(i) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(p[i]) : "v"(p[(i + 1) & 7]));
#define SUBCO(i) asm volatile("v_sub_co_u32 %0, vcc, %0, %1" : "+v"(a[i]) : "v"(b) : "vcc");
#define CMP64(i) asm volatile("v_cmp_gt_u64 vcc, %0, %1\n v_cndmask_b32 %2, %2, %3, vcc" : : "v"(p[i]), "v"(p[(i + 3) & 7]), "v"(a[i]), "v"(b) : "vcc");
    if (OP == 0) { REP8(ADD) }
    if (OP == 1) { REP8(MULLO) }
    if (OP == 2) { REP8(MULHI) }
    if (OP == 3) { REP8(MAD64) }
    if (OP == 4) { REP8(LSHLADD) }
    if (OP == 5) { REP8(SUBCO) }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += a[i] + (uint32_t)p[i] + (uint32_t)(p[i] >> 32);
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int waves_per_simd = 8;  // 8 waves/SIMD -> 8 blocks of 4 waves per CU
  const int blocks = cus * waves_per_simd;
  uint32_t* out;
  uint64_t* clk;
  CHECK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  CHECK(hipMalloc(&clk, 16));
  const char* names[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_lshl_add_u64",
                         "v_sub_co_u32"};
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int op = 0; op < 6; ++op) {
    for (int rep = 0; rep < 3; ++rep) {
      CHECK(hipEventRecord(e0));
      switch (op) {
        case 0: rate_kernel<0><<<blocks, 256>>>(out, rep, clk); break;
        case 1: rate_kernel<1><<<blocks, 256>>>(out, rep, clk); break;
        case 2: rate_kernel<2><<<blocks, 256>>>(out, rep, clk); break;
        case 3: rate_kernel<3><<<blocks, 256>>>(out, rep, clk); break;
        case 4: rate_kernel<4><<<blocks, 256>>>(out, rep, clk); break;
        case 5: rate_kernel<5><<<blocks, 256>>>(out, rep, clk); break;
      }
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      uint64_t c[2];
      CHECK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
      const double ghz = (double)c[0] / ((double)c[1] * 10.0);  // memrealtime: 100 MHz
      // wave-instructions per SIMD = waves/SIMD * iters * 8
      const double inst = (double)waves_per_simd * kIters * 8;
      const double cyc_wall = ms * 1e-3 * ghz * 1e9 / inst;
      const double cyc_kernel = (double)c[0] / ((double)kIters * 8);  // one wave's own view
      if (rep == 2)
        printf("%-16s %7.3f ms  clock %.2f GHz  %5.2f cyc/wave-inst/SIMD (wall)  %6.2f cyc per inst in one wave\n",
               names[op], ms, ghz, cyc_wall, cyc_kernel);
    }
  }
  return 0;
}

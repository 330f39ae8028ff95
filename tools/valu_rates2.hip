// Issue cost of more gfx950 VALU forms (round 3): is the ~4-cycle cost of the butterflies'
// instructions the VOP3 encoding or the operation?  Same method as valu_rates.hip: cycles
// per wave64 instruction per SIMD at 8 waves/SIMD, 8 independent chains per thread, from the
// kernel time and the shader clock block 0 measures (s_memtime vs s_memrealtime).
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rates2 tools/valu_rates2.hip && tools/valu_rates2
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

constexpr int kIters = 2048;

#define B8(OP) OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)
#define B8R(OP) OP(r0) OP(r1) OP(r2) OP(r3) OP(r4) OP(r5) OP(r6) OP(r7)

#define V_ADD_E32(x) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(x) : "v"(b));
#define V_ADD_E64(x) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(x) : "v"(b));
#define V_AND_E32(x) asm volatile("v_and_b32_e32 %0, %0, %1" : "+v"(x) : "v"(b));
#define V_LSHL_E32(x) asm volatile("v_lshlrev_b32_e32 %0, %1, %0" : "+v"(x) : "v"(b));
#define V_MUL24_E32(x) asm volatile("v_mul_u32_u24_e32 %0, %0, %1" : "+v"(x) : "v"(b));
#define V_MULHI24_E32(x) asm volatile("v_mul_hi_u32_u24_e32 %0, %0, %1" : "+v"(x) : "v"(b));
#define V_ALIGNBIT(x) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(x) : "v"(b));
#define V_LSHL_OR(x) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(x) : "v"(b));
#define V_SUB_CO_E32(x) asm volatile("v_sub_co_u32_e32 %0, vcc, %0, %1" : "+v"(x) : "v"(b) : "vcc");
#define V_SUB_CO_E64(x) asm volatile("v_sub_co_u32_e64 %0, s[40:41], %0, %1" : "+v"(x) : "v"(b) : "s40", "s41");
#define V_LSHLREV_B64(r) asm volatile("v_lshlrev_b64 %0, 1, %0" : "+v"(r));
#define V_MOV_B64(r) asm volatile("v_mov_b64 %0, %1" : "=v"(r) : "v"(bb + (r & 0)));
#define V_MAD24(x) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(x) : "v"(b));
#define V_XOR_E32(x) asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(x) : "v"(b));
#define V_CNDMASK_E64(x) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(x) : "v"(b) : "s40", "s41");
#define V_PERM(x) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(x) : "v"(b));
#define V_MAX_E32(x) asm volatile("v_max_u32_e32 %0, %0, %1" : "+v"(x) : "v"(b));
#define V_PK_ADD_F32(r) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(r) : "v"(bb));
#define V_ADD_F32(x) asm volatile("v_add_f32_e32 %0, %0, %1" : "+v"(x) : "v"(b));
#define V_ADD_F64(r) asm volatile("v_add_f64 %0, %0, %1" : "+v"(r) : "v"(bb));
#define V_MUL_LO_U16(x) asm volatile("v_mul_lo_u16_e32 %0, %0, %1" : "+v"(x) : "v"(b));
#define V_MUL_F64(r) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(r) : "v"(bb));


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
  const uint64_t bb = (uint64_t)b * 77;
#pragma unroll 1
  for (int i = 0; i < kIters / 16; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (KIND == 0) { B8(V_ADD_E32) }
      if (KIND == 1) { B8(V_ADD_E64) }
      if (KIND == 2) { B8(V_AND_E32) }
      if (KIND == 3) { B8(V_LSHL_E32) }
      if (KIND == 4) { B8(V_MUL24_E32) }
      if (KIND == 5) { B8(V_MULHI24_E32) }
      if (KIND == 6) { B8(V_ALIGNBIT) }
      if (KIND == 7) { B8(V_LSHL_OR) }
      if (KIND == 8) { B8(V_SUB_CO_E32) }
      if (KIND == 9) { B8(V_SUB_CO_E64) }
      if (KIND == 10) { B8R(V_LSHLREV_B64) }
      if (KIND == 11) { B8R(V_MOV_B64) }
      if (KIND == 12) { B8(V_MAD24) }
      if (KIND == 13) { B8(V_XOR_E32) }
      if (KIND == 14) { B8(V_CNDMASK_E64) }
      if (KIND == 15) { B8(V_PERM) }
      if (KIND == 16) { B8(V_MAX_E32) }
      if (KIND == 17) { B8R(V_PK_ADD_F32) }
      if (KIND == 18) { B8(V_ADD_F32) }
      if (KIND == 19) { B8R(V_ADD_F64) }
      if (KIND == 20) { B8(V_MUL_LO_U16) }
      if (KIND == 21) { B8R(V_MUL_F64) }
    }
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = __builtin_amdgcn_s_memtime() - c0;
    clk[1] = __builtin_amdgcn_s_memrealtime() - c1;
  }
  out[blockIdx.x * 256 + threadIdx.x] =
      a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7) ^ (uint32_t)bb;
}
static const char* kNames[] = {"v_add_u32_e32",      "v_add_u32_e64",    "v_and_b32_e32",    "v_lshlrev_b32_e32",
                               "v_mul_u32_u24_e32",  "v_mul_hi_u32_u24", "v_alignbit_b32",   "v_lshl_or_b32",
                               "v_sub_co_u32_e32",   "v_sub_co_u32_e64", "v_lshlrev_b64",    "v_mov_b64",
                               "v_mad_u32_u24",      "v_xor_b32_e32",    "v_cndmask_b32_e64", "v_perm_b32",
                               "v_max_u32_e32",      "v_pk_add_f32",     "v_add_f32_e32",    "v_add_f64",
                               "v_mul_lo_u16_e32",   "v_mul_f64"};

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
  const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
  const double wave_inst = (double)blocks * 4 * kIters * 8 * 5;
  const double cyc = (ms * 1e-3) * ghz * 1e9 * (cus * 4.0) / wave_inst;
  printf("%-22s %7.3f ms  clock %.2f GHz  %.2f cycles per wave64 instruction per SIMD\n", kNames[KIND], ms / 5, ghz,
         cyc);
  return 0;
}

template <int K>
static int run_all(int cus, uint32_t* out, uint64_t* clk) {
  if (run<K>(cus, out, clk)) return 1;
  if constexpr (K + 1 < (int)(sizeof(kNames) / sizeof(kNames[0]))) return run_all<K + 1>(cus, out, clk);
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
  return run_all<0>(cus, out, clk);
}

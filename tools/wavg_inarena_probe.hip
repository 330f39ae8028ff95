// Probe: does writing the weighted sum into an extra slot of the interleaved arena
// (reads and the write of a block in one contiguous (C+1) x 4 KiB region) make the
// wavg launch less sensitive to physical placement than a separate output buffer?
// Same kernel body as wavg_kernel<true> (kernels.hip); the only difference is where
// each block's 4 KiB of output goes.  Alternates the two layouts A/B in one process,
// over several fresh allocations.
//   hipcc -O3 --offload-arch=gfx950 -o tools/build/wavg_inarena tools/wavg_inarena_probe.hip
//   tools/build/wavg_inarena [K] [C] [allocs]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
struct TC {
  uint64_t q, one_shoup, r30, r30_shoup, r60, r60_shoup;
};
constexpr int kT = 256, kPB = 512;

__device__ __forceinline__ uint64_t red64(uint64_t x, uint64_t q, uint64_t s) {
  uint64_t r = x - __umul64hi(x, s) * q;
  return r >= q ? r - q : r;
}
__device__ __forceinline__ uint64_t smul(uint64_t x, uint64_t w, uint64_t wp, uint64_t q) {
  uint64_t r = x * w - __umul64hi(x, wp) * q;
  return r >= q ? r - q : r;
}
__device__ __forceinline__ uint64_t addm(uint64_t a, uint64_t b, uint64_t q) {
  uint64_t s = a + b;
  return s >= q ? s - q : s;
}
__device__ __forceinline__ uint64_t fold(uint64_t s00, uint64_t s01, uint64_t s10, uint64_t s11, const TC& c) {
  uint64_t a = red64(s00, c.q, c.one_shoup);
  uint64_t m = red64(s01, c.q, c.one_shoup) + red64(s10, c.q, c.one_shoup);
  uint64_t b = smul(m, c.r30, c.r30_shoup, c.q);
  uint64_t d = smul(red64(s11, c.q, c.one_shoup), c.r60, c.r60_shoup, c.q);
  return addm(addm(a, b, c.q), d, c.q);
}

// slots = learners per chunk in the arena (C, or C + 1 with the output in slot C);
// out == nullptr -> write into slot C of the block's chunk.
__global__ __launch_bounds__(kT) void wavg(const uint64_t* __restrict__ arena, uint32_t C, uint32_t slots,
                                          uint32_t logN, uint32_t L, const TC* __restrict__ tcs,
                                          const uint32_t* __restrict__ wl, uint64_t* __restrict__ out) {
  const uint64_t base = (uint64_t)blockIdx.x * kPB;
  const uint32_t t = (uint32_t)((base >> logN) % L);
  const TC c = tcs[t];
  const uint32_t M30 = (1u << 30) - 1;
  const uint64_t* __restrict__ src = arena + (uint64_t)blockIdx.x * slots * kPB + 2u * threadIdx.x;
  uint64_t s00a = 0, s01a = 0, s10a = 0, s11a = 0, s00b = 0, s01b = 0, s10b = 0, s11b = 0;
#pragma unroll 8
  for (uint32_t k = 0; k < C; ++k) {
    const uint32_t w0 = wl[(k * L + t) * 2], w1 = wl[(k * L + t) * 2 + 1];
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + (uint64_t)k * kPB));
    const uint32_t xa0 = v.x & M30, xa1 = (v.x >> 30) | (v.y << 2);
    const uint32_t xb0 = v.z & M30, xb1 = (v.z >> 30) | (v.w << 2);
    s00a += (uint64_t)xa0 * w0;
    s01a += (uint64_t)xa0 * w1;
    s10a += (uint64_t)xa1 * w0;
    s11a += (uint64_t)xa1 * w1;
    s00b += (uint64_t)xb0 * w0;
    s01b += (uint64_t)xb0 * w1;
    s10b += (uint64_t)xb1 * w0;
    s11b += (uint64_t)xb1 * w1;
  }
  const uint64_t r0 = fold(s00a, s01a, s10a, s11a, c), r1 = fold(s00b, s01b, s10b, s11b, c);
  u32x4 o;
  o.x = (uint32_t)r0;
  o.y = (uint32_t)(r0 >> 32);
  o.z = (uint32_t)r1;
  o.w = (uint32_t)(r1 >> 32);
  uint64_t* dst = out ? out + base + 2u * threadIdx.x
                      : const_cast<uint64_t*>(arena) + ((uint64_t)blockIdx.x * slots + C) * kPB + 2u * threadIdx.x;
  __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(dst));
}

__global__ void fill(uint64_t* p, uint64_t n, uint64_t q) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = i * 0x9E3779B97F4A7C15ull;
    z ^= z >> 29;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 32;
    p[i] = z % q;
  }
}

static uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) { return (unsigned __int128)a * b % q; }
static uint64_t shoup(uint64_t w, uint64_t q) { return (uint64_t)(((unsigned __int128)w << 64) / q); }

int main(int argc, char** argv) {
  const uint64_t K = argc > 1 ? atoll(argv[1]) : 714;
  const uint32_t C = argc > 2 ? atoi(argv[2]) : 16;
  const int allocs = argc > 3 ? atoi(argv[3]) : 3;
  const uint32_t logN = 15, L = 4;
  const uint64_t rows = K * 2 * L, words = rows << logN, chunks = words / kPB;
  std::vector<TC> tc(L);
  const uint64_t qs[4] = {0x0FFFFFFFFFFFC001ull, 0x0010000000060001ull, 0x000FFFFFFFE20001ull, 0x000FFFFFFFBE0001ull};
  for (uint32_t t = 0; t < L; ++t) {
    uint64_t q = qs[t];
    tc[t].q = q;
    tc[t].one_shoup = shoup(1, q);
    tc[t].r30 = (1ull << 30) % q;
    tc[t].r30_shoup = shoup(tc[t].r30, q);
    tc[t].r60 = mulmod(1ull << 30, 1ull << 30, q);
    tc[t].r60_shoup = shoup(tc[t].r60, q);
  }
  std::vector<uint32_t> wl(C * L * 2);
  for (uint32_t k = 0; k < C; ++k)
    for (uint32_t t = 0; t < L; ++t) {
      uint64_t W = (uint64_t)(tc[t].q / (C + 3)) * (k + 1) % tc[t].q;
      wl[(k * L + t) * 2] = (uint32_t)(W & ((1u << 30) - 1));
      wl[(k * L + t) * 2 + 1] = (uint32_t)(W >> 30);
    }
  TC* dtc;
  uint32_t* dwl;
  CK(hipMalloc(&dtc, L * sizeof(TC)));
  CK(hipMalloc(&dwl, wl.size() * 4));
  CK(hipMemcpy(dtc, tc.data(), L * sizeof(TC), hipMemcpyHostToDevice));
  CK(hipMemcpy(dwl, wl.data(), wl.size() * 4, hipMemcpyHostToDevice));
  const double bytes = (double)(C + 1) * words * 8;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("K=%llu C=%u: %.2f GB per launch, %llu blocks\n", (unsigned long long)K, C, bytes / 1e9,
         (unsigned long long)chunks);
  const int nout = argc > 4 ? atoi(argv[4]) : 0;
  if (nout > 0) {  // matrix mode: arenas x output buffers, separate-output layout only
    for (int a = 0; a < allocs; ++a) {
      uint64_t* ar;
      CK(hipMalloc(&ar, chunks * C * kPB * 8));
      hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, ar, chunks * C * kPB, qs[1]);
      std::vector<uint64_t*> outs(nout);
      for (auto& o : outs) CK(hipMalloc(&o, words * 8));
      CK(hipDeviceSynchronize());
      printf("arena %d:", a);
      for (int rep = 0; rep < 2; ++rep) {
        for (int j = 0; j < nout; ++j) {
          hipLaunchKernelGGL(wavg, dim3((uint32_t)chunks), dim3(kT), 0, 0, ar, C, C, logN, L, dtc, dwl, outs[j]);
          CK(hipEventRecord(e0, 0));
          for (int w = 0; w < 3; ++w)
            hipLaunchKernelGGL(wavg, dim3((uint32_t)chunks), dim3(kT), 0, 0, ar, C, C, logN, L, dtc, dwl, outs[j]);
          CK(hipEventRecord(e1, 0));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          printf(" %.3f", ms / 3);
        }
        printf(rep ? "\n" : "  |");
      }
      fflush(stdout);
      for (auto& o : outs) CK(hipFree(o));
      CK(hipFree(ar));
    }
    return 0;
  }
  for (int a = 0; a < allocs; ++a) {
    uint64_t *arA, *outA, *arB;
    CK(hipMalloc(&arA, chunks * C * kPB * 8));
    CK(hipMalloc(&outA, words * 8));
    CK(hipMalloc(&arB, chunks * (C + 1) * kPB * 8));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, arA, chunks * C * kPB, qs[1]);
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, arB, chunks * (C + 1) * kPB, qs[1]);
    CK(hipDeviceSynchronize());
    std::vector<float> tA, tB;
    for (int rep = 0; rep < 8; ++rep) {
      for (int v = 0; v < 2; ++v) {
        for (int w = 0; w < 2; ++w) {  // warm
          if (v == 0)
            hipLaunchKernelGGL(wavg, dim3((uint32_t)chunks), dim3(kT), 0, 0, arA, C, C, logN, L, dtc, dwl, outA);
          else
            hipLaunchKernelGGL(wavg, dim3((uint32_t)chunks), dim3(kT), 0, 0, arB, C, C + 1, logN, L, dtc, dwl,
                               (uint64_t*)nullptr);
        }
        CK(hipEventRecord(e0, 0));
        for (int w = 0; w < 5; ++w) {
          if (v == 0)
            hipLaunchKernelGGL(wavg, dim3((uint32_t)chunks), dim3(kT), 0, 0, arA, C, C, logN, L, dtc, dwl, outA);
          else
            hipLaunchKernelGGL(wavg, dim3((uint32_t)chunks), dim3(kT), 0, 0, arB, C, C + 1, logN, L, dtc, dwl,
                               (uint64_t*)nullptr);
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        (v == 0 ? tA : tB).push_back(ms / 5);
      }
    }
    std::sort(tA.begin(), tA.end());
    std::sort(tB.begin(), tB.end());
    printf("alloc %d: separate out %.3f ms (%.2f TB/s)   in-arena out %.3f ms (%.2f TB/s)\n", a, tA[4],
           bytes / tA[4] / 1e9, tB[4], bytes / tB[4] / 1e9);
    fflush(stdout);
    CK(hipFree(arA));
    CK(hipFree(outA));
    CK(hipFree(arB));
  }
  return 0;
}

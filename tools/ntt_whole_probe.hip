// Round 6 probe: a whole-polynomial forward NTT at 2^15 -- one 1024-thread
// workgroup per polynomial, 32 residues per thread in registers, no HBM round trip between the
// column stages and the block stages -- to A/B against the library's two-pass NTT (columns pass +
// 2^11 blocks pass through HBM, launch_ntt) and against the per-NTT cost inside encrypt.
// Not product code: built into tools/ntt_whole_probe.so by tools/ntt_whole_ab.py's recipe and
// loaded only by that script.
//
// Layouts (j = coefficient index, T = thread, w = wave, l = lane, m = register 0..31):
//   columns  j = T + 1024 m                              stages 0..4  (half-sizes 2^14 .. 2^10)
//   X        j = 2048 w + (l & 31) + 32 m + 1024 (l >> 5)  stages 5..9  (2^9 .. 2^5)
//   Y        j = 2048 w + 32 l + m                        stages 10..14 (2^4 .. 2^0)
// columns -> X is a workgroup transpose through LDS, X -> Y stays inside each wave's 2048
// residues (wave_lds_sync only).  LDS holds one 32-bit half of the polynomial at a time
// (32 K words + 1 K padding, address j + (j >> 5): both transposes are bank-conflict-free).
// Twiddles: psi_rev[2^s + g] with its Shoup companion, g = j >> (15 - s) of the pair's first
// element; wave-uniform in the columns stages, per half-wave in X, per lane in Y.
#include "../fhe-fed_amd/csrc/dev_common.h"

using namespace shelfi;

namespace {

constexpr uint32_t kN = 1u << 15;
constexpr uint32_t kLds = kN + (kN >> 5);

__device__ __forceinline__ uint32_t pad(uint32_t j) { return j + (j >> 5); }

struct TowerQ {
  uint64_t q, n8q, one_sh, pad_;
};

// An opaque zero that exists only once v does: a load indexed with it cannot be issued before v
// is computed (twiddle loads hoisted to the top of a phase take 4 VGPRs each under the 128 cap).
__device__ __forceinline__ int after(uint64_t v) {
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z) : "v"((uint32_t)v));
  return z;
}

// the stage of half-size HALF (in registers) over x; twiddle of group grp = twf(grp).  Group
// grp + 1's twiddle is requested once group grp - 1 is done (one group of prefetch).
template <int HALF, bool RED, class TWF>
__device__ __forceinline__ void reg_stage(uint64_t (&x)[32], TWF twf, uint64_t q, uint64_t n8q) {
  constexpr int G = 32 / (2 * HALF);
  ulonglong2 Wc = twf(after(x[0]));
#pragma unroll
  for (int grp = 0; grp < G; ++grp) {
    ulonglong2 Wn = Wc;
    if (grp + 1 < G) Wn = twf(grp + 1 + after(x[grp > 0 ? (grp - 1) * 2 * HALF : 0]));
#pragma unroll
    for (int i = 0; i < HALF; ++i) {
      const int m0 = grp * 2 * HALF + i;
      ct_bfly_s<RED>(x[m0], x[m0 + HALF], Wc.x, Wc.y, q, n8q);
    }
    Wc = Wn;
  }
}

template <bool NR>
__device__ __forceinline__ constexpr bool red_at(int s) {
  return NR ? false : fwd_red_at(s);
}

// x[m] from address P(m) to address Q(m) through LDS, low halves then high halves
template <bool WG, class PF, class QF>
__device__ __forceinline__ void exchange(uint64_t (&x)[32], uint32_t* __restrict__ lds, PF P, QF Qf) {
#pragma unroll
  for (int part = 0; part < 2; ++part) {
#pragma unroll
    for (int m = 0; m < 32; ++m) lds[P(m)] = part ? (uint32_t)(x[m] >> 32) : (uint32_t)x[m];
    if (WG)
      __syncthreads();
    else
      wave_lds_sync();
#pragma unroll
    for (int m = 0; m < 32; ++m) {
      const uint32_t v = lds[Qf(m)];
      x[m] = part ? ((x[m] & 0xffffffffull) | ((uint64_t)v << 32)) : ((x[m] & ~0xffffffffull) | v);
    }
    if (WG)
      __syncthreads();
    else
      wave_lds_sync();
  }
}

template <bool NR>
__device__ __forceinline__ void ntt_body(uint64_t* __restrict__ a, const ulonglong2* __restrict__ tw, const TowerQ& c,
                                         uint32_t* __restrict__ lds) {
  const uint32_t T = threadIdx.x, w = T >> 6, l = T & 63, hb = l >> 5;
  const uint64_t q = c.q, n8q = c.n8q;
  uint64_t x[32];
#pragma unroll
  for (int m = 0; m < 32; ++m) x[m] = a[T + 1024u * m];
  // columns: stages 0..4, wave-uniform twiddles psi_rev[2^s + (m >> (5 - s))]
  reg_stage<16, red_at<NR>(0)>(x, [&](int g) { return tw[1 + g]; }, q, n8q);
  reg_stage<8, red_at<NR>(1)>(x, [&](int g) { return tw[2 + g]; }, q, n8q);
  reg_stage<4, red_at<NR>(2)>(x, [&](int g) { return tw[4 + g]; }, q, n8q);
  reg_stage<2, red_at<NR>(3)>(x, [&](int g) { return tw[8 + g]; }, q, n8q);
  reg_stage<1, red_at<NR>(4)>(x, [&](int g) { return tw[16 + g]; }, q, n8q);
  // columns -> X (workgroup)
  const uint32_t xb = 2048u * w + (l & 31u) + 1024u * hb;
  exchange<true>(x, lds, [&](int m) { return pad(T + 1024u * m); }, [&](int m) { return pad(xb + 32u * m); });
  // X: stages 5..9, g = 2^(s-4) w + 2^(s-5) hb + (m >> (10 - s))
  reg_stage<16, red_at<NR>(5)>(x, [&](int g) { return tw[32 + 2 * w + hb + g]; }, q, n8q);
  reg_stage<8, red_at<NR>(6)>(x, [&](int g) { return tw[64 + 4 * w + 2 * hb + g]; }, q, n8q);
  reg_stage<4, red_at<NR>(7)>(x, [&](int g) { return tw[128 + 8 * w + 4 * hb + g]; }, q, n8q);
  reg_stage<2, red_at<NR>(8)>(x, [&](int g) { return tw[256 + 16 * w + 8 * hb + g]; }, q, n8q);
  reg_stage<1, red_at<NR>(9)>(x, [&](int g) { return tw[512 + 32 * w + 16 * hb + g]; }, q, n8q);
  // X -> Y (inside the wave's 2048 residues)
  const uint32_t yb = 2048u * w + 32u * l;
  exchange<false>(x, lds, [&](int m) { return pad(xb + 32u * m); }, [&](int m) { return pad(yb + m); });
  // Y: stages 10..14, g = (yb + m) >> (15 - s)
  reg_stage<16, red_at<NR>(10)>(x, [&](int g) { return tw[1024 + (yb >> 5) + g]; }, q, n8q);
  reg_stage<8, red_at<NR>(11)>(x, [&](int g) { return tw[2048 + (yb >> 4) + g]; }, q, n8q);
  reg_stage<4, red_at<NR>(12)>(x, [&](int g) { return tw[4096 + (yb >> 3) + g]; }, q, n8q);
  reg_stage<2, red_at<NR>(13)>(x, [&](int g) { return tw[8192 + (yb >> 2) + g]; }, q, n8q);
  reg_stage<1, red_at<NR>(14)>(x, [&](int g) { return tw[16384 + (yb >> 1) + g]; }, q, n8q);
  ulonglong2* __restrict__ o = reinterpret_cast<ulonglong2*>(a + yb);
#pragma unroll
  for (int m = 0; m < 32; m += 2) o[m / 2] = make_ulonglong2(red64(x[m], q, c.one_sh), red64(x[m + 1], q, c.one_sh));
}

// one workgroup per polynomial of towers [t0, t0 + nt) (poly p = L (b / nt) + t0 + b % nt); NR: every
// tower of the launch is below kNoRedQ (no reductions before the last stage, as encrypt's NORED split)
template <bool NR>
__global__ __launch_bounds__(1024) void ntt_fwd_whole15(uint64_t* __restrict__ polys, uint32_t L, uint32_t t0,
                                                        uint32_t nt, const ulonglong2* __restrict__ tw,
                                                        const TowerQ* __restrict__ tq) {
  __shared__ uint32_t lds[kLds];
  const uint32_t t = t0 + blockIdx.x % nt;
  const uint64_t p = (uint64_t)L * (blockIdx.x / nt) + t;
  const TowerQ c = tq[t];
  ntt_body<NR>(polys + p * kN, tw + (uint64_t)t * kN, c, lds);
}

}  // namespace

// P polynomials [P][2^15] (P a multiple of L, tower p % L), towers [t0, t0 + nt) of each ciphertext
extern "C" int ntt_whole_fwd(uint64_t* polys, uint64_t P, uint32_t L, uint32_t t0, uint32_t nt, int nored,
                             const void* tw, const void* tq, void* stream) {
  if (!P || !nt || P % L || t0 + nt > L) return 1;
  const dim3 grid((uint32_t)(P / L * nt));
  if (nored)
    hipLaunchKernelGGL(ntt_fwd_whole15<true>, grid, dim3(1024), 0, (hipStream_t)stream, polys, L, t0, nt,
                       (const ulonglong2*)tw, (const TowerQ*)tq);
  else
    hipLaunchKernelGGL(ntt_fwd_whole15<false>, grid, dim3(1024), 0, (hipStream_t)stream, polys, L, t0, nt,
                       (const ulonglong2*)tw, (const TowerQ*)tq);
  return (int)hipGetLastError();
}

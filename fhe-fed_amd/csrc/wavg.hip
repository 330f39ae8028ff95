// wavg.hip — the aggregation kernels of the RNS-CKKS path (computeWeightedAverage,
// ckks.cpp:264-320: EvalMult(ct, (float)w) at :286-289 + EvalAdd at :291-297), all HBM-bound:
//   wavg_kernel        separate uint64 learner batches (bytes API, shelfi_dev_wavg)
//   wavg_packed        the resident packed arena (shelfi_dev_wavg_arena, the headline)
//   arena_pack_kernel  a learner's upload into its packed slices + the residue check
//   blob_{un}pack      the packed wire format (C = 1 slices)
//   modq_kernel        fold a collective's uint64 sum of partials back to [0, q)
// Split out of kernels.hip in round 4 (the NTT / FFT / encrypt / decrypt kernels stay there).
#include <hip/hip_runtime.h>

#include <type_traits>

#include "dev_common.h"
#include "shelfi_internal.h"

namespace shelfi {

// ------------------------------------------------------------------ wavg ----
// One thread = 2 adjacent residues (one 16-byte load per learner); one block =
// 512 residues of a single (ct, poly, tower) row, so the tower — and with it
// q and every learner's weight — is block-uniform and lives in SGPRs.  Up to 16
// learners per launch travel in the kernel-argument segment (pointers + weight
// limbs, read with s_load); more learners accumulate over further launches.
//
// Lazy accumulation without carries: x = x1*2^30 + x0 and W = w1*2^30 + w0
// (x, W < q < 2^60, so all four limbs are < 2^30).  Each limb product is < 2^60,
// so 16 of them fit a u64: per learner 4 v_mad_u64_u32 and no reduction.  After
// the (<= 16) learners of a launch the four sums are folded: T = S00 + 2^30 (S01 + S10) +
// 2^60 S11 mod q.  Bit-exact with sum_c (W_c x_c mod q) in any order.
constexpr int kWavgThreads = 256;
constexpr int kWavgPerBlock = 2 * kWavgThreads;

__device__ __forceinline__ uint64_t wavg_fold(uint64_t s00, uint64_t s01, uint64_t s10,
                                              uint64_t s11, const TowerConst& c) {
  uint64_t a = red64(s00, c.q, c.one_shoup);
  uint64_t m = red64(s01, c.q, c.one_shoup) + red64(s10, c.q, c.one_shoup);  // < 2q
  uint64_t b = shoup_mul(m, c.r30, c.r30_shoup, c.q);
  uint64_t d = shoup_mul(red64(s11, c.q, c.one_shoup), c.r60, c.r60_shoup, c.q);
  return addmod(addmod(a, b, c.q), d, c.q);
}

// Separate per-learner batches (ptrs[k] + e): the bytes API's staged uploads and
// shelfi_dev_wavg.  The aggregator's resident layout is the packed arena below.
// CHECK (the bytes API, whose inputs are untrusted learner uploads): also flag any input
// residue >= q_t in *a.bad (the carry-free limb sums assume canonical residues).
// R rows per block (R = 2 for C <= 8 learners): with few learners one 512-residue row gives
// a thread only C 16-byte loads in flight; two adjacent rows (same tower: N / 512 is even)
// double that.
// UNR learners' loads in flight per thread (8 / R; all 16 in flight measured no faster, round 4).
template <bool CHECK = false, int R = 1, int UNR = 8 / R>
__global__ __launch_bounds__(kWavgThreads) void wavg_kernel(WavgArgs a,
                                                            const TowerConst* __restrict__ tcs) {
  const uint64_t row0 = (uint64_t)blockIdx.x * R;
  const uint64_t base = row0 * kWavgPerBlock;
  const uint32_t t = (uint32_t)((base >> a.logN) % a.L);  // block-uniform tower
  const TowerConst c = tcs[t];
  const uint32_t M30 = (1u << 30) - 1;

  uint64_t s[R][8];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) s[i][j] = 0;
  bool bad = false;
#pragma unroll UNR
  for (uint32_t k = 0; k < a.C; ++k) {
    const uint64_t* __restrict__ p = a.ptrs[k] + base + 2u * threadIdx.x;
    const uint32_t w0 = a.wl[k][t][0], w1 = a.wl[k][t][1];
    u32x4 v[R];
#pragma unroll
    for (int i = 0; i < R; ++i) v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + i * kWavgPerBlock));
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if (CHECK)
        bad |= (((uint64_t)v[i].y << 32) | v[i].x) >= c.q || (((uint64_t)v[i].w << 32) | v[i].z) >= c.q;
      // element a: (v.x, v.y), element b: (v.z, v.w); 30-bit limbs
      const uint32_t xa0 = v[i].x & M30, xa1 = (v[i].x >> 30) | (v[i].y << 2);
      const uint32_t xb0 = v[i].z & M30, xb1 = (v[i].z >> 30) | (v[i].w << 2);
      s[i][0] += (uint64_t)xa0 * w0;
      s[i][1] += (uint64_t)xa0 * w1;
      s[i][2] += (uint64_t)xa1 * w0;
      s[i][3] += (uint64_t)xa1 * w1;
      s[i][4] += (uint64_t)xb0 * w0;
      s[i][5] += (uint64_t)xb0 * w1;
      s[i][6] += (uint64_t)xb1 * w0;
      s[i][7] += (uint64_t)xb1 * w1;
    }
  }
  if (CHECK && bad) atomicOr(a.bad, 1u);
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const uint64_t e = base + (uint64_t)i * kWavgPerBlock + 2u * threadIdx.x;
    uint64_t r0 = wavg_fold(s[i][0], s[i][1], s[i][2], s[i][3], c);
    uint64_t r1 = wavg_fold(s[i][4], s[i][5], s[i][6], s[i][7], c);
    if (a.accumulate) {  // learners beyond the first 16: fold into the running sum
      const u32x4 o = *reinterpret_cast<const u32x4*>(a.out + e);
      r0 = addmod(r0, (uint64_t)o.x | ((uint64_t)o.y << 32), c.q);
      r1 = addmod(r1, (uint64_t)o.z | ((uint64_t)o.w << 32), c.q);
    }
    u32x4 o;
    o.x = (uint32_t)r0;
    o.y = (uint32_t)(r0 >> 32);
    o.z = (uint32_t)r1;
    o.w = (uint32_t)(r1 >> 32);
    __builtin_nontemporal_store(o, reinterpret_cast<u32x4*>(a.out + e));
  }
}

// ------------------------------------------------------------ packed arena ----
// The aggregator's resident layout (round 3; ArenaPack in shelfi_internal.h).  A residue of
// tower t carries bitlength(q_t) bits of information; storing it in 64 wastes 4 of them for the
// 60-bit q_0 and 11-12 for the 52/53-bit towers of the reference parameters (ckks.cpp:26-33:
// scaleFactorBits 52, first modulus 60).  wavg is HBM-bound and reads every learner's residues
// once, so the arena keeps tower t at U_t = bitlength(q_t) bits when that is 1 mod 4 (a field of
// B_t = U_t - 1 bits plus one top bit in a flag plane) and at U_t = B_t = 4 ceil(bitlength / 4)
// otherwise (at least 32).  At 2^15 / L4 (60, 53, 52, 53 bits) a client ciphertext is 218 / 256
// of its uint64 size, and the launch moves 16 x 218 + 256 instead of 17 x 256 bits per
// coefficient (the aggregate is written as uint64 [K][2][L][N] for decrypt and the collectives).
//
// Geometry: rows of 512 residues (one (ct, poly, tower) polynomial has N / 512 rows) in the
// natural [K][2][L][N] order; a row holds C learner slices side by side; a slice is 512 U_t bits
// = 16 U_t dwords.  One wave handles one row: lane l owns the 8 residues 2l + (j & 1) + 128 (j >> 1),
// j < 8 — so the uint64 output of a row is 4 coalesced 16-byte stores per lane — and their low
// B_t bits, concatenated low bit first, are B_t / 4 dwords d = 0 .. D-1 stored as planes: d < 4 N4
// in N4 16-byte planes (plane p: lane l's dwords 4p .. 4p+3 at dword p 256 + 4 l of the slice),
// then an 8-byte plane (if D mod 4 >= 2) and a 4-byte plane (if D is odd); with a flag plane, byte
// 64 B_t + l of the slice holds bit B_t of lane l's 8 residues.  Every plane access is one
// contiguous wave access.
template <int UB>
struct PackShape {
  static constexpr int B = UB & ~3, F = UB & 3;   // field bits, flag plane (0 / 1)
  static_assert(F <= 1 && B >= 32 && UB <= 60, "packed width");
  static constexpr int D = B / 4;                 // field dwords per lane (8 residues)
  static constexpr int N4 = D / 4;                // 16-byte planes
  static constexpr int H2 = (D % 4) >= 2 ? 1 : 0; // an 8-byte plane
  static constexpr int H1 = D & 1;                // a 4-byte plane
  static constexpr int O2 = N4 * 256, O1 = O2 + H2 * 128;
  static constexpr int OF = 64 * B;               // flag plane (bytes)
  static constexpr int SLICE = 16 * UB;           // dwords per learner slice
};
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

template <int UB>
__device__ __forceinline__ void pk_load(const uint32_t* __restrict__ sl, uint32_t lane,
                                        uint32_t (&w)[PackShape<UB>::D], uint32_t& fl) {
  using S = PackShape<UB>;
#pragma unroll
  for (int p = 0; p < S::N4; ++p) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sl + p * 256 + 4 * lane));
    w[4 * p] = v.x;
    w[4 * p + 1] = v.y;
    w[4 * p + 2] = v.z;
    w[4 * p + 3] = v.w;
  }
  if (S::H2) {
    const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(sl + S::O2 + 2 * lane));
    w[4 * S::N4] = v.x;
    w[4 * S::N4 + 1] = v.y;
  }
  if (S::H1) w[S::D - 1] = __builtin_nontemporal_load(sl + S::O1 + lane);
  fl = S::F ? (uint32_t)__builtin_nontemporal_load(reinterpret_cast<const uint8_t*>(sl) + S::OF + lane) : 0u;
}
template <int UB>
__device__ __forceinline__ void pk_store(uint32_t* __restrict__ sl, uint32_t lane,
                                         const uint32_t (&w)[PackShape<UB>::D], uint32_t fl) {
  using S = PackShape<UB>;
#pragma unroll
  for (int p = 0; p < S::N4; ++p) {
    u32x4 v;
    v.x = w[4 * p];
    v.y = w[4 * p + 1];
    v.z = w[4 * p + 2];
    v.w = w[4 * p + 3];
    *reinterpret_cast<u32x4*>(sl + p * 256 + 4 * lane) = v;
  }
  if (S::H2) {
    u32x2 v;
    v.x = w[4 * S::N4];
    v.y = w[4 * S::N4 + 1];
    *reinterpret_cast<u32x2*>(sl + S::O2 + 2 * lane) = v;
  }
  if (S::H1) sl[S::O1 + lane] = w[S::D - 1];
  if (S::F) reinterpret_cast<uint8_t*>(sl)[S::OF + lane] = (uint8_t)fl;
}
// Bits [o, o + nb) of a lane's field stream (o, nb compile-time after unrolling, nb <= 30):
// one v_bfe_u32 inside a dword, v_alignbit_b32 + mask across two.
template <int D>
__device__ __forceinline__ uint32_t pk_bits(const uint32_t (&w)[D], int o, int nb) {
  const int i = o >> 5, s = o & 31;
  const uint32_t m = (1u << nb) - 1;
  if (s + nb <= 32) return (w[i] >> s) & m;
  return __builtin_amdgcn_alignbit(w[i + 1], w[i], (uint32_t)s) & m;
}

// The 8 residues x[j] of a lane (< 2^(B+1), canonical) as its slice words: the low B bits
// concatenated low bit first, bit B into the flag byte (kept only with a flag plane).
template <int UB>
__device__ __forceinline__ void pk_pack(const uint64_t (&x)[8], uint32_t (&w)[PackShape<UB>::D], uint32_t& fl) {
  using S = PackShape<UB>;
  constexpr int B = S::B;
  fl = 0;
#pragma unroll
  for (int d = 0; d < S::D; ++d) w[d] = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint64_t v = x[j] & ((1ull << B) - 1);
    fl |= (uint32_t)((x[j] >> B) & 1) << j;
    const int o = j * B, i = o >> 5, sh = o & 31;
    w[i] |= (uint32_t)(v << sh);
    if (sh + B > 32) w[i + 1] |= (uint32_t)(v >> (32 - sh));
    if (sh + B > 64) w[i + 2] |= (uint32_t)(v >> (64 - sh));
  }
}

// Row geometry of a packed arena, wave-uniform: the row's learner-0 slice (dwords from the
// arena base), its tower and width U_t.
struct PackedRow {
  uint64_t base;
  uint32_t t, U;
};
__device__ __forceinline__ PackedRow packed_row(uint64_t r, uint32_t C, uint32_t L, uint32_t logN,
                                                const ArenaPack& ap) {
  const uint32_t lr = logN - 9;  // rows per tower polynomial: N / 512
  const uint64_t tp = r >> lr;   // (ct, poly, tower) index
  const uint32_t t = (uint32_t)(tp % L);
  const uint64_t g = tp / L;     // (ct, poly) index
  const uint32_t chunk = (uint32_t)(r & ((1u << lr) - 1));
  const uint32_t U = ap.w[t];
  const uint64_t base = 16ull * C * (((g * ap.sum + ap.pre[t]) << lr) + (uint64_t)chunk * U);
  return {base, t, U};
}
// One instantiation per width class (a wave-uniform switch on U_t)
#define SHELFI_PACK_WIDTHS(X) \
  X(32) X(33) X(36) X(37) X(40) X(41) X(44) X(45) X(48) X(49) X(52) X(53) X(56) X(57) X(60)

// One wave = one row: sum_c W_c x_c mod q_t over the row's C learner slices, stored as the row's
// uint64 output o (lane l's residues 2l + (j & 1) + 128 (j >> 1), 4 coalesced 16-byte stores).
//
// Three carry-free accumulators per residue (round 4; four in round 3): with x = x1 2^30 + x0 and
// W = w1 2^30 + w0, S0 = sum x0 w0, Sm = sum (x0 w1 + x1 w0) and S1 = sum x1 w1, folded as
// S0 + 2^30 Sm + 2^60 S1 mod q.  x0, w0 < 2^30 and x1, w1 < 2^(b - 30) for a b-bit modulus, so a
// learner adds < 2^60 to S0 and < 2^(b+1) to Sm: G = 16 learners fit 64 bits up to b = 59, and the
// 60-bit width class (b <= 60) folds every G = 8.  The 8 residues' accumulators drop from 64 to 48
// VGPRs, and the running sum over groups (C > G) lives in LDS instead of 16 more VGPRs: 5 waves per
// SIMD instead of 3 (the launch's bytes in flight, which small launches -- cfg2's 2,048 rows --
// are short of).
template <int UB>
constexpr int pack_group() { return UB <= 57 ? 16 : 8; }

__device__ __forceinline__ uint64_t wavg_fold3(uint64_t s0, uint64_t sm, uint64_t s1, const TowerConst& c) {
  const uint64_t a = red64(s0, c.q, c.one_shoup);
  const uint64_t b = shoup_mul(red64(sm, c.q, c.one_shoup), c.r30, c.r30_shoup, c.q);
  const uint64_t d = shoup_mul(red64(s1, c.q, c.one_shoup), c.r60, c.r60_shoup, c.q);
  return addmod(addmod(a, b, c.q), d, c.q);
}

// Learner k's slice of the row sits `step` dwords after learner 0's: S::SLICE in an arena (the C
// slices side by side), or a caller's stride between stacked C = 1 batches (STK: the packed share
// exchange's sum_packed).  Learners [kbeg, kend) are summed; the row's 8 residues per lane come
// back in x (canonical; zero for an empty range).
template <int UB, int UR, bool STK>
__device__ __forceinline__ void wavg_packed_row(const uint32_t* __restrict__ sl, uint32_t kbeg, uint32_t kend,
                                                uint64_t lstride, const uint32_t* __restrict__ wlt,
                                                uint32_t wl_stride, const TowerConst& c, uint32_t lane,
                                                uint64_t* __restrict__ run, uint64_t (&x)[8]) {
  using S = PackShape<UB>;
  constexpr int B = S::B, G = pack_group<UB>();
  const uint64_t step = STK ? lstride : (uint64_t)S::SLICE;
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = 0;
  for (uint32_t k0 = kbeg; k0 < kend; k0 += G) {
    const uint32_t k1 = min(kend, k0 + (uint32_t)G);
    uint64_t s0[8], sm[8], s1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s0[j] = sm[j] = s1[j] = 0;
#pragma unroll UR
    for (uint32_t k = k0; k < k1; ++k) {
      uint32_t w[S::D], fl;
      pk_load<UB>(sl + (uint64_t)k * step, lane, w, fl);
      const uint32_t w0 = wlt[k * wl_stride], w1 = wlt[k * wl_stride + 1];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t x0 = pk_bits(w, j * B, 30);
        uint32_t x1 = pk_bits(w, j * B + 30, B - 30);
        if (S::F) x1 |= ((fl >> j) & 1u) << (B - 30);  // bit B of the residue (< 2^(B+1) <= 2^57)
        s0[j] += (uint64_t)x0 * w0;
        sm[j] += (uint64_t)x0 * w1;
        sm[j] += (uint64_t)x1 * w0;
        s1[j] += (uint64_t)x1 * w1;
      }
    }
    const bool first = k0 == kbeg, last = k1 >= kend;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      uint64_t r = wavg_fold3(s0[j], sm[j], s1[j], c);
      if (!first) r = addmod(r, run[64 * j + lane], c.q);
      if (last) x[j] = r;
      else run[64 * j + lane] = r;
    }
  }
}

// A row's 8 residues per lane as uint64 (4 coalesced 16-byte non-temporal stores per lane).
__device__ __forceinline__ void store_row_u64(uint64_t* __restrict__ o, uint32_t lane, const uint64_t (&x)[8]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    u32x4 v;
    v.x = (uint32_t)x[2 * g];
    v.y = (uint32_t)(x[2 * g] >> 32);
    v.z = (uint32_t)x[2 * g + 1];
    v.w = (uint32_t)(x[2 * g + 1] >> 32);
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(o + 128 * g + 2 * lane));
  }
}

constexpr int kPackedWaves = 4;  // waves per block, one row each

// crow: the learner count of the input's row layout (C for an arena, 1 for stacked C = 1 batches
// lstride dwords apart); out (uint64) or, with PO, pout (packed, C = 1 layout) receives the result.
// (Round 4 also measured two waves per row for small launches and an XCD-contiguous block order:
// within +-1% and 8% slower; both were removed in round 5.)
template <int UR, int WV = kPackedWaves, bool PO = false, bool STK = false>
__global__ __launch_bounds__(64 * WV) void wavg_packed(const uint32_t* __restrict__ arena,
                                                      const uint32_t* __restrict__ wl, uint32_t C, uint32_t crow,
                                                      uint64_t lstride, uint64_t rows, uint32_t L, uint32_t logN,
                                                      ArenaPack ap, const TowerConst* __restrict__ tcs,
                                                      uint64_t* __restrict__ out, uint32_t* __restrict__ pout,
                                                      uint32_t strands, uint32_t nblocks) {
  // the running sum of the rows' residues across learner groups (C > 16): 8 x 64 per wave
  __shared__ uint64_t run_lds[WV][8 * 64];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // strands > 1 (probe): dispatch order interleaves `strands` contiguous runs of blocks spread over
  // the buffers (block b -> (b mod strands) * per + b / strands), so the blocks in flight read and
  // write `strands` separate windows of the arena and the output instead of one
  uint32_t bi = blockIdx.x;
  if (strands > 1) {
    const uint32_t per = (nblocks + strands - 1) / strands;
    bi = (bi % strands) * per + bi / strands;
    if (bi >= nblocks) return;
  }
  const uint64_t r = (uint64_t)bi * WV + wave;
  if (r >= rows) return;
  const uint32_t lane = threadIdx.x & 63;
  uint64_t x[8];
  const PackedRow pr = packed_row(r, crow, L, logN, ap);
  const TowerConst c = tcs[pr.t];
  const uint32_t* __restrict__ sl = arena + pr.base;
  const uint32_t* __restrict__ wlt = wl + 2 * pr.t;
  uint32_t* __restrict__ po = PO ? pout + packed_row(r, 1, L, logN, ap).base : nullptr;
  switch (pr.U) {
#define WPR(UU)                                                                               \
  case UU:                                                                                    \
    wavg_packed_row<UU, UR, STK>(sl, 0u, C, lstride, wlt, 2 * L, c, lane, run_lds[wave], x);  \
    if (PO) {                                                                                 \
      uint32_t pw[PackShape<UU>::D], pf;                                                      \
      pk_pack<UU>(x, pw, pf);                                                                 \
      pk_store<UU>(po, lane, pw, pf);                                                         \
    }                                                                                         \
    break;
    SHELFI_PACK_WIDTHS(WPR)
#undef WPR
    default:
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = 0;
      break;
  }
  if (!PO) store_row_u64(out + r * kArenaChunk, lane, x);
}

// Round 3's form (four accumulators, running sum in registers; 134-145 VGPRs, 3 waves per SIMD),
// kept as the A/B reference for wavg_packed (SHELFI_PACK_KERNEL=r3, read per launch).
// One wave = one row: sum_c W_c x_c mod q_t over the row's C learner slices (carry-free limb sums
// per group of 16 learners, as wavg_kernel), into r[8] (lane l's residues 2l + (j & 1) + 128 (j >> 1)).
template <int UB, int UR>
__device__ __forceinline__ void wavg_packed_row_r3(const uint32_t* __restrict__ sl, uint32_t C,
                                                const uint32_t* __restrict__ wlt,
                                                uint32_t wl_stride, const TowerConst& c, uint32_t lane,
                                                uint64_t (&r)[8]) {
  using S = PackShape<UB>;
  constexpr int B = S::B;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = 0;
  for (uint32_t k0 = 0; k0 < C; k0 += kWavgMaxLearners) {
    const uint32_t k1 = min(C, k0 + (uint32_t)kWavgMaxLearners);
    uint64_t s[8][4];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) s[j][i] = 0;
#pragma unroll UR
    for (uint32_t k = k0; k < k1; ++k) {
      uint32_t w[S::D], fl;
      pk_load<UB>(sl + (uint64_t)k * S::SLICE, lane, w, fl);
      const uint32_t w0 = wlt[k * wl_stride], w1 = wlt[k * wl_stride + 1];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t x0 = pk_bits(w, j * B, 30);
        uint32_t x1 = pk_bits(w, j * B + 30, B - 30);
        if (S::F) x1 |= ((fl >> j) & 1u) << (B - 30);  // bit B of the residue (< 2^(B+1) <= 2^57)
        s[j][0] += (uint64_t)x0 * w0;
        s[j][1] += (uint64_t)x0 * w1;
        s[j][2] += (uint64_t)x1 * w0;
        s[j][3] += (uint64_t)x1 * w1;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = addmod(r[j], wavg_fold(s[j][0], s[j][1], s[j][2], s[j][3], c), c.q);
  }
}


template <int UR, int WV = kPackedWaves>
__global__ __launch_bounds__(64 * WV) void wavg_packed_r3(const uint32_t* __restrict__ arena,
                                                      const uint32_t* __restrict__ wl, uint32_t C,
                                                      uint64_t rows, uint32_t L, uint32_t logN, ArenaPack ap,
                                                      const TowerConst* __restrict__ tcs,
                                                      uint64_t* __restrict__ out) {
  const uint64_t r = (uint64_t)blockIdx.x * WV + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (r >= rows) return;
  const uint32_t lane = threadIdx.x & 63;
  const PackedRow pr = packed_row(r, C, L, logN, ap);
  const TowerConst c = tcs[pr.t];
  const uint32_t* __restrict__ sl = arena + pr.base;
  const uint32_t* __restrict__ wlt = wl + 2 * pr.t;
  uint64_t res[8];
  switch (pr.U) {
#define WPR(UU) \
  case UU: wavg_packed_row_r3<UU, UR>(sl, C, wlt, 2 * L, c, lane, res); break;
    SHELFI_PACK_WIDTHS(WPR)
#undef WPR
    default:
#pragma unroll
      for (int j = 0; j < 8; ++j) res[j] = 0;
      break;
  }
  uint64_t* __restrict__ o = out + r * kArenaChunk;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    u32x4 v;
    v.x = (uint32_t)res[2 * g];
    v.y = (uint32_t)(res[2 * g] >> 32);
    v.z = (uint32_t)res[2 * g + 1];
    v.w = (uint32_t)(res[2 * g + 1] >> 32);
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(o + 128 * g + 2 * lane));
  }
}

// Upload of one learner's rows into its packed slices, with the canonical-residue check of
// every residue (the limb sums above assume x < q_t; a refused slot is never aggregated).
template <int UB>
__device__ __forceinline__ bool pack_row(const uint64_t* __restrict__ src, uint32_t* __restrict__ sl, uint64_t q,
                                         uint32_t lane) {
  using S = PackShape<UB>;
  uint64_t x[8];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + 128 * g + 2 * lane));
    x[2 * g] = ((uint64_t)v.y << 32) | v.x;
    x[2 * g + 1] = ((uint64_t)v.w << 32) | v.z;
  }
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 8; ++j) bad |= x[j] >= q;  // (x >= 2^(B+1) > q without a flag plane: refused)
  uint32_t w[S::D], fl;
  pk_pack<UB>(x, w, fl);
  pk_store<UB>(sl, lane, w, fl);
  return bad;
}

__global__ __launch_bounds__(64 * kPackedWaves) void arena_pack_kernel(
    const uint64_t* __restrict__ src, uint64_t row0, uint64_t rows, uint32_t C, uint32_t learner, uint32_t L,
    uint32_t logN, ArenaPack ap, const TowerConst* __restrict__ tcs, uint32_t* __restrict__ arena,
    uint32_t* __restrict__ bad) {
  const uint64_t i = (uint64_t)blockIdx.x * kPackedWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (i >= rows) return;
  const uint32_t lane = threadIdx.x & 63;
  const PackedRow pr = packed_row(row0 + i, C, L, logN, ap);
  const uint64_t q = tcs[pr.t].q;
  const uint64_t* __restrict__ s = src + i * kArenaChunk;
  uint32_t* __restrict__ sl = arena + pr.base + (uint64_t)learner * 16 * pr.U;
  bool b = false;
  switch (pr.U) {
#define PKR(UU) \
  case UU: b = pack_row<UU>(s, sl, q, lane); break;
    SHELFI_PACK_WIDTHS(PKR)
#undef PKR
    default: b = true; break;
  }
  if (b) atomicOr(bad, 1u);
}

void launch_wavg_packed_ex(const uint32_t* in, const uint32_t* wl_dev, uint32_t C, uint32_t crow, uint64_t lstride,
                           uint64_t rows, uint32_t L, uint32_t logN, const ArenaPack& ap, const TowerConst* tc,
                           uint64_t* out, uint32_t* pout, hipStream_t s) {
  const uint64_t nrows = (rows << logN) / kArenaChunk;
  if (!nrows) return;
  if (nrows > 0xFFFFFFFFull) throw Error{SHELFI_ERR_ARG, "aggregation batch too large"};
  const bool po = pout != nullptr, stk = lstride != 0;
  // A/B probe switches (Switches; profiles/probes/r03_wavg_packed_ab.txt, profiles/r04a/probes/):
  // learners unrolled per iteration SHELFI_PACK_UNROLL=1|2|4|8, waves (rows) per block
  // SHELFI_PACK_WAVES=2|8, the kernel SHELFI_PACK_KERNEL=r3|v4 (the packed-output and stacked forms
  // always use v4).  Without switches the launch picks by shape from the same-process A/Bs
  // (profiles/r04a/probes/wavg_kernel_ab.txt, r04d/): see auto_v4.
  const Switches& sw = switches();
  const bool forced = sw.pack_kernel || sw.pack_unroll || sw.pack_waves;
  const int wv = sw.pack_waves ? sw.pack_waves : kPackedWaves;
  const int u = sw.pack_unroll ? sw.pack_unroll : (!forced && C == 16 && nrows >= 16384 ? 8 : 2);
  // default: v4 with 8 learners in flight for 16-learner arenas of >= 16384 rows (cfg3's per-GPU
  // shard, cfg4: +0.6-1.4% over r3 in the same-process A/B), round 3's kernel otherwise (cfg5's 8,
  // the cts-sharded 128 learners, and small grids, where it leads by 1-4%)
  const bool auto_v4 = !forced && C == 16 && nrows >= 16384;
  const bool v4 = po || stk || auto_v4 || sw.pack_kernel == 4;
  const int wvs = (wv == 2 || wv == 8) && u == 2 && !po && !stk ? wv : kPackedWaves;
  if (!v4) {
    const uint64_t blocks = (nrows + wvs - 1) / wvs;
    if (blocks > 0x7FFFFFFFull) throw Error{SHELFI_ERR_ARG, "aggregation batch too large"};
#define WPK3(UU, WW)                                                                                         \
  hipLaunchKernelGGL((wavg_packed_r3<UU, WW>), dim3((uint32_t)blocks), dim3(64 * WW), 0, s, in, wl_dev, C, nrows, \
                     L, logN, ap, tc, out)
    if (wvs == 2)
      WPK3(2, 2);
    else if (wvs == 8)
      WPK3(2, 8);
    else if (u == 1)
      WPK3(1, 4);
    else if (u == 4)
      WPK3(4, 4);
    else
      WPK3(2, 4);
#undef WPK3
    SHELFI_HIP(hipGetLastError());
    return;
  }
  const uint64_t blocks = (nrows + wvs - 1) / wvs;
  if (blocks > 0x7FFFFFFFull) throw Error{SHELFI_ERR_ARG, "aggregation batch too large"};
  const uint32_t strands = sw.wavg_strands > 1 && blocks >= 4ull * sw.wavg_strands ? sw.wavg_strands : 0;
  const uint64_t grid = strands ? (blocks + strands - 1) / strands * strands : blocks;
#define WPK(UU, WW, PO, STK)                                                                                 \
  hipLaunchKernelGGL((wavg_packed<UU, WW, PO, STK>), dim3((uint32_t)grid), dim3(64 * WW), 0, s, in, wl_dev,    \
                     C, crow, lstride, nrows, L, logN, ap, tc, out, pout, strands, (uint32_t)blocks)
  if (stk && po)
    throw Error{SHELFI_ERR_ARG, "stacked inputs with a packed output"};
  else if (stk)
    WPK(2, 4, false, true);
  else if (po)
    WPK(2, 4, true, false);
  else if (wvs == 2)
    WPK(2, 2, false, false);
  else if (wvs == 8)
    WPK(2, 8, false, false);
  else if (u == 1)
    WPK(1, 4, false, false);
  else if (u == 4)
    WPK(4, 4, false, false);
  else if (u == 8)
    WPK(8, 4, false, false);
  else
    WPK(2, 4, false, false);
#undef WPK
  SHELFI_HIP(hipGetLastError());
}

void launch_wavg_packed(const uint64_t* arena, const uint32_t* wl_dev, uint32_t C, uint64_t rows, uint32_t L,
                        uint32_t logN, const ArenaPack& ap, const TowerConst* tc, uint64_t* out, hipStream_t s) {
  launch_wavg_packed_ex(reinterpret_cast<const uint32_t*>(arena), wl_dev, C, C, 0, rows, L, logN, ap, tc, out,
                        nullptr, s);
}

void launch_arena_pack(const uint64_t* src, uint64_t row0, uint64_t rows, uint32_t C, uint32_t learner,
                       uint32_t L, uint32_t logN, const ArenaPack& ap, const TowerConst* tc, uint64_t* arena,
                       uint32_t* bad, hipStream_t s) {
  if (!rows) return;
  const uint64_t blocks = (rows + kPackedWaves - 1) / kPackedWaves;
  if (blocks > 0x7FFFFFFFull) throw Error{SHELFI_ERR_ARG, "arena too large"};
  hipLaunchKernelGGL(arena_pack_kernel, dim3((uint32_t)blocks), dim3(64 * kPackedWaves), 0, s, src, row0,
                     rows, C, learner, L, logN, ap, tc, reinterpret_cast<uint32_t*>(arena), bad);
  SHELFI_HIP(hipGetLastError());
}

// ------------------------------------------------------- packed wire blobs ----
// A packed library blob (wire format "packed", shelfi_set_wire_format 2) carries its payload in the
// arena's slice format with C = 1: ciphertexts [k0, k0 + kn) of a blob are kn consecutive
// (ct, poly) groups, so a chunk packs / unpacks with row indices relative to its first ciphertext.
template <int UB>
__device__ __forceinline__ void unpack_row(const uint32_t* __restrict__ sl, uint64_t* __restrict__ dst,
                                           uint32_t lane) {
  using S = PackShape<UB>;
  constexpr int B = S::B;
  uint32_t w[S::D], fl;
  pk_load<UB>(sl, lane, w, fl);
  uint64_t x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int o = j * B, i = o >> 5, s = o & 31;
    uint64_t v = (uint64_t)w[i] >> s;
    if (s + B > 32) v |= (uint64_t)w[i + 1] << (32 - s);
    if (s + B > 64) v |= (uint64_t)w[i + 2] << (64 - s);
    v &= (1ull << B) - 1;
    if (S::F) v |= (uint64_t)((fl >> j) & 1u) << B;
    x[j] = v;
  }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    u32x4 v;
    v.x = (uint32_t)x[2 * g];
    v.y = (uint32_t)(x[2 * g] >> 32);
    v.z = (uint32_t)x[2 * g + 1];
    v.w = (uint32_t)(x[2 * g + 1] >> 32);
    *reinterpret_cast<u32x4*>(dst + 128 * g + 2 * lane) = v;
  }
}

__global__ __launch_bounds__(64 * kPackedWaves) void blob_unpack_kernel(const uint32_t* __restrict__ src,
                                                                       uint64_t rows, uint32_t L, uint32_t logN,
                                                                       ArenaPack ap, uint64_t* __restrict__ dst) {
  const uint64_t r = (uint64_t)blockIdx.x * kPackedWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (r >= rows) return;
  const uint32_t lane = threadIdx.x & 63;
  const PackedRow pr = packed_row(r, 1, L, logN, ap);
  const uint32_t* __restrict__ sl = src + pr.base;
  uint64_t* __restrict__ o = dst + r * kArenaChunk;
  switch (pr.U) {
#define UPR(UU) \
  case UU: unpack_row<UU>(sl, o, lane); break;
    SHELFI_PACK_WIDTHS(UPR)
#undef UPR
    default: break;
  }
}

void launch_blob_pack(const uint64_t* src, uint64_t K, uint32_t L, uint32_t logN, const ArenaPack& ap,
                      const TowerConst* tc, uint32_t* dst, uint32_t* bad, hipStream_t s) {
  launch_arena_pack(src, 0, K * 2 * L << (logN - 9), 1, 0, L, logN, ap, tc, reinterpret_cast<uint64_t*>(dst), bad,
                    s);
}

void launch_blob_unpack(const uint32_t* src, uint64_t K, uint32_t L, uint32_t logN, const ArenaPack& ap,
                        uint64_t* dst, hipStream_t s) {
  const uint64_t rows = K * 2 * L << (logN - 9);
  if (!rows) return;
  const uint64_t blocks = (rows + kPackedWaves - 1) / kPackedWaves;
  if (blocks > 0x7FFFFFFFull) throw Error{SHELFI_ERR_ARG, "blob too large"};
  hipLaunchKernelGGL(blob_unpack_kernel, dim3((uint32_t)blocks), dim3(64 * kPackedWaves), 0, s, src, rows, L, logN,
                     ap, dst);
  SHELFI_HIP(hipGetLastError());
}

// The direct uploads' gather (round 5): 16 output bytes per thread from 5 aligned dwords of the raw
// upload and v_alignbyte (the archive's tower runs sit at arbitrary byte offsets); blockIdx.y = run.
__global__ __launch_bounds__(256) void gather_runs_kernel(const uint8_t* __restrict__ raw,
                                                          const uint64_t* __restrict__ src_off, uint32_t run_bytes,
                                                          uint8_t* __restrict__ dst) {
  const uint64_t j = blockIdx.y;
  const uint8_t* s = raw + src_off[j];
  u32x4* d = reinterpret_cast<u32x4*>(dst + j * run_bytes);
  const uint32_t sh = (uint32_t)((uintptr_t)s & 3u);
  const uint32_t* w = reinterpret_cast<const uint32_t*>((uintptr_t)s & ~(uintptr_t)3);
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < run_bytes / 16; i += gridDim.x * 256) {
    const uint32_t* p = w + 4 * i;
    const uint32_t a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3], a4 = sh ? p[4] : 0u;
    u32x4 v;
    v.x = __builtin_amdgcn_alignbyte(a1, a0, sh);
    v.y = __builtin_amdgcn_alignbyte(a2, a1, sh);
    v.z = __builtin_amdgcn_alignbyte(a3, a2, sh);
    v.w = __builtin_amdgcn_alignbyte(a4, a3, sh);
    d[i] = v;
  }
}

void launch_gather_runs(const uint8_t* raw, const uint64_t* src_off, uint64_t runs, uint32_t run_bytes, uint8_t* dst,
                        hipStream_t s) {
  if (run_bytes % 16) throw Error{SHELFI_ERR_ARG, "gather: run size not a multiple of 16 bytes"};
  const uint32_t per = std::max(1u, std::min(16u, run_bytes / (256u * 16u * 4u)));
  for (uint64_t j0 = 0; j0 < runs; j0 += 65535) {  // grid.y <= 65535
    const uint32_t nj = (uint32_t)std::min<uint64_t>(65535, runs - j0);
    hipLaunchKernelGGL(gather_runs_kernel, dim3(per, nj), dim3(256), 0, s, raw, src_off + j0, run_bytes,
                       dst + j0 * run_bytes);
    SHELFI_HIP(hipGetLastError());
  }
}

// Rows per wavg block: with C <= 8 learners a one-row thread has only C 16-byte loads in
// flight; the kernel then takes 2 rows.  Measured in one process per shape (tools/wavg_rows_ab.py,
// profiles/probes/r03_wavg_rows_ab.txt).  SHELFI_WAVG_ROWS=1|2 forces one (A/B probe switch).
static int wavg_rows(uint32_t C, uint64_t rows) {
  if (switches().wavg_rows) return switches().wavg_rows;
  if (C <= 8) return 2;
  return C >= 16 && rows >= 16384 ? 2 : 1;
}

void launch_wavg(const WavgArgs& a, const TowerConst* tc, hipStream_t s) {
  const uint64_t total = a.rows << a.logN;
  const uint64_t rows = total / kWavgPerBlock;  // always even: N / 512 >= 2 rows per tower
  if (!rows) return;
  int R = wavg_rows(a.C, rows);
  while (R > 1 && ((1ull << a.logN) / kWavgPerBlock) % R) R >>= 1;  // a block stays in one tower
  const uint64_t blocks = rows / R;
  if (blocks > 0xFFFFFFFFull) throw Error{SHELFI_ERR_ARG, "aggregation batch too large"};
  const dim3 g((uint32_t)blocks), b(kWavgThreads);
  if (a.bad && R == 2)
    hipLaunchKernelGGL((wavg_kernel<true, 2>), g, b, 0, s, a, tc);
  else if (a.bad)
    hipLaunchKernelGGL((wavg_kernel<true, 1>), g, b, 0, s, a, tc);
  else if (R == 2)
    hipLaunchKernelGGL((wavg_kernel<false, 2>), g, b, 0, s, a, tc);
  else
    hipLaunchKernelGGL((wavg_kernel<false, 1>), g, b, 0, s, a, tc);
  SHELFI_HIP(hipGetLastError());
}

// Every residue of a [K][2][L][N] batch < q_t? (*bad |= 1 otherwise): the uint64 arena layout's
// upload check (the packed layout checks while packing, arena_pack_kernel).
__global__ __launch_bounds__(256) void check_residues_kernel(const uint64_t* __restrict__ ct, uint32_t L,
                                                             uint32_t logN, const TowerConst* __restrict__ tcs,
                                                             uint32_t* __restrict__ bad) {
  const uint64_t base = (uint64_t)blockIdx.x * 512;
  const uint32_t t = (uint32_t)((base >> logN) % L);
  const uint64_t q = tcs[t].q;
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(ct + base + 2u * threadIdx.x));
  if ((((uint64_t)v.y << 32) | v.x) >= q || (((uint64_t)v.w << 32) | v.z) >= q) atomicOr(bad, 1u);
}

void launch_check_residues(const uint64_t* ct, uint64_t rows, uint32_t L, uint32_t logN, const TowerConst* tc,
                           uint32_t* bad, hipStream_t s) {
  const uint64_t blocks = (rows << logN) / 512;
  if (!blocks) return;
  if (blocks > 0x7FFFFFFFull) throw Error{SHELFI_ERR_ARG, "batch too large"};
  hipLaunchKernelGGL(check_residues_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, ct, L, logN, tc, bad);
  SHELFI_HIP(hipGetLastError());
}

// A collective's uint64 sum of G <= 15 partial sums (each < q < 2^60) -> [0, q).
__global__ __launch_bounds__(256) void modq_kernel(uint64_t* buf, uint32_t L, uint32_t logN,
                                                   const TowerConst* __restrict__ tcs) {
  const uint64_t base = (uint64_t)blockIdx.x * 512;
  const uint32_t t = (uint32_t)((base >> logN) % L);
  const uint64_t q = tcs[t].q, osh = tcs[t].one_shoup;
  uint64_t* p = buf + base + 2u * threadIdx.x;
  p[0] = red64(p[0], q, osh);
  p[1] = red64(p[1], q, osh);
}

void launch_modq(uint64_t* buf, uint64_t rows, uint32_t L, uint32_t logN, const TowerConst* tc,
                 hipStream_t s) {
  const uint64_t blocks = (rows << logN) / 512;
  if (!blocks) return;
  hipLaunchKernelGGL(modq_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, buf, L, logN, tc);
  SHELFI_HIP(hipGetLastError());
}

}  // namespace shelfi

// kernels.hip — hand-written gfx950 kernels for the RNS-CKKS aggregation path.
//
// Data layout in HBM (all uint64 residues, EVALUATION domain, PALISADE's
// bit-reversed order):  ciphertext batch [K][2][L][N]  (ct, poly, tower, coeff) —
// the order of a serialized vector<Ciphertext<DCRTPoly>> (ckks.cpp:98-100).
//
// Kernels (roofline class in DESIGN.md):
//   (wavg_kernel, wavg_packed, the arena packing and modq_kernel -- EvalMult(ct, (float)w) +
//    EvalAdd over C learners, ckks.cpp:286-297, HBM-bound -- live in wavg.hip)
//   ntt_*              negacyclic NTT/INTT, 2 passes (register columns + LDS blocks)
//   fft_*              CKKS special FFT / inverse (encode / decode), 2 passes
//   enc_prep_kernel    round/scale the encoded slots + ChaCha20 sampling of (v, e0, e1)
//                      into a compact 10-byte record per coefficient (ckks.cpp:80-81)
//   ntt_fwd_cols_enc   expand the record per tower + first NTT stages
//   ntt_fwd_blocks_enc(_ct)  last NTT stages of v, m+e0, e1 + c0 = v*b + (m+e0), c1 = v*a + e1
//                      (_ct: compile-time shape over per-block twiddle slices)
//   ntt_inv_blocks(_dec_ct)  (decrypt) c0 + c1*s formed on load (ckks.cpp:189) + first INTT stages
//   ntt_inv_cols_crt   last INTT stages fused with the exact centered CRT -> double / scale
//   crt_decode_kernel  the CRT alone (shapes the fused kernel does not cover)
//   keygen_*           ternary s, Gaussian e, uniform a; b = e - a*s
//
// 64-bit modular arithmetic: CDNA4 has no 64x64->128 multiply; products are
// built from v_mad_u64_u32 / v_mul_hi_u32 by the compiler (__umul64hi).  Constant
// multiplications use Shoup's precomputed quotient (w' = floor(w 2^64 / q)).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <type_traits>
#include <vector>

#include "dev_common.h"
#include "shelfi_internal.h"

namespace shelfi {

// Host side of xcd_block: the combo count G when the block passes may deal (tower, block)
// combos per XCD (G % 8 == 0), else 0.  SHELFI_XCD_ORDER=0 keeps the natural order (A/B
// probe switch).
static uint32_t xcd_combos(uint64_t G) {
  if (!switches().xcd_order) return 0;
  return (G % 8 == 0 && G <= 0xFFFFFFFFull) ? (uint32_t)G : 0;
}

// ------------------------------------------------------------------- NTT ----
// Forward (Cooley-Tukey, natural -> bit-reversed), stage m (= 2^s) pairs
// (j, j + N/2m) with twiddle psi_rev[m + j/(N/m)].  The first LOGR stages pair
// elements R = 2^LOGR apart in the top bits: each thread holds one column of R
// elements (stride N/R) in registers, all twiddles wave-uniform.  The remaining
// stages act inside contiguous blocks of N/R elements, staged in LDS.
template <int LOGR>
__global__ __launch_bounds__(256) void ntt_fwd_cols(uint64_t* __restrict__ polys, uint32_t L,
                                                    uint32_t logN, const uint64_t* __restrict__ tw,
                                                    const uint64_t* __restrict__ twp,
                                                    const TowerConst* __restrict__ tcs) {
  constexpr int R = 1 << LOGR;
  const uint32_t N = 1u << logN;
  const uint32_t BLK = N >> LOGR;
  const uint32_t bpp = BLK / 256;
  const uint64_t poly = blockIdx.x / bpp;
  const uint32_t col = (blockIdx.x % bpp) * 256 + threadIdx.x;
  const uint32_t t = (uint32_t)(poly % L);
  const uint64_t q = tcs[t].q;
  const uint64_t* __restrict__ w = tw + (uint64_t)t * N;
  const uint64_t* __restrict__ wp = twp + (uint64_t)t * N;
  uint64_t* __restrict__ a = polys + poly * N + col;
  uint64_t x[R];
#pragma unroll
  for (int r = 0; r < R; ++r) x[r] = a[(uint64_t)r * BLK];
#pragma unroll
  for (int s = 0; s < LOGR; ++s) {
    const int m = 1 << s, tr = R >> (s + 1);
#pragma unroll
    for (int i = 0; i < m; ++i) {
      const uint64_t W = w[m + i], Wp = wp[m + i];
#pragma unroll
      for (int jj = 0; jj < tr; ++jj) {
        const int r0 = 2 * i * tr + jj, r1 = r0 + tr;
        ct_bfly(x[r0], x[r1], W, Wp, q);
      }
    }
  }
  // lazy values in [0, 8q): the blocks pass that follows canonicalises
#pragma unroll
  for (int r = 0; r < R; ++r) a[(uint64_t)r * BLK] = x[r];
}

// Blocks pass, stages s = sstart .. logN-1 on contiguous blocks of 2^(logN-sstart).
__global__ __launch_bounds__(256) void ntt_fwd_blocks(uint64_t* __restrict__ polys, uint32_t L,
                                                      uint32_t logN, uint32_t sstart,
                                                      const uint64_t* __restrict__ tw,
                                                      const uint64_t* __restrict__ twp,
                                                      const TowerConst* __restrict__ tcs) {
  extern __shared__ __attribute__((aligned(16))) uint64_t sm[];
  const uint32_t N = 1u << logN, blkLog = logN - sstart, blk = 1u << blkLog;
  const uint32_t nb = 1u << sstart;
  const uint64_t poly = blockIdx.x >> sstart;
  const uint32_t b = blockIdx.x & (nb - 1);
  const uint32_t t = (uint32_t)(poly % L);
  const uint64_t q = tcs[t].q;
  uint64_t* __restrict__ a = polys + poly * N + ((uint64_t)b << blkLog);
  for (uint32_t p = threadIdx.x; p < blk / 2; p += 256)
    lds_put2(sm, p, reinterpret_cast<const ulonglong2*>(a)[p]);
  __syncthreads();
  ntt_fwd_block_stages(sm, blkLog, b, logN, tw + (uint64_t)t * N, twp + (uint64_t)t * N, q);
  for (uint32_t p = threadIdx.x; p < blk / 2; p += 256) {
    const ulonglong2 v = lds_get2(sm, p);
    reinterpret_cast<ulonglong2*>(a)[p] = make_ulonglong2(canon8(v.x, q), canon8(v.y, q));
  }
}

// Encrypt's last NTT pass fused with the public-key combine: one workgroup owns block
// b of tower t of ciphertext k, transforms v, m + e0 and e1 (pbuf [K][3][L][N], lazy
// after the columns pass) one after the other through the same LDS block, and writes
// c0 = v*b + (m + e0), c1 = v*a + e1 (ckks.cpp:81, PALISADE Encrypt) — the transformed
// polynomials never return to HBM.
template <int PP>  // 16-byte pairs per thread: blk / 512
__global__ __launch_bounds__(256) void ntt_fwd_blocks_enc(const uint64_t* __restrict__ pbuf,
                                                          uint32_t L, uint32_t logN, uint32_t sstart,
                                                          const uint64_t* __restrict__ tw,
                                                          const uint64_t* __restrict__ twp,
                                                          const TowerConst* __restrict__ tcs,
                                                          const uint64_t* __restrict__ pk,
                                                          const uint64_t* __restrict__ pksh,
                                                          uint64_t* __restrict__ ct,
                                                          const int64_t* __restrict__ me0,
                                                          const int16_t* __restrict__ ve) {
  extern __shared__ __attribute__((aligned(16))) uint64_t sm[];
  const uint32_t blkLog = logN - sstart, blk = 1u << blkLog;
  const uint32_t b = blockIdx.x & ((1u << sstart) - 1);
  const uint64_t rest = blockIdx.x >> sstart;
  const uint32_t t = (uint32_t)(rest % L);
  const uint64_t k = rest / L;
  const uint64_t q = tcs[t].q;
  const uint64_t* __restrict__ w = tw + ((uint64_t)t << logN);
  const uint64_t* __restrict__ wp = twp + ((uint64_t)t << logN);
  const uint64_t off = ((uint64_t)t << logN) + ((uint64_t)b << blkLog);  // within [L][N]
  const uint64_t LN = (uint64_t)L << logN;
  ulonglong2 V[PP];  // NTT(v), kept for both products
#pragma unroll
  for (int poly = 0; poly < 3; ++poly) {
    if (me0) {  // single-pass ring: expand the compact sample record (no columns pass)
      const TowerConst& cst = tcs[t];
      const uint64_t base = (k << logN) + ((uint64_t)b << blkLog);
      for (uint32_t i = threadIdx.x; i < blk; i += 256) {
        const int32_t sv = ve[base + i];
        sm[lds_sw(i)] = poly == 1 ? mod_signed_dev(me0[base + i], cst)
                                  : small_mod(poly == 0 ? (int32_t)(int8_t)(sv & 0xFF) : (sv >> 8), q);
      }
    } else {
      const ulonglong2* src = reinterpret_cast<const ulonglong2*>(pbuf + (k * 3 + poly) * LN + off);
      for (uint32_t p = threadIdx.x; p < blk / 2; p += 256) lds_put2(sm, p, src[p]);
    }
    __syncthreads();
    ntt_fwd_block_stages(sm, blkLog, b, logN, w, wp, q);
#pragma unroll
    for (int i = 0; i < PP; ++i) {
      const uint32_t p = threadIdx.x + 256 * i;
      if (p >= blk / 2) break;
      ulonglong2 v = lds_get2(sm, p);
      v = make_ulonglong2(canon8(v.x, q), canon8(v.y, q));
      const uint64_t e = off + 2 * p;
      if (poly == 0) {
        V[i] = v;
      } else {  // poly 1: c0 = v*b + (m + e0); poly 2: c1 = v*a + e1
        const uint64_t off_pk = (poly == 1 ? 0 : LN) + e;
        const ulonglong2 P = *reinterpret_cast<const ulonglong2*>(pk + off_pk);
        const ulonglong2 Ps = *reinterpret_cast<const ulonglong2*>(pksh + off_pk);
        ulonglong2 c;
        c.x = addmod(shoup_mul(V[i].x, P.x, Ps.x, q), v.x, q);
        c.y = addmod(shoup_mul(V[i].y, P.y, Ps.y, q), v.y, q);
        *reinterpret_cast<ulonglong2*>(ct + (k * 2 + (poly - 1)) * LN + e) = c;
      }
    }
    __syncthreads();  // LDS is refilled by the next polynomial
  }
}

// XCD-aware block order for the block passes.  Blocks b and b + 8 share an XCD (observed
// round-robin dealing, MI355X_MICROARCH "Workgroup dispatch"; used for speed only: any
// placement gives the same results).  The G = L 2^sstart (tower, block) combos each own a
// shared slice of twiddles and key words (64-160 KiB per workgroup, 4-6 MiB per launch at
// 2^15/L4, more than one XCD's 4 MiB L2); dealt in natural order every XCD touches all of
// them and they stream from the Infinity Cache.  With xg = G (G % 8 == 0) XCD slot x = bid % 8
// owns combos [x G/8, (x+1) G/8) for every ciphertext, 1/8 of the slices.  Returns the
// logical block id k G + combo; xg == 0 keeps the natural order.
__device__ __forceinline__ uint32_t xcd_block(uint32_t bid, uint32_t xg) {
  if (!xg) return bid;
  const uint32_t g8 = xg >> 3, i = bid >> 3;
  const uint32_t k = i / g8;
  return k * xg + (bid & 7) * g8 + (i - k * g8);
}

// Inverse (GS) chunk of KC stages starting at local half-size 2^T0: set s -> g = s >> T0,
// j0 = g 2^(T0+KC) + (s mod 2^T0), elements j0 + m 2^T0; stage-i twiddles are
// tb[2^l + g 2^(KC-1-i) + gs], gs < 2^(KC-1-i), l = BL - 1 - T0 - i.
template <int BL, int T0, int KC, bool IN8, class Load, class Store>
__device__ __forceinline__ void inv_chunk_ct(const ulonglong2* __restrict__ tb, uint64_t q,
                                             uint64_t n8q, Load ld, Store st) {
  constexpr int M = 1 << KC, NS = (1 << (BL - KC)) / 256;
  static_assert(NS >= 1, "chunk plan");
#pragma unroll
  for (int r = 0; r < NS; ++r) {
    const uint32_t s = threadIdx.x + 256u * r;
    const uint32_t g = s >> T0;
    const uint32_t j0 = (g << (T0 + KC)) + (s & ((1u << T0) - 1));
    const uint32_t pj0 = lpad(j0);
    uint64_t x[M];
#pragma unroll
    for (int m = 0; m < M; ++m) x[m] = ld(j0 + (m << T0), pj0 + lofs<(1 << T0)>(m));
#pragma unroll
    for (int i = 0; i < KC; ++i) {
      const int hm = 1 << i;
      const ulonglong2* __restrict__ tw = tb + (1u << (BL - 1 - T0 - i)) + (g << (KC - 1 - i));
#pragma unroll
      for (int gs = 0; gs < (M >> (i + 1)); ++gs) {
        const ulonglong2 W = tw[gs];
#pragma unroll
        for (int mm = 0; mm < hm; ++mm) {
          if (gs_in8<IN8>(i, mm))
            gs_bfly_b<true>(x[gs * 2 * hm + mm], x[gs * 2 * hm + mm + hm], W.x, W.y, q, n8q);
          else
            gs_bfly_b<false>(x[gs * 2 * hm + mm], x[gs * 2 * hm + mm + hm], W.x, W.y, q, n8q);
        }
      }
    }
    st(r, j0, pj0, x);
  }
}

// Encrypt's blocks pass at compile-time shape: chunks K1..K4 (sum BL) per polynomial,
// the first on registers loaded straight from pbuf, the last combined with the public key straight
// from registers (3 LDS round trips and 3 barriers per polynomial instead of 5 and 5).
// Same contract as ntt_fwd_blocks_enc.
template <int BL, int K1, int K2, int K3, int K4>
__global__ __launch_bounds__(256) void ntt_fwd_blocks_enc_ct(
    const uint64_t* __restrict__ pbuf, uint32_t L, uint32_t logN, const ulonglong2* __restrict__ twb,
    const TowerConst* __restrict__ tcs, const uint64_t* __restrict__ pk,
    const uint64_t* __restrict__ pksh, uint64_t* __restrict__ ct, uint32_t zero, uint32_t xg) {
  static_assert(K1 + K2 + K3 + K4 == BL, "chunk plan must cover the block");
  constexpr int M1 = 1 << K1, NS1 = (1 << (BL - K1)) / 256, D1 = BL - K1;
  constexpr int ML = 1 << K4, NSL = (1 << (BL - K4)) / 256;
  __shared__ __attribute__((aligned(16))) uint64_t sm[lpad_size(BL)];
  const uint32_t sstart = logN - BL;
  const uint32_t bid = xcd_block(blockIdx.x, xg);
  const uint32_t b = bid & ((1u << sstart) - 1);
  const uint32_t rest = bid >> sstart;
  const uint32_t t = rest % L, k = rest / L;
  const TowerConst& cst = tcs[t];
  const uint64_t q = cst.q, n8q = cst.n8q;
  const ulonglong2* tb0 = twb + ((uint64_t)t << logN) + ((uint64_t)b << BL);
  const uint64_t off = ((uint64_t)t << logN) + ((uint64_t)b << BL);
  const uint64_t LN = (uint64_t)L << logN;
  const auto lds_ld = [&](uint32_t, uint32_t pj) { return sm[pj]; };
  uint64_t V[NSL][ML];  // NTT(v) at this thread's last-chunk positions
#pragma unroll 1
  for (int poly = 0; poly < 3; ++poly) {
    // reload the twiddles per polynomial (zero == 0 is opaque to the compiler): hoisted
    // out of this loop they would hold ~100 VGPRs for the whole kernel
    const ulonglong2* __restrict__ tb = tb0 + poly * zero;
    const uint64_t* __restrict__ src = pbuf + ((uint64_t)k * 3 + poly) * LN + off;
#pragma unroll
    for (int r = 0; r < NS1; ++r) {  // first chunk: one group, block-uniform twiddles
      uint64_t x[M1];
#pragma unroll
      for (int m = 0; m < M1; ++m) x[m] = src[threadIdx.x + 256u * r + (m << D1)];
      fwd_set_ct<BL, BL - 1, K1>(x, 0u, tb, q, n8q);
      const uint32_t p0 = lpad(threadIdx.x + 256u * r);
#pragma unroll
      for (int m = 0; m < M1; ++m) sm[p0 + lofs<(1 << D1)>(m)] = x[m];
    }
    __syncthreads();
    fwd_chunk_ct<BL, BL - 1 - K1, K2>(tb, q, n8q, lds_ld, [&](int, uint32_t, uint32_t pj0, auto& x) {
#pragma unroll
      for (int m = 0; m < (1 << K2); ++m) sm[pj0 + lofs<(1 << (BL - K1 - K2))>(m)] = x[m];
    });
    __syncthreads();
    fwd_chunk_ct<BL, BL - 1 - K1 - K2, K3>(tb, q, n8q, lds_ld, [&](int, uint32_t, uint32_t pj0, auto& x) {
#pragma unroll
      for (int m = 0; m < (1 << K3); ++m) sm[pj0 + lofs<(1 << (BL - K1 - K2 - K3))>(m)] = x[m];
    });
    __syncthreads();
    // last chunk (contiguous sets of ML, written inline: V captured by a lambda would
    // live in scratch)
#pragma unroll
    for (int r = 0; r < NSL; ++r) {
      const uint32_t g = threadIdx.x + 256u * r, j0 = g << K4, pj0 = lpad(j0);
      uint64_t x[ML];
#pragma unroll
      for (int m = 0; m < ML; ++m) x[m] = sm[pj0 + m];
      fwd_set_ct<BL, K4 - 1, K4>(x, g, tb, q, n8q);
      if (poly == 0) {  // NTT(v), lazy (< 12q): only ever a Shoup multiplicand
#pragma unroll
        for (int m = 0; m < ML; ++m) V[r][m] = x[m];
      } else {  // poly 1: c0 = v*b + (m + e0); poly 2: c1 = v*a + e1 (< 4q + 12q, then [0, q))
        const uint64_t e = off + j0;
        const uint64_t off_pk = (poly == 1 ? 0 : LN) + e;
        uint64_t* __restrict__ dst = ct + ((uint64_t)k * 2 + (poly - 1)) * LN + e;
#pragma unroll
        for (int m = 0; m < ML; m += 2) {
          const ulonglong2 P = *reinterpret_cast<const ulonglong2*>(pk + off_pk + m);
          const ulonglong2 Ps = *reinterpret_cast<const ulonglong2*>(pksh + off_pk + m);
          ulonglong2 c;
          c.x = red_any(shoup_lazy(V[r][m], P.x, Ps.x, q) + x[m], cst);
          c.y = red_any(shoup_lazy(V[r][m + 1], P.y, Ps.y, q) + x[m + 1], cst);
          *reinterpret_cast<ulonglong2*>(dst + m) = c;
        }
      }
    }
    __syncthreads();  // LDS is refilled by the next polynomial
  }
}

// Persistent, software-pipelined form of ntt_fwd_blocks_enc_ct (round 3), the same idea as
// ntt_inv_blocks_dec_pp: a workgroup owns one (tower, block) combo and walks ciphertexts
// k0, k0 + P, ...; the combo's twiddle slice sits in LDS (copied once); each polynomial's
// first-chunk pbuf words are loaded into registers while the previous polynomial is being
// transformed, and the public-key words of the combine are requested one polynomial ahead.
// Same arithmetic and outputs as ntt_fwd_blocks_enc_ct.
// NR: the launch covers towers [t0, t0 + nt) whose columns pass ran unreduced (q < kNoRedQ,
// enc_cols_fused's t_split): no reductions in the block stages either (fwd_set_ct).
// WL (round 4): only the first chunk's exchange crosses waves.  After the stages of half-size
// 2^(BL-1) .. 2^(BL-K1) the block falls apart into 2^K1 independent sub-blocks; the middle chunks'
// sets already keep each wave inside 512 contiguous elements, and the last chunk's sets are dealt
// so that they do too (set g = 2 * 64 w + 64 r + lane), so the exchanges between the middle chunks
// and into the last one need only the wave's own LDS ordering (wave_lds_sync), not a workgroup
// barrier: 2 barriers per polynomial instead of 4.
// VT (round 5): v's columns pass never ran (enc_cols_fused<..., VT>): the first chunk's v words are
// the column's packed group patterns, and each row value is the sum of its block's 4 enc_vtab entries
// (< 4q), looked up in a 2.6 KiB LDS slice copied once per workgroup (the combo's block b is the row).
template <int BL, int K1, int K2, int K3, int K4, bool NR, bool WL = false, bool VT = false>
__global__ __launch_bounds__(256) void ntt_fwd_blocks_enc_pp(
    const uint64_t* __restrict__ pbuf, uint32_t L, uint32_t logN, const ulonglong2* __restrict__ twb,
    const TowerConst* __restrict__ tcs, const uint64_t* __restrict__ pk, const uint64_t* __restrict__ pksh,
    uint64_t* __restrict__ ct, uint32_t K, uint32_t per_combo, uint32_t t0, uint32_t nt,
    const uint64_t* __restrict__ vtab) {
  static_assert(K1 + K2 + K3 + K4 == BL, "chunk plan must cover the block");
  static_assert(!VT || (BL == 11 && K1 == 3), "v tables: a 16-row columns pass, 8 columns per thread");
  constexpr int M1 = 1 << K1, NS1 = (1 << (BL - K1)) / 256, D1 = BL - K1;
  constexpr int ML = 1 << K4, NSL = (1 << (BL - K4)) / 256;
  // WL needs every middle-chunk set of a wave inside its 64 * 2^(BL-8) contiguous elements
  static_assert(!WL || (BL == 11 && K1 == 3 && K2 == 3 && K3 == 3 && K4 == 2), "wave-local plan");
  __shared__ __attribute__((aligned(16))) ulonglong2 tws[1 << BL];
  __shared__ __attribute__((aligned(16))) uint64_t sm[lpad_size(BL)];
  __shared__ uint64_t vts[VT ? 4 * 81 : 1];
  // the last chunk's set r of this thread
  const auto last_g = [&](int r) -> uint32_t {
    return WL ? ((threadIdx.x >> 6) * (64u * NSL) + 64u * r + (threadIdx.x & 63u)) : threadIdx.x + 256u * r;
  };
  const uint32_t sstart = logN - BL;
  const uint32_t ncombo = nt << sstart;
  const uint32_t combo = blockIdx.x % ncombo;
  const uint32_t b = combo & ((1u << sstart) - 1), t = t0 + (combo >> sstart);
  const TowerConst& cst = tcs[t];
  const uint64_t q = cst.q, n8q = cst.n8q;
  const uint64_t off = ((uint64_t)t << logN) + ((uint64_t)b << BL);
  const uint64_t LN = (uint64_t)L << logN;
  {
    const ulonglong2* __restrict__ src = twb + off;
    for (uint32_t i = threadIdx.x; i < (1u << BL); i += 256) tws[i] = src[i];
    if (VT)  // rows = blocks: this combo's row b of tower t
      for (uint32_t i = threadIdx.x; i < 4 * 81; i += 256) vts[i] = vtab[((uint64_t)t * 16 + b) * (4 * 81) + i];
  }
  uint64_t pf[NS1][M1];              // the next polynomial's first-chunk words
  ulonglong2 P[NSL][ML / 2], Ps[NSL][ML / 2];  // the next combine's key words (b or a)
  uint64_t V[NSL][ML];                // NTT(v) at this thread's last-chunk positions
  const auto fetch = [&](uint32_t kk, int poly) {
    if (VT && poly == 0) {  // the packed patterns of columns tid + 256 m (this block's row of each)
      const uint32_t* __restrict__ vp = reinterpret_cast<const uint32_t*>(pbuf + (uint64_t)kk * 3 * LN);
#pragma unroll
      for (int m = 0; m < M1; ++m) pf[0][m] = vp[threadIdx.x + (m << D1)];
      return;
    }
    const uint64_t* __restrict__ src = pbuf + ((uint64_t)kk * 3 + poly) * LN + off;
#pragma unroll
    for (int r = 0; r < NS1; ++r)
#pragma unroll
      for (int m = 0; m < M1; ++m) pf[r][m] = __builtin_nontemporal_load(src + threadIdx.x + 256u * r + (m << D1));
  };
  const auto fetch_key = [&](int poly) {  // poly 1: b, poly 2: a
#pragma unroll
    for (int r = 0; r < NSL; ++r) {
      const uint64_t e = (poly == 1 ? 0 : LN) + off + (last_g(r) << K4);
#pragma unroll
      for (int m = 0; m < ML; m += 2) {
        P[r][m / 2] = *reinterpret_cast<const ulonglong2*>(pk + e + m);
        Ps[r][m / 2] = *reinterpret_cast<const ulonglong2*>(pksh + e + m);
      }
    }
  };
  uint32_t k = blockIdx.x / ncombo;
  if (k < K) fetch(k, 0);
  __syncthreads();  // the twiddle slice is in LDS
  const auto lds_ld = [&](uint32_t, uint32_t pj) { return sm[pj]; };
  const auto mid_sync = [] {
    if (WL)
      wave_lds_sync();
    else
      __syncthreads();
  };
#pragma unroll 1
  for (; k < K; k += per_combo) {
#pragma unroll 1
    for (int poly = 0; poly < 3; ++poly) {
      uint64_t x[NS1][M1];
      if (VT && poly == 0) {  // NTT(v)'s columns pass as table sums: row b of each column, < 4q
#pragma unroll
        for (int m = 0; m < M1; ++m) {
          const uint32_t w = (uint32_t)pf[0][m];
          x[0][m] = vts[w & 127u] + vts[81 + ((w >> 7) & 127u)] + vts[162 + ((w >> 14) & 127u)] + vts[243 + (w >> 21)];
        }
      } else {
#pragma unroll
        for (int r = 0; r < NS1; ++r)
#pragma unroll
          for (int m = 0; m < M1; ++m) x[r][m] = pf[r][m];
      }
      // the next polynomial's words (or the next ciphertext's v) and this one's key words
      if (poly < 2)
        fetch(k, poly + 1);
      else if (k + per_combo < K)
        fetch(k + per_combo, 0);
      if (poly > 0) fetch_key(poly);
#pragma unroll
      for (int r = 0; r < NS1; ++r)  // first chunk: one group, block-uniform twiddles
        fwd_set_ct<BL, BL - 1, K1, NR>(x[r], 0u, tws, q, n8q);
      // WL: the previous polynomial's last-chunk reads must be done before LDS is refilled; with the
      // first chunk computed in registers first, a wave that reaches this barrier early has already
      // done that work (without WL the barrier sits at the end of the previous polynomial)
      if (WL) __syncthreads();
#pragma unroll
      for (int r = 0; r < NS1; ++r) {
        const uint32_t p0 = lpad(threadIdx.x + 256u * r);
#pragma unroll
        for (int m = 0; m < M1; ++m) sm[p0 + lofs<(1 << D1)>(m)] = x[r][m];
      }
      __syncthreads();
      fwd_chunk_ct<BL, BL - 1 - K1, K2, NR>(tws, q, n8q, lds_ld, [&](int, uint32_t, uint32_t pj0, auto& y) {
#pragma unroll
        for (int m = 0; m < (1 << K2); ++m) sm[pj0 + lofs<(1 << (BL - K1 - K2))>(m)] = y[m];
      });
      mid_sync();
      fwd_chunk_ct<BL, BL - 1 - K1 - K2, K3, NR>(tws, q, n8q, lds_ld, [&](int, uint32_t, uint32_t pj0, auto& y) {
#pragma unroll
        for (int m = 0; m < (1 << K3); ++m) sm[pj0 + lofs<(1 << (BL - K1 - K2 - K3))>(m)] = y[m];
      });
      mid_sync();
#pragma unroll
      for (int r = 0; r < NSL; ++r) {
        const uint32_t g = last_g(r), j0 = g << K4, pj0 = lpad(j0);
        uint64_t y[ML];
#pragma unroll
        for (int m = 0; m < ML; ++m) y[m] = sm[pj0 + m];
        fwd_set_ct<BL, K4 - 1, K4, NR>(y, g, tws, q, n8q);
        if (poly == 0) {  // NTT(v), lazy (< 12q): only ever a Shoup multiplicand
#pragma unroll
          for (int m = 0; m < ML; ++m) V[r][m] = y[m];
        } else {  // poly 1: c0 = v*b + (m + e0); poly 2: c1 = v*a + e1
          uint64_t* __restrict__ dst = ct + ((uint64_t)k * 2 + (poly - 1)) * LN + off + j0;
#pragma unroll
          for (int m = 0; m < ML; m += 2) {
            ulonglong2 c;
            c.x = red_any(shoup_lazy(V[r][m], P[r][m / 2].x, Ps[r][m / 2].x, q) + y[m], cst);
            c.y = red_any(shoup_lazy(V[r][m + 1], P[r][m / 2].y, Ps[r][m / 2].y, q) + y[m + 1], cst);
            *reinterpret_cast<ulonglong2*>(dst + m) = c;
          }
        }
      }
      if (!WL) __syncthreads();  // LDS is refilled by the next polynomial
    }
  }
}

// Decrypt's first INTT pass at compile-time shape (chunks K1..K4, sum BL; needs
// logN > BL): c0 + c1*s is formed straight into the first chunk's registers from the
// ciphertext batch [K][2][L][N], and the last chunk writes the lazy ([0, 8q)) block to
// dbuf [K][L][N] from registers for ntt_inv_cols.  Same contract as ntt_inv_blocks with
// ct != nullptr and scale_ninv = 0.
// SUM: the ciphertexts are a collective's unfolded uint64 sums of <= 16 canonical residues
// (shelfi_dev_combine_arena with fold = 0): c0 is reduced on load (red_any, [0, 2q)), c1 needs
// nothing (the lazy Shoup product takes any 64-bit multiplicand) — the mod-q fold of the
// combine happens here instead of in a separate pass over the share.
template <int BL, int K1, int K2, int K3, int K4, bool SUM = false>
__global__ __launch_bounds__(256) void ntt_inv_blocks_dec_ct(uint64_t* __restrict__ dbuf, uint32_t L,
                                                             uint32_t logN,
                                                             const ulonglong2* __restrict__ twb,
                                                             const TowerConst* __restrict__ tcs,
                                                             const uint64_t* __restrict__ ct,
                                                             const uint64_t* __restrict__ sk,
                                                             const uint64_t* __restrict__ sksh,
                                                             uint32_t xg, uint32_t ctL) {
  static_assert(K1 + K2 + K3 + K4 == BL, "chunk plan must cover the block");
  __shared__ __attribute__((aligned(16))) uint64_t sm[lpad_size(BL)];
  const uint32_t sstart = logN - BL;
  const uint32_t bid = xcd_block(blockIdx.x, xg);
  const uint32_t b = bid & ((1u << sstart) - 1);
  const uint32_t poly = bid >> sstart;  // k * L + t
  const uint32_t t = poly % L, k = poly / L;
  const TowerConst& cst = tcs[t];
  const uint64_t q = cst.q, n4q = cst.n4q, n8q = cst.n8q;
  const ulonglong2* __restrict__ tb = twb + ((uint64_t)t << logN) + ((uint64_t)b << BL);
  const uint64_t off = ((uint64_t)t << logN) + ((uint64_t)b << BL);
  const uint64_t LN = (uint64_t)L << logN;
  const uint64_t CLN = (uint64_t)ctL << logN;  // the ciphertexts' towers (>= L, decode_towers)
  const uint64_t* __restrict__ c0 = ct + (uint64_t)k * 2 * CLN + off;
  const uint64_t* __restrict__ c1 = c0 + CLN;
  const uint64_t* __restrict__ s = sk + off;
  const uint64_t* __restrict__ ss = sksh + off;
  const auto lds_ld = [&](uint32_t, uint32_t pj) { return sm[pj]; };
  // first chunk: contiguous sets of 2^K1 (T0 = 0)
  inv_chunk_ct<BL, 0, K1, false>(tb, q, n8q,
                          [&](uint32_t j, uint32_t) {
                            const uint64_t a0 = SUM ? red_any(c0[j], cst) : c0[j];
                            return csub_neg(a0 + shoup_lazy(c1[j], s[j], ss[j], q), n4q);
                          },
                          [&](int, uint32_t, uint32_t pj0, auto& x) {
#pragma unroll
                            for (int m = 0; m < (1 << K1); ++m) sm[pj0 + lofs<1>(m)] = x[m];
                          });
  __syncthreads();
  inv_chunk_ct<BL, K1, K2, true>(tb, q, n8q, lds_ld, [&](int, uint32_t, uint32_t pj0, auto& x) {
#pragma unroll
    for (int m = 0; m < (1 << K2); ++m) sm[pj0 + lofs<(1 << K1)>(m)] = x[m];
  });
  __syncthreads();
  inv_chunk_ct<BL, K1 + K2, K3, true>(tb, q, n8q, lds_ld, [&](int, uint32_t, uint32_t pj0, auto& x) {
#pragma unroll
    for (int m = 0; m < (1 << K3); ++m) sm[pj0 + lofs<(1 << (K1 + K2))>(m)] = x[m];
  });
  __syncthreads();
  uint64_t* __restrict__ dst = dbuf + (uint64_t)k * LN + off;
  inv_chunk_ct<BL, BL - K4, K4, true>(tb, q, n8q, lds_ld, [&](int, uint32_t j0, uint32_t, auto& x) {
#pragma unroll
    for (int m = 0; m < (1 << K4); ++m) dst[j0 + (m << (BL - K4))] = x[m];
  });
}

// Persistent, software-pipelined form of ntt_inv_blocks_dec_ct (round 3).  The one-shot
// kernel loads its whole first chunk from HBM and only then computes, and all its workgroups
// start together: measured 0.48 of the VALU issue peak and ~3.6 TB/s, neither bound reached.
// Here a workgroup owns one (tower, block) combo and walks ciphertexts k0, k0 + P, ...:
//  * the combo's 2^BL twiddle pairs are copied into LDS once (32 KiB), so the per-chunk
//    twiddle reads leave the vector-memory queue (whose in-order vmcnt would otherwise make
//    every twiddle wait drain the prefetch below);
//  * the secret-key words s, s' of the first chunk's elements stay in registers;
//  * ciphertext k + P's c0 / c1 words are loaded into registers right after ciphertext k's
//    have been consumed, so their HBM latency hides behind k's stages.
// Same arithmetic, same lazy bounds and same dbuf contents as ntt_inv_blocks_dec_ct.
// WL: as ntt_fwd_blocks_enc_pp's, mirrored: the first three chunks (half-sizes 1 .. 2^(BL-K4-1))
// stay inside 512-element sub-blocks, each wave's own once the first chunk's sets are dealt as
// g = 2 * 64 w + 64 r + lane; only the exchange into the last chunk crosses waves.
template <int BL, int K1, int K2, int K3, int K4, bool SUM = false, bool WL = false>
__global__ __launch_bounds__(256) void ntt_inv_blocks_dec_pp(uint64_t* __restrict__ dbuf, uint32_t L,
                                                             uint32_t logN,
                                                             const ulonglong2* __restrict__ twb,
                                                             const TowerConst* __restrict__ tcs,
                                                             const uint64_t* __restrict__ ct,
                                                             const uint64_t* __restrict__ sk,
                                                             const uint64_t* __restrict__ sksh, uint32_t K,
                                                             uint32_t per_combo, uint32_t ctL) {
  static_assert(K1 + K2 + K3 + K4 == BL, "chunk plan must cover the block");
  constexpr int M1 = 1 << K1, NS1 = (1 << (BL - K1)) / 256;
  static_assert(!WL || (BL == 11 && K1 == 2 && K2 == 3 && K3 == 3 && K4 == 3), "wave-local plan");
  __shared__ __attribute__((aligned(16))) ulonglong2 tws[1 << BL];
  __shared__ __attribute__((aligned(16))) uint64_t sm[lpad_size(BL)];
  // the first chunk's set r of this thread (its elements g 2^K1 + m)
  const auto first_g = [&](int r) -> uint32_t {
    return WL ? ((threadIdx.x >> 6) * (64u * NS1) + 64u * r + (threadIdx.x & 63u)) : threadIdx.x + 256u * r;
  };
  const uint32_t sstart = logN - BL;
  const uint32_t ncombo = L << sstart;
  const uint32_t combo = blockIdx.x % ncombo;
  const uint32_t b = combo & ((1u << sstart) - 1), t = combo >> sstart;
  const TowerConst& cst = tcs[t];
  const uint64_t q = cst.q, n4q = cst.n4q, n8q = cst.n8q;
  const uint64_t off = ((uint64_t)t << logN) + ((uint64_t)b << BL);
  const uint64_t LN = (uint64_t)L << logN;
  {
    const ulonglong2* __restrict__ src = twb + off;
    for (uint32_t i = threadIdx.x; i < (1u << BL); i += 256) tws[i] = src[i];
  }
  // first chunk (T0 = 0): set r of this thread = elements (tid + 256 r) 2^K1 + m
  uint64_t sv[NS1][M1], sw[NS1][M1], p0[NS1][M1], p1[NS1][M1];
#pragma unroll
  for (int r = 0; r < NS1; ++r)
#pragma unroll
    for (int m = 0; m < M1; ++m) {
      const uint32_t j = (first_g(r) << K1) + m;
      sv[r][m] = sk[off + j];
      sw[r][m] = sksh[off + j];
    }
  uint32_t k = blockIdx.x / ncombo;
  const uint64_t CLN = (uint64_t)ctL << logN;  // the ciphertexts' towers (>= L, decode_towers)
  const auto fetch = [&](uint32_t kk) {
    const uint64_t* __restrict__ c0 = ct + (uint64_t)kk * 2 * CLN + off;
#pragma unroll
    for (int r = 0; r < NS1; ++r)
#pragma unroll
      for (int m = 0; m < M1; ++m) {
        const uint32_t j = (first_g(r) << K1) + m;
        p0[r][m] = __builtin_nontemporal_load(c0 + j);
        p1[r][m] = __builtin_nontemporal_load(c0 + CLN + j);
      }
  };
  if (k < K) fetch(k);
  __syncthreads();  // the twiddle slice is in LDS
  const auto lds_ld = [&](uint32_t, uint32_t pj) { return sm[pj]; };
#pragma unroll 1
  for (; k < K; k += per_combo) {
    uint64_t x[NS1][M1];
#pragma unroll
    for (int r = 0; r < NS1; ++r)
#pragma unroll
      for (int m = 0; m < M1; ++m) {
        const uint64_t a0 = SUM ? red_any(p0[r][m], cst) : p0[r][m];
        x[r][m] = csub_neg(a0 + shoup_lazy(p1[r][m], sv[r][m], sw[r][m], q), n4q);
      }
    if (k + per_combo < K) fetch(k + per_combo);  // lands while this ciphertext is transformed
#pragma unroll
    for (int r = 0; r < NS1; ++r) {  // first chunk: stages i < K1 of the contiguous sets
      const uint32_t g = first_g(r);
#pragma unroll
      for (int i = 0; i < K1; ++i) {
        const int hm = 1 << i;
        const ulonglong2* tw = tws + (1u << (BL - 1 - i)) + (g << (K1 - 1 - i));
#pragma unroll
        for (int gs = 0; gs < (M1 >> (i + 1)); ++gs) {
          const ulonglong2 W = tw[gs];
#pragma unroll
          for (int mm = 0; mm < hm; ++mm) {
            if (gs_in8<false>(i, mm))
              gs_bfly_b<true>(x[r][gs * 2 * hm + mm], x[r][gs * 2 * hm + mm + hm], W.x, W.y, q, n8q);
            else
              gs_bfly_b<false>(x[r][gs * 2 * hm + mm], x[r][gs * 2 * hm + mm + hm], W.x, W.y, q, n8q);
          }
        }
      }
      if (!WL) {
        const uint32_t pj0 = lpad(g << K1);
#pragma unroll
        for (int m = 0; m < M1; ++m) sm[pj0 + lofs<1>(m)] = x[r][m];
      }
    }
    if (WL) {
      // the previous ciphertext's last-chunk reads (every wave's) must be done before this wave
      // refills its sub-block; the first chunk above already ran in registers meanwhile
      __syncthreads();
#pragma unroll
      for (int r = 0; r < NS1; ++r) {
        const uint32_t pj0 = lpad(first_g(r) << K1);
#pragma unroll
        for (int m = 0; m < M1; ++m) sm[pj0 + lofs<1>(m)] = x[r][m];
      }
      wave_lds_sync();
    } else {
      __syncthreads();
    }
    inv_chunk_ct<BL, K1, K2, true>(tws, q, n8q, lds_ld, [&](int, uint32_t, uint32_t pj0, auto& y) {
#pragma unroll
      for (int m = 0; m < (1 << K2); ++m) sm[pj0 + lofs<(1 << K1)>(m)] = y[m];
    });
    if (WL)
      wave_lds_sync();
    else
      __syncthreads();
    inv_chunk_ct<BL, K1 + K2, K3, true>(tws, q, n8q, lds_ld, [&](int, uint32_t, uint32_t pj0, auto& y) {
#pragma unroll
      for (int m = 0; m < (1 << K3); ++m) sm[pj0 + lofs<(1 << (K1 + K2))>(m)] = y[m];
    });
    __syncthreads();
    uint64_t* __restrict__ dst = dbuf + (uint64_t)k * LN + off;
    inv_chunk_ct<BL, BL - K4, K4, true>(tws, q, n8q, lds_ld, [&](int, uint32_t j0, uint32_t, auto& y) {
#pragma unroll
      for (int m = 0; m < (1 << K4); ++m) dst[j0 + (m << (BL - K4))] = y[m];
    });
    if (!WL) __syncthreads();  // sm is rewritten by the next ciphertext's first chunk
  }
}

// Wave-local exchanges in the persistent block passes (the default since round 4; SHELFI_NTT_WL=0
// keeps the four-barrier form): bit-identical, decrypt 2-3% and flooded decrypt ~2% faster, encrypt
// within 1% (profiles/r04r/wl_ab*.txt).
static bool ntt_wave_local() { return switches().ntt_wl; }

// Workgroups of the persistent decrypt / encrypt block passes: LDS-bound residency per CU
// times the CUs, spread evenly over the (tower, block) combos (at least one each).
static uint32_t pp_per_combo(uint32_t ncombo, uint64_t K, uint32_t per_cu) {
  static const uint32_t cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    return (uint32_t)n;
  }();
  uint64_t pc = (uint64_t)cus * per_cu / ncombo;
  if (pc < 1) pc = 1;
  if (pc > K) pc = K;
  return (uint32_t)pc;
}

// Inverse blocks pass: small half-sizes first (LDS), then the top LOGR stages on
// register columns (ntt_inv_cols), scaled by N^-1 in the last pass.
// With ct != nullptr the input is decrypt's c0 + c1*s (ckks.cpp:189), formed while
// filling LDS from the ciphertext batch [K][2][L][N] (poly p = k*L + t).
__global__ __launch_bounds__(256) void ntt_inv_blocks(uint64_t* __restrict__ polys, uint32_t L,
                                                      uint32_t logN, uint32_t blkLog,
                                                      const uint64_t* __restrict__ tw,
                                                      const uint64_t* __restrict__ twp,
                                                      const TowerConst* __restrict__ tcs,
                                                      int scale_ninv,
                                                      const uint64_t* __restrict__ ct,
                                                      const uint64_t* __restrict__ sk,
                                                      const uint64_t* __restrict__ sksh, int sum_in,
                                                      uint32_t ctL) {
  extern __shared__ __attribute__((aligned(16))) uint64_t sm[];
  const uint32_t N = 1u << logN, blk = 1u << blkLog;
  const uint32_t sh = logN - blkLog, nb = 1u << sh;
  const uint64_t poly = blockIdx.x >> sh;
  const uint32_t b = blockIdx.x & (nb - 1);
  const uint32_t t = (uint32_t)(poly % L);
  const TowerConst& c = tcs[t];
  const uint64_t q = c.q;
  uint64_t* __restrict__ a = polys + poly * N + ((uint64_t)b << blkLog);
  if (ct) {
    const uint64_t kk = poly / L, off = ((uint64_t)t << logN) + ((uint64_t)b << blkLog);
    const ulonglong2* c0 = reinterpret_cast<const ulonglong2*>(ct + (kk * 2 * ctL << logN) + off);
    const ulonglong2* c1 = reinterpret_cast<const ulonglong2*>(ct + ((kk * 2 + 1) * ctL << logN) + off);
    const ulonglong2* s = reinterpret_cast<const ulonglong2*>(sk + off);
    const ulonglong2* ss = reinterpret_cast<const ulonglong2*>(sksh + off);
    for (uint32_t p = threadIdx.x; p < blk / 2; p += 256) {
      ulonglong2 x0 = c0[p];
      const ulonglong2 x1 = c1[p], sv = s[p], sw = ss[p];
      if (sum_in) x0 = make_ulonglong2(red64(x0.x, q, c.one_shoup), red64(x0.y, q, c.one_shoup));
      lds_put2(sm, p, make_ulonglong2(addmod(x0.x, shoup_mul(x1.x, sv.x, sw.x, q), q),
                                      addmod(x0.y, shoup_mul(x1.y, sv.y, sw.y, q), q)));
    }
  } else {
    for (uint32_t p = threadIdx.x; p < blk / 2; p += 256)
      lds_put2(sm, p, reinterpret_cast<const ulonglong2*>(a)[p]);
  }
  __syncthreads();
  ntt_inv_block_stages(sm, blkLog, b, logN, tw + (uint64_t)t * N, twp + (uint64_t)t * N, q);
  if (scale_ninv) {
    const uint64_t ni = c.ninv, nip = c.ninv_shoup;
    for (uint32_t p = threadIdx.x; p < blk / 2; p += 256) {
      const ulonglong2 v = lds_get2(sm, p);
      reinterpret_cast<ulonglong2*>(a)[p] = make_ulonglong2(canon4(shoup_lazy(v.x, ni, nip, q), q),
                                                            canon4(shoup_lazy(v.y, ni, nip, q), q));
    }
  } else {  // lazy values in [0, 4q): the columns pass canonicalises
    for (uint32_t p = threadIdx.x; p < blk / 2; p += 256)
      reinterpret_cast<ulonglong2*>(a)[p] = lds_get2(sm, p);
  }
}

template <int LOGR>
__global__ __launch_bounds__(256) void ntt_inv_cols(uint64_t* __restrict__ polys, uint32_t L,
                                                    uint32_t logN, const uint64_t* __restrict__ tw,
                                                    const uint64_t* __restrict__ twp,
                                                    const TowerConst* __restrict__ tcs) {
  constexpr int R = 1 << LOGR;
  const uint32_t N = 1u << logN;
  const uint32_t BLK = N >> LOGR;
  const uint32_t bpp = BLK / 256;
  const uint64_t poly = blockIdx.x / bpp;
  const uint32_t col = (blockIdx.x % bpp) * 256 + threadIdx.x;
  const uint32_t t = (uint32_t)(poly % L);
  const TowerConst& c = tcs[t];
  const uint64_t q = c.q;
  const uint64_t* __restrict__ w = tw + (uint64_t)t * N;
  const uint64_t* __restrict__ wp = twp + (uint64_t)t * N;
  uint64_t* __restrict__ a = polys + poly * N + col;
  uint64_t x[R];
#pragma unroll
  for (int r = 0; r < R; ++r) x[r] = a[(uint64_t)r * BLK];
#pragma unroll
  for (int v = 0; v < LOGR; ++v) {
    const int tr = 1 << v, h = R >> (v + 1);
#pragma unroll
    for (int i = 0; i < h; ++i) {
      const uint64_t W = w[h + i], Wp = wp[h + i];
#pragma unroll
      for (int jj = 0; jj < tr; ++jj) {
        const int r0 = 2 * i * tr + jj, r1 = r0 + tr;
        if (gs_in8<true>(v, jj))  // inputs below 8q (ntt_inv_blocks_dec_ct leaves sums < 8q)
          gs_bfly_b<true>(x[r0], x[r1], W, Wp, q, c.n8q);
        else
          gs_bfly_b<false>(x[r0], x[r1], W, Wp, q, c.n8q);
      }
    }
  }
  const uint64_t ni = c.ninv, nip = c.ninv_shoup;
#pragma unroll
  for (int r = 0; r < R; ++r) a[(uint64_t)r * BLK] = canon4(shoup_lazy(x[r], ni, nip, q), q);
}

#define NTT_DISPATCH(LOGRV, KERNEL, ...)                                                   \
  switch (LOGRV) {                                                                       \
    case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break;                           \
    case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;                           \
    case 3: hipLaunchKernelGGL(KERNEL<3>, __VA_ARGS__); break;                           \
    case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;                           \
    case 5: hipLaunchKernelGGL(KERNEL<5>, __VA_ARGS__); break;                           \
    case 6: hipLaunchKernelGGL(KERNEL<6>, __VA_ARGS__); break;                           \
    default: throw Error{SHELFI_ERR_ARG, "unsupported ring dimension"};                  \
  }

// launch_ntt's block passes at compile-time shape (rings with a columns pass whose blocks are
// 2^11 or 2^12 elements and every q >= 2^40), in place over the per-block twiddle slices:
// forward after ntt_fwd_cols (inputs < 8q, canonical outputs), inverse before ntt_inv_cols
// (canonical inputs, lazy outputs below 8q).  A workgroup reads its whole block in the first
// chunk, before any of its writes.
template <int BL, int K1, int K2, int K3, int K4>
__global__ __launch_bounds__(256) void ntt_fwd_blocks_ct(uint64_t* polys, uint32_t L, uint32_t logN,
                                                         const ulonglong2* __restrict__ twb,
                                                         const TowerConst* __restrict__ tcs) {
  __shared__ __attribute__((aligned(16))) uint64_t sm[lpad_size(BL)];
  const uint32_t sh = logN - BL;
  const uint64_t poly = blockIdx.x >> sh;
  const uint32_t b = blockIdx.x & ((1u << sh) - 1);
  const uint32_t t = (uint32_t)(poly % L);
  const TowerConst& c = tcs[t];
  uint64_t* base = polys + (poly << logN) + ((uint64_t)b << BL);
  fwd_block_pass_ct<BL, K1, K2, K3, K4>(base, twb + ((uint64_t)t << logN) + ((uint64_t)b << BL), c.q, c.n8q, sm,
                                        [&](uint32_t j0, auto& x) {
#pragma unroll
                                          for (int m = 0; m < (1 << K4); m += 2)
                                            *reinterpret_cast<ulonglong2*>(base + j0 + m) =
                                                make_ulonglong2(red_any(x[m], c), red_any(x[m + 1], c));
                                        });
}
template <int BL, int K1, int K2, int K3, int K4>
__global__ __launch_bounds__(256) void ntt_inv_blocks_ct(uint64_t* polys, uint32_t L, uint32_t logN,
                                                         const ulonglong2* __restrict__ twb,
                                                         const TowerConst* __restrict__ tcs) {
  static_assert(K1 + K2 + K3 + K4 == BL, "chunk plan must cover the block");
  __shared__ __attribute__((aligned(16))) uint64_t sm[lpad_size(BL)];
  const uint32_t sh = logN - BL;
  const uint64_t poly = blockIdx.x >> sh;
  const uint32_t b = blockIdx.x & ((1u << sh) - 1);
  const uint32_t t = (uint32_t)(poly % L);
  const uint64_t q = tcs[t].q, n8q = tcs[t].n8q;
  uint64_t* base = polys + (poly << logN) + ((uint64_t)b << BL);
  const ulonglong2* __restrict__ tb = twb + ((uint64_t)t << logN) + ((uint64_t)b << BL);
  const auto lds_ld = [&](uint32_t, uint32_t pj) { return sm[pj]; };
  inv_chunk_ct<BL, 0, K1, false>(tb, q, n8q, [&](uint32_t j, uint32_t) { return base[j]; },
                                 [&](int, uint32_t, uint32_t pj0, auto& x) {
#pragma unroll
                                   for (int m = 0; m < (1 << K1); ++m) sm[pj0 + lofs<1>(m)] = x[m];
                                 });
  __syncthreads();
  inv_chunk_ct<BL, K1, K2, true>(tb, q, n8q, lds_ld, [&](int, uint32_t, uint32_t pj0, auto& x) {
#pragma unroll
    for (int m = 0; m < (1 << K2); ++m) sm[pj0 + lofs<(1 << K1)>(m)] = x[m];
  });
  __syncthreads();
  inv_chunk_ct<BL, K1 + K2, K3, true>(tb, q, n8q, lds_ld, [&](int, uint32_t, uint32_t pj0, auto& x) {
#pragma unroll
    for (int m = 0; m < (1 << K3); ++m) sm[pj0 + lofs<(1 << (K1 + K2))>(m)] = x[m];
  });
  __syncthreads();
  inv_chunk_ct<BL, BL - K4, K4, true>(tb, q, n8q, lds_ld, [&](int, uint32_t j0, uint32_t, auto& x) {
#pragma unroll
    for (int m = 0; m < (1 << K4); ++m) base[j0 + (m << (BL - K4))] = x[m];
  });
}

void launch_ntt(uint64_t* polys, uint64_t P, uint32_t L, uint32_t logN, bool inverse,
                const DeviceTables& dt, hipStream_t s) {
  if (!P) return;
  const uint32_t N = 1u << logN;
  const uint32_t blkLog = ntt_block_log(logN);
  const int logR = (int)(logN - blkLog);
  const uint32_t blk = 1u << blkLog;
  const size_t lds = (size_t)blk * sizeof(uint64_t);
  const uint64_t nbBlocks = P << logR;
  const uint64_t nbCols = P * ((N >> logR) / 256);
  if (nbBlocks > 0x7FFFFFFFull || nbCols > 0x7FFFFFFFull)
    throw Error{SHELFI_ERR_ARG, "NTT batch too large"};
  if (!inverse) {
    if (logR > 0) {
      NTT_DISPATCH(logR, ntt_fwd_cols, dim3((uint32_t)nbCols), dim3(256), 0, s, polys, L, logN,
                   dt.psi_rev, dt.psi_rev_sh, dt.tc);
    }
    if (logR > 0 && blkLog == 11 && dt.red_ok)
      hipLaunchKernelGGL((ntt_fwd_blocks_ct<11, 3, 3, 3, 2>), dim3((uint32_t)nbBlocks), dim3(256), 0, s, polys, L,
                         logN, dt.tw_fwd_blk, dt.tc);
    else if (logR > 0 && blkLog == 12 && dt.red_ok)
      hipLaunchKernelGGL((ntt_fwd_blocks_ct<12, 3, 3, 3, 3>), dim3((uint32_t)nbBlocks), dim3(256), 0, s, polys, L,
                         logN, dt.tw_fwd_blk, dt.tc);
    else
      hipLaunchKernelGGL(ntt_fwd_blocks, dim3((uint32_t)nbBlocks), dim3(256), lds, s, polys, L,
                         logN, (uint32_t)logR, dt.psi_rev, dt.psi_rev_sh, dt.tc);
  } else {
    if (logR > 0 && blkLog == 11 && dt.red_ok)
      hipLaunchKernelGGL((ntt_inv_blocks_ct<11, 2, 3, 3, 3>), dim3((uint32_t)nbBlocks), dim3(256), 0, s, polys, L,
                         logN, dt.tw_inv_blk, dt.tc);
    else if (logR > 0 && blkLog == 12 && dt.red_ok)
      hipLaunchKernelGGL((ntt_inv_blocks_ct<12, 3, 3, 3, 3>), dim3((uint32_t)nbBlocks), dim3(256), 0, s, polys, L,
                         logN, dt.tw_inv_blk, dt.tc);
    else
      hipLaunchKernelGGL(ntt_inv_blocks, dim3((uint32_t)nbBlocks), dim3(256), lds, s, polys, L,
                         logN, blkLog, dt.ipsi_rev, dt.ipsi_rev_sh, dt.tc, logR == 0 ? 1 : 0,
                         (const uint64_t*)nullptr, (const uint64_t*)nullptr, (const uint64_t*)nullptr, 0, L);
    if (logR > 0) {
      NTT_DISPATCH(logR, ntt_inv_cols, dim3((uint32_t)nbCols), dim3(256), 0, s, polys, L, logN,
                   dt.ipsi_rev, dt.ipsi_rev_sh, dt.tc);
    }
  }
  SHELFI_HIP(hipGetLastError());
}

// The register-columns pass alone (the first logN - BL forward stages / the last inverse
// stages), for callers that fuse their own blocks pass (keyswitch.hip).  No-op when the
// whole transform is one block (N <= 2^BL).
void launch_ntt_cols(uint64_t* polys, uint64_t P, uint32_t L, uint32_t logN, bool inverse,
                     const DeviceTables& dt, hipStream_t s) {
  const uint32_t N = 1u << logN;
  const int logR = (int)(logN - ntt_block_log(logN));
  if (!P || logR == 0) return;
  const uint64_t nbCols = P * ((N >> logR) / 256);
  if (nbCols > 0x7FFFFFFFull) throw Error{SHELFI_ERR_ARG, "NTT batch too large"};
  if (!inverse)
    NTT_DISPATCH(logR, ntt_fwd_cols, dim3((uint32_t)nbCols), dim3(256), 0, s, polys, L, logN, dt.psi_rev,
                 dt.psi_rev_sh, dt.tc)
  else
    NTT_DISPATCH(logR, ntt_inv_cols, dim3((uint32_t)nbCols), dim3(256), 0, s, polys, L, logN, dt.ipsi_rev,
                 dt.ipsi_rev_sh, dt.tc)
  SHELFI_HIP(hipGetLastError());
}

// ------------------------------------------------------- special FFT (f64) ----
// FFTSpecialInv (encode): DIF stages len = S..2 with twiddle finv[len/2 + (x mod
// len)], then BitReverse and /S (both folded into enc_prep).  First LOGR stages
// on register columns (reading the learner's real vector directly), the rest in
// LDS blocks of 2^fft_block_log(logS) complex values.
template <int LOGR>
__global__ __launch_bounds__(256) void fft_inv_cols(const double* __restrict__ x, uint64_t n,
                                                    double2* __restrict__ buf, uint32_t logS,
                                                    const double2* __restrict__ tw) {
  constexpr int R = 1 << LOGR;
  const uint32_t S = 1u << logS;
  const uint32_t BLK = S >> LOGR;
  const uint32_t bpp = BLK / 256;
  const uint64_t k = blockIdx.x / bpp;
  const uint32_t col = (blockIdx.x % bpp) * 256 + threadIdx.x;
  double2 v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t gi = k * S + col + (uint64_t)r * BLK;
    v[r] = make_double2(gi < n ? x[gi] : 0.0, 0.0);
  }
#pragma unroll
  for (int s = 0; s < LOGR; ++s) {
    const uint32_t len = S >> s, lenh = len >> 1;
    const int trr = R >> (s + 1);
#pragma unroll
    for (int r0 = 0; r0 < R; ++r0) {
      if ((r0 / trr) % 2) continue;
      const int r1 = r0 + trr;
      // (col + r0 BLK) mod len, written so rows sharing a twiddle share its load
      const uint32_t j = col + (uint32_t)(r0 & ((R >> s) - 1)) * BLK;
      const double2 W = tw[lenh + j];
      const double2 u = cadd(v[r0], v[r1]);
      const double2 d = csub(v[r0], v[r1]);
      v[r0] = u;
      v[r1] = cmul(d, W);
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) buf[k * S + col + (uint64_t)r * BLK] = v[r];
}

__global__ __launch_bounds__(256) void fft_inv_blocks(const double* __restrict__ x, uint64_t n,
                                                      double2* __restrict__ buf, uint32_t logS,
                                                      uint32_t blkLog, int from_x,
                                                      const double2* __restrict__ tw) {
  extern __shared__ __attribute__((aligned(16))) double2 smc[];
  const uint32_t S = 1u << logS, blk = 1u << blkLog;
  const uint32_t sh = logS - blkLog;
  const uint64_t k = blockIdx.x >> sh;
  const uint32_t b = blockIdx.x & ((1u << sh) - 1);
  const uint64_t off = k * S + ((uint64_t)b << blkLog);
  for (uint32_t i = threadIdx.x; i < blk; i += 256) {
    if (from_x) {
      const uint64_t gi = off + i;
      smc[i] = make_double2(gi < n ? x[gi] : 0.0, 0.0);
    } else {
      smc[i] = buf[off + i];
    }
  }
  __syncthreads();
  for (uint32_t len = blk; len >= 2; len >>= 1) {
    const uint32_t lenh = len >> 1;
    for (uint32_t p = threadIdx.x; p < blk / 2; p += 256) {
      const uint32_t j = p & (lenh - 1);
      const uint32_t i0 = (p - j) * 2 + j;
      const double2 W = tw[lenh + j];
      const double2 a0 = smc[i0], a1 = smc[i0 + lenh];
      smc[i0] = cadd(a0, a1);
      smc[i0 + lenh] = cmul(csub(a0, a1), W);
    }
    __syncthreads();
  }
  for (uint32_t i = threadIdx.x; i < blk; i += 256) buf[off + i] = smc[i];
}

// Compile-time forms of the FFT block passes (round 3): the same butterflies, in the same order
// per element, as fft_fwd_blocks / fft_inv_blocks, but run as register chunks of 2^KC
// elements (a set j0 + m 2^A, m < 2^KC, covers the stages of half-size 2^A .. 2^(A+KC-1)) with
// the LDS block exchanged only between chunks: 3 barriers instead of 10-11, the first chunk
// loaded and the last chunk stored straight from registers.  Bit-identical outputs.
template <int KC, int A>
__device__ __forceinline__ void fft_dit_set(double2 (&v)[1 << KC], uint32_t l, const double2* __restrict__ tw) {
#pragma unroll
  for (int i = 0; i < KC; ++i) {  // half-size 2^(A+i), ascending (DIT)
#pragma unroll
    for (int m0 = 0; m0 < (1 << KC); ++m0) {
      if (m0 & (1 << i)) continue;
      const int m1 = m0 + (1 << i);
      const double2 W = tw[(1u << (A + i)) + l + ((uint32_t)(m0 & ((1 << i) - 1)) << A)];
      const double2 u = v[m0];
      const double2 w = cmul(v[m1], W);
      v[m0] = cadd(u, w);
      v[m1] = csub(u, w);
    }
  }
}
template <int KC, int A>
__device__ __forceinline__ void fft_dif_set(double2 (&v)[1 << KC], uint32_t l, const double2* __restrict__ tw) {
#pragma unroll
  for (int i = KC - 1; i >= 0; --i) {  // half-size 2^(A+i), descending (DIF)
#pragma unroll
    for (int m0 = 0; m0 < (1 << KC); ++m0) {
      if (m0 & (1 << i)) continue;
      const int m1 = m0 + (1 << i);
      const double2 W = tw[(1u << (A + i)) + l + ((uint32_t)(m0 & ((1 << i) - 1)) << A)];
      const double2 a0 = v[m0], a1 = v[m1];
      v[m0] = cadd(a0, a1);
      v[m1] = cmul(csub(a0, a1), W);
    }
  }
}
// One chunk over all 2^(BL-KC) sets of a block, 2^(BL-3) threads: ld(j) / st(j, v) take block
// offsets.
template <int BL, int KC, int A, bool DIT, class Load, class Store>
__device__ __forceinline__ void fft_chunk(const double2* __restrict__ tw, Load ld, Store st) {
  constexpr int T = 1 << (BL - 3), NS = (1 << (BL - KC)) / T;
  static_assert(NS >= 1, "chunk plan");
#pragma unroll
  for (int r = 0; r < NS; ++r) {
    const uint32_t s = threadIdx.x + (uint32_t)T * r;
    const uint32_t l = s & ((1u << A) - 1), j0 = ((s >> A) << (A + KC)) | l;
    double2 v[1 << KC];
#pragma unroll
    for (int m = 0; m < (1 << KC); ++m) v[m] = ld(j0 + ((uint32_t)m << A));
    if (DIT)
      fft_dit_set<KC, A>(v, l, tw);
    else
      fft_dif_set<KC, A>(v, l, tw);
#pragma unroll
    for (int m = 0; m < (1 << KC); ++m) st(j0 + ((uint32_t)m << A), v[m]);
  }
}
// The LDS block of the FFT chunk passes is XOR-swizzled (round 4): element j lives at
// j ^ ((j >> 3) & 15), a bijection of every aligned 128-element group.  A chunk at stride 2^A hands
// lane l the elements j0(l) + m 2^A; with A = 0 (the DIT pass's first chunk, 8 consecutive elements
// per lane) every lane of a ds_write_b128 group hit the same 16-B slot mod 128 B (8-way), and the
// DIF pass's A = 2 and A = 0 chunks hit 4 slots per 16-lane ds_read_b128 group.  Counted per
// instruction by a model of the chunk addresses and the gfx950 lane groups (MI355X_MICROARCH.md
// §LDS), which reproduces the measured SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS of round 3 exactly
// (10.0 for fft_fwd_blocks_ct<10,...>, 5.33 for fft_inv_blocks_ct<10,...>): swizzled, 0 and 1.33
// (the DIF A = 2 chunk's stores keep a 2-way conflict), and 0 for both BL = 11 passes.
template <bool SWZ = true>
__device__ __forceinline__ uint32_t fft_swz(uint32_t j) { return SWZ ? j ^ ((j >> 3) & 15u) : j; }

// FFTSpecialInv's second pass (encode, after fft_inv_cols): DIF half-sizes 2^(BL-1) .. 1.
template <int BL, int K1, int K2, int K3, int K4, bool SWZ = true>
__global__ __launch_bounds__(1 << (BL - 3)) void fft_inv_blocks_ct(double2* __restrict__ buf, uint32_t logS,
                                                                  const double2* __restrict__ tw) {
  static_assert(K1 + K2 + K3 + K4 == BL, "chunk plan");
  __shared__ __attribute__((aligned(16))) double2 sm[1 << BL];
  const uint32_t S = 1u << logS, sh = logS - BL;
  const uint64_t k = blockIdx.x >> sh;
  const uint32_t b = blockIdx.x & ((1u << sh) - 1);
  double2* __restrict__ g = buf + k * S + ((uint64_t)b << BL);
  const auto lds_ld = [&](uint32_t j) { return sm[fft_swz<SWZ>(j)]; };
  const auto lds_st = [&](uint32_t j, double2 v) { sm[fft_swz<SWZ>(j)] = v; };
  fft_chunk<BL, K1, BL - K1, false>(tw, [&](uint32_t j) { return g[j]; }, lds_st);
  __syncthreads();
  fft_chunk<BL, K2, BL - K1 - K2, false>(tw, lds_ld, lds_st);
  __syncthreads();
  fft_chunk<BL, K3, BL - K1 - K2 - K3, false>(tw, lds_ld, lds_st);
  __syncthreads();
  fft_chunk<BL, K4, 0, false>(tw, lds_ld, [&](uint32_t j, double2 v) { g[j] = v; });
}

// Whole-vector FFT passes (round 5): one 1024-thread workgroup per ciphertext at 2^14 slots holds the
// vector in registers (16 complex values per thread), so the columns and blocks passes share one
// launch and the [K][S] intermediate never goes through HBM (encode: 1.18 -> 0.39 MB per ciphertext;
// decode: 0.92 -> 0.39).  The same butterflies on the same operands as fft_inv_cols<4> +
// fft_inv_blocks_ct<10, ...> (fft_fwd_blocks_ct<10, ...> + fft_fwd_cols<4>): bit-identical outputs.
// Rows <-> blocks go through LDS one component at a time (16 x 1088 doubles = 136 KiB, one workgroup
// per CU); inside a block, a wave exchanges its own 1024 elements (8 KiB) with no workgroup barrier.
// LDS layouts.  Padded rows (not an XOR swizzle) keep each thread's 16 addresses at compile-time offsets
// from one base: an XOR swizzle's 32 live addresses spilled under the 128-VGPR cap of 1024-thread
// workgroups.  Each exchange has its own padding, chosen with a model of the ds_read_b64 (2 x 32 lanes, 64
// banks) and ds_write_b64 / read2 (4 x 16 lanes, 32 banks) groups of MI355X_MICROARCH.md §LDS so that both
// of its access shapes are conflict-free (one shared padding left 2-way conflicts: SQ_LDS_BANK_CONFLICT 3.4
// cycles per LDS instruction in fft_inv_whole, profiles/r05p):
//   blocks <-> rows transposes and the flooding statistics, e + (e >> 5)   (fft_wpad, fft_wt1, fft_wx3)
//   exchanges between 4 s + m and 64 (s >> 2) + (s & 3) + 4 m, e + (e >> 4)     (fft_xa1, fft_xa2)
//   exchanges between 64 (s >> 2) + (s & 3) + 4 m and s + 64 m, e + 2 (e >> 5)  (fft_xb2, fft_xb3)
// The closed forms below are those paddings of the set shapes 4 (l + 64 q) + r (m = 4 q + r),
// 64 (l >> 2) + (l & 3) + 4 m and l + 64 m, for lane l and register m.
constexpr uint32_t kFftWholeLogS = 14;
// One 1024-thread workgroup per vector fills the chip only for batches of hundreds of ciphertexts: below
// kFftWholeMinK the multi-pass FFTs (many workgroups per vector) are faster -- at K = 4 / 16 / 64 encrypt
// 21.3 / 6.9 / 3.70 vs 24.9 / 7.7 / 3.73 us/ct, decrypt 10.5 / 3.5 / 1.53 vs 13.7 / 4.2 / 1.64; at K = 256
// the whole-vector kernels win, 2.93 vs 2.97 and 0.99 vs 1.03 (profiles/r05zc/small_k.txt)
constexpr uint64_t kFftWholeMinK = 128;
constexpr uint64_t kEncNoredMinK = 192;  // launch_encrypt: the NORED tower split from this many ciphertexts
// launch_decrypt: the persistent first INTT pass (ntt_inv_blocks_dec_pp) from this many (ciphertext, decode
// tower, 2^11 block) items, the one-shot ntt_inv_blocks_dec_ct below.  Decrypt / flooded us/ct, one-shot vs
// persistent (profiles/r06f/dpk_*, ppk_*): 2^15 / 3 decode towers K = 4 9.96 / 12.53 vs 10.37 / 13.07, K = 64
// (3,072 items) 1.52 / 1.75 vs 1.55 / 1.82, K = 96 (4,608) 1.53 / 1.67 vs 1.43 / 1.55; 2^16 K = 32 (3,072)
// 3.17-3.28 / 3.59-3.70 vs 3.30 / 3.73, K = 64 (6,144) 3.00 / 3.19 vs 2.76-2.84 / 2.92
constexpr uint64_t kDecPpMinItems = 4096;
constexpr uint32_t kFftWholeRow = 1088;  // doubles per 1024-element block slice (the largest padding, 1087)
__device__ __forceinline__ uint32_t fft_wpad(uint32_t e) { return e + (e >> 5); }
__device__ __forceinline__ uint32_t fft_wt1(uint32_t l, int m) { return 4 * l + (l >> 3) + 264u * (m >> 2) + (m & 3); }
__device__ __forceinline__ uint32_t fft_wx3(uint32_t l, int m) { return l + (l >> 5) + 66u * m; }
__device__ __forceinline__ uint32_t fft_xa1(uint32_t l, int m) { return 4 * l + (l >> 2) + 272u * (m >> 2) + (m & 3); }
__device__ __forceinline__ uint32_t fft_xa2(uint32_t l, int m) { return 68 * (l >> 2) + (l & 3) + 4u * m + (m >> 2); }
__device__ __forceinline__ uint32_t fft_xb2(uint32_t l, int m) {
  return 68 * (l >> 2) + (l & 3) + 4u * m + 2u * (m >> 3);
}
__device__ __forceinline__ uint32_t fft_xb3(uint32_t l, int m) { return l + 2 * (l >> 5) + 68u * m; }

// A wave's exchange inside its block's 1024 elements: a[m] (at padded block position P(m)) -> a[m] (at
// Q(m)), real parts first, then imaginary parts, through the wave's LDS slice.
template <class PF, class QF>
__device__ __forceinline__ void fft_wave_xch(double2 (&a)[16], double* __restrict__ Ls, PF P, QF Q) {
#pragma unroll
  for (int m = 0; m < 16; ++m) Ls[P(m)] = a[m].x;
  wave_lds_sync();
#pragma unroll
  for (int m = 0; m < 16; ++m) a[m].x = Ls[Q(m)];
  wave_lds_sync();
#pragma unroll
  for (int m = 0; m < 16; ++m) Ls[P(m)] = a[m].y;
  wave_lds_sync();
#pragma unroll
  for (int m = 0; m < 16; ++m) a[m].y = Ls[Q(m)];
  wave_lds_sync();
}

// Rows (thread T holds row r's column T in a[r]) <-> blocks (wave w holds block w's element l + 64 m in
// a[m]) through the workgroup's 16 x 1024-double LDS, one component at a time.  TO_BLOCKS: rows -> blocks.
template <bool TO_BLOCKS>
__device__ __forceinline__ void fft_whole_transpose(double2 (&a)[16], double* __restrict__ lds) {
  const uint32_t T = threadIdx.x, w = T >> 6, l = T & 63;
#pragma unroll
  for (int part = 0; part < 2; ++part) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const double v = part ? a[i].y : a[i].x;
      if (TO_BLOCKS)
        lds[i * kFftWholeRow + fft_wpad(T)] = v;
      else
        lds[w * kFftWholeRow + fft_wx3(l, i)] = v;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const double v = TO_BLOCKS ? lds[w * kFftWholeRow + fft_wx3(l, i)] : lds[i * kFftWholeRow + fft_wpad(T)];
      if (part)
        a[i].y = v;
      else
        a[i].x = v;
    }
    __syncthreads();
  }
}

// FFTSpecialInv (encode) of one 2^14-slot vector per workgroup: x (n doubles, zero-padded) -> buf [K][S].
__global__ __launch_bounds__(1024) void fft_inv_whole(const double* __restrict__ x, uint64_t n,
                                                      double2* __restrict__ buf, const double2* __restrict__ tw) {
  constexpr uint32_t S = 1u << kFftWholeLogS, BLK = 1024;
  constexpr int R = 16;
  __shared__ double lds[16 * kFftWholeRow];
  const uint64_t k = blockIdx.x;
  const uint32_t T = threadIdx.x, w = T >> 6, l = T & 63;
  double2 a[R];
  // columns: DIF stages len S .. S/8 on column T (fft_inv_cols<4>)
  const double* __restrict__ xk = x + k * S;
  const uint32_t rem = n > k * S ? (uint32_t)std::min<uint64_t>(n - k * S, S) : 0u;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t i = T + (uint32_t)r * BLK;
    a[r] = make_double2(i < rem ? xk[i] : 0.0, 0.0);
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    asm volatile("" ::: "memory");  // each stage's twiddle loads stay in the stage (fft_fwd_whole)
    const uint32_t lenh = (S >> s) >> 1;
    const int trr = R >> (s + 1);
#pragma unroll
    for (int r0 = 0; r0 < R; ++r0) {
      if ((r0 / trr) % 2) continue;
      const int r1 = r0 + trr;
      const double2 W = tw[lenh + T + (uint32_t)(r0 & ((R >> s) - 1)) * BLK];
      const double2 u = cadd(a[r0], a[r1]);
      const double2 d = csub(a[r0], a[r1]);
      a[r0] = u;
      a[r1] = cmul(d, W);
    }
  }
  fft_whole_transpose<true>(a, lds);
  // block w: DIF half-sizes 512 .. 64 on set l (elements l + 64 m), 32 .. 4 on set l (elements
  // 64 (l >> 2) + (l & 3) + 4 m), 2 .. 1 on sets l + 64 q (elements 4 (l + 64 q) + m)
  double* Ls = lds + w * kFftWholeRow;
  fft_dif_set<4, 6>(a, l, tw);
  fft_wave_xch(a, Ls, [&](int m) { return fft_xb3(l, m); }, [&](int m) { return fft_xb2(l, m); });
  fft_dif_set<4, 2>(a, l & 3, tw);
  fft_wave_xch(a, Ls, [&](int m) { return fft_xa2(l, m); }, [&](int m) { return fft_xa1(l, m); });
  double2* __restrict__ g = buf + k * S + (uint64_t)w * BLK;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    double2 c[4] = {a[4 * q], a[4 * q + 1], a[4 * q + 2], a[4 * q + 3]};
    fft_dif_set<2, 0>(c, 0u, tw);
#pragma unroll
    for (int m = 0; m < 4; ++m) g[4 * (l + 64 * q) + m] = c[m];
  }
}

// FFTSpecial (decode): input already bit-reversed by crt_decode's scatter; DIT
// stages len = 2..S with twiddle ffwd[len/2 + (x mod len)].  Small len in LDS
// blocks, the top LOGR stages on register columns; the last pass writes the real
// parts of the first `n` slots straight into the caller's output vector.
// fft_fwd_blocks (the first FFTSpecial pass) is defined with the decode-noise flooding
// below, which it can fuse into its load.

#define FFT_DISPATCH(LOGRV, KERNEL, ...)                                                   \
  switch (LOGRV) {                                                                       \
    case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break;                           \
    case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;                           \
    case 3: hipLaunchKernelGGL(KERNEL<3>, __VA_ARGS__); break;                           \
    case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;                           \
    case 5: hipLaunchKernelGGL(KERNEL<5>, __VA_ARGS__); break;                           \
    case 6: hipLaunchKernelGGL(KERNEL<6>, __VA_ARGS__); break;                           \
    default: throw Error{SHELFI_ERR_ARG, "unsupported batch size"};                      \
  }


// -------------------------------------------------------------- encrypt ----
// One thread = sample group h of a ciphertext: the 16 coefficients j = h + (N/16) i of the
// v2 sampler stream (dev_common.h), so every store is a coalesced row.
// m_j = llround(FFTinv(x)[bitrev(i)] / S * Delta) at j = i*gap (real part) and
// N/2 + i*gap (imaginary part) (CKKSPackedEncoding::Encode layout).  Output is the
// compact per-coefficient record {int64 m + e0, int16 (e1 << 8) | (uint8)v} — 10 bytes
// instead of the 3 L residues the NTT needs, which ntt_fwd_cols_enc expands per tower.
__device__ __forceinline__ void load_cdt32(const uint64_t* __restrict__ cdt, int T, uint32_t* hi, uint32_t* lo) {
  if (threadIdx.x < 64) {
    const uint64_t v = (int)threadIdx.x < T ? cdt[threadIdx.x] : ~0ull;
    hi[threadIdx.x] = (int)threadIdx.x < T ? (uint32_t)(v >> 32) : 0xFFFFFFFFu;
    lo[threadIdx.x] = (uint32_t)v;
  }
}

// Encode's range flag (GenFlag words): [0] = a |x Delta| above 2^61 (a finite one: the call is redone on
// the large-value path, launch_encrypt_approx), [1] = a non-finite value (refused).
__device__ __forceinline__ void gen_flag_set(GenFlag f, int word) {
  __hip_atomic_store(f.p + word, f.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void enc_range_flag(GenFlag f, double val) {
  gen_flag_set(f, 0);
  if (!isfinite(val)) gen_flag_set(f, 1);
}

__global__ __launch_bounds__(256) void enc_prep_kernel(const double2* __restrict__ fbuf,
                                                       uint64_t K, uint32_t logN, uint32_t logS,
                                                       double delta,
                                                       const uint64_t* __restrict__ cdt, int T,
                                                       Key8 key, uint64_t g0,
                                                       int64_t* __restrict__ me0,
                                                       int16_t* __restrict__ ve,
                                                       GenFlag flag) {
  const uint32_t N = 1u << logN, S = 1u << logS, N16 = N >> 4, V0 = N >> 6;
  __shared__ uint32_t thi[64], tlo[64];
  load_cdt32(cdt, T, thi, tlo);
  __syncthreads();
  const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t k = gid >> (logN - 4);
  if (k >= K) return;
  const uint32_t h = (uint32_t)(gid & (N16 - 1));
  const uint64_t nonce = (1ull << 56) | (g0 + k);
  const uint32_t half = N >> 1, gapLog = logN - 1 - logS;
  const double dS = (double)S;
  const double lim = 2305843009213693952.0;  // 2^61: beyond, the call is redone by launch_encrypt_approx
  uint32_t w[16];
  chacha20_block32(key, h >> 2, nonce, w);
  uint32_t u[4] = {w[4 * (h & 3)], w[4 * (h & 3) + 1], w[4 * (h & 3) + 2], w[4 * (h & 3) + 3]};
  int32_t vv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) vv[i] = (int32_t)trit_next(u) - 1;
  chacha20_block32(key, V0 + h, nonce, w);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t j = h + N16 * i;
    const uint32_t jj = j < half ? j : j - half;
    int64_t m = 0;
    if ((jj & ((1u << gapLog) - 1)) == 0) {
      const double2 cv = fbuf[k * S + bitrev_dev(jj >> gapLog, logS)];
      const double val = __dmul_rn(__ddiv_rn(j < half ? cv.x : cv.y, dS), delta);
      if (!(fabs(val) <= lim)) enc_range_flag(flag, val);
      m = round_half_away(val);
    }
    me0[(k << logN) + j] = m + gauss32(w[i], thi, tlo, [&] { return chacha20_word(key, V0 + 2 * N16 + h, nonce, i); });
  }
  chacha20_block32(key, V0 + N16 + h, nonce, w);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int32_t e1 =
        (int32_t)gauss32(w[i], thi, tlo, [&] { return chacha20_word(key, V0 + 3 * N16 + h, nonce, i); });
    ve[(k << logN) + h + N16 * i] = (int16_t)((e1 << 8) | (vv[i] & 0xFF));
  }
}

// Encrypt's first NTT pass reading the compact sample record (enc_prep_kernel):
// thread = column c of ciphertext k, coefficients j = c + BLK r.  For every tower the
// three polynomials v, m + e0, e1 are reduced, run through the first LOGR stages and
// stored lazily ([0, 8q)) into pbuf [K][3][L][N] for ntt_fwd_blocks_enc.
template <int LOGR, int POLY>
__global__ __launch_bounds__(256) void ntt_fwd_cols_enc(const int64_t* __restrict__ me0,
                                                        const int16_t* __restrict__ ve, uint64_t K,
                                                        uint32_t logN, uint32_t L,
                                                        const TowerConst* __restrict__ tcs,
                                                        const uint64_t* __restrict__ tw,
                                                        const uint64_t* __restrict__ twp,
                                                        uint64_t* __restrict__ out) {
  constexpr int R = 1 << LOGR;
  const uint32_t BLK = (1u << logN) >> LOGR;
  const uint32_t bpp = BLK / 256;
  const uint64_t k = blockIdx.x / bpp;
  if (k >= K) return;
  const uint32_t c = (blockIdx.x % bpp) * 256 + threadIdx.x;
  const uint64_t LN = (uint64_t)L << logN;
  const uint64_t j0 = (k << logN) + c;
  // POLY: 0 = v, 1 = m + e0, 2 = e1 (one launch each).  The record is re-read for every
  // tower (L1/L2 hits) rather than kept live beside the R residues: keeping R int64
  // sources across the tower loop cost 2 waves/SIMD of occupancy (170 VGPRs).
#pragma unroll 1
  for (uint32_t t = 0; t < L; ++t) {
    const TowerConst cst = tcs[t];
    const uint64_t q = cst.q;
    const uint64_t* __restrict__ w = tw + ((uint64_t)t << logN);
    const uint64_t* __restrict__ wp = twp + ((uint64_t)t << logN);
    uint64_t x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t j = j0 + (uint64_t)BLK * r;
      if (POLY == 1) {
        x[r] = mod_signed_dev(me0[j], cst);
        if ((r & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // bound reductions in flight
      } else {
        const int32_t sv = ve[j];
        x[r] = small_mod(POLY == 0 ? (int32_t)(int8_t)(sv & 0xFF) : (sv >> 8), q);
      }
    }
#pragma unroll
    for (int s = 0; s < LOGR; ++s) {
      const int m = 1 << s, tr = R >> (s + 1);
#pragma unroll
      for (int i = 0; i < m; ++i) {
        const uint64_t W = w[m + i], Wp = wp[m + i];
#pragma unroll
        for (int jj = 0; jj < tr; ++jj) {
          const int r0 = 2 * i * tr + jj, r1 = r0 + tr;
          if (fwd_red_at(s))
            ct_bfly_s<true>(x[r0], x[r1], W, Wp, q, cst.n8q);
          else
            ct_bfly_s<false>(x[r0], x[r1], W, Wp, q, cst.n8q);
        }
      }
    }
    uint64_t* __restrict__ o = out + (k * 3 + POLY) * LN + ((uint64_t)t << logN) + c;
    // the blocks passes take inputs below 8q
#pragma unroll
    for (int r = 0; r < R; ++r) o[(uint64_t)r * BLK] = fwd_bound(LOGR) > 8 ? csub_neg(x[r], cst.n8q) : x[r];
  }
}

// Encode + sampling + the columns pass in one kernel (enc_prep_kernel followed by the three
// ntt_fwd_cols_enc launches, without the 10-byte-per-coefficient record in between):
// thread = column c of ciphertext k, coefficients j = c + BLK r (r < R = 2^LOGR).  In the v2
// sampler stream (dev_common.h) coefficient j = h + (N/16) i: the column's rows are the sample
// indices i = i0 + (16/R) r of group h = c mod N/16 (i0 = c div N/16; LOGR = 4: the whole group).
// Same samples and rounding as enc_prep_kernel, then for every tower the columns stages of v,
// m + e0 and e1 and the lazy stores into pbuf that the blocks pass reads.
// WV: waves per SIMD the register budget is cut for.  TWL: the tower's column-stage twiddles are
// staged in LDS per tower instead of scalar-loaded (the scalar loads of 15 {w, w'} pairs per polynomial
// were spilling SGPRs).
// TS (round 4, small batches): wave w of a workgroup takes tower w (L = 4) of 64 columns, each wave
// sampling its columns itself (4x the sampler work, no cross-wave traffic): a K = 4 call's 8192
// columns become 512 waves instead of 128, for calls too small to fill the chip one column per thread
// (register budget for 2 waves per SIMD: a small call has no more to give it).
// VT (round 5; LOGR = 4, TAB, not TS): v's columns pass is left to the blocks pass, which sums
// DeviceTables::enc_vtab entries for each row; this kernel writes only the column's 4 radix-4 group
// patterns, packed 7 bits each into one uint32 at word c of the ciphertext's pbuf v region (8 KiB per
// ciphertext instead of v's 4 towers x 256 KiB).
// X5 (round 6; LOGR = 4, not TS / VT): one more columns stage for rings whose blocks pass starts at
// global stage 5 (2^16 over 2^11 blocks, nlogR = 5).  A workgroup's threads hold columns c (tid < 128)
// and c + BLK/2 (tid >= 128) of the 16-row decomposition; stage 4 pairs row r of the two (twiddle
// psi_rev[16 + r]), so after the register stages each thread trades 8 rows with its partner through
// LDS and runs 8 of the 16 butterflies: the low thread keeps rows 0-7 of both columns, the high one
// rows 8-15.  pbuf then holds what a 32-row columns pass leaves, without 32-row register columns.
template <int LOGR, bool TAB, int WV = 4, bool TWL = false, bool TS = false, bool VT = false, bool X5 = false>
__global__ __launch_bounds__(256, TS ? 2 : WV) void enc_cols_fused(const double2* __restrict__ fbuf, uint64_t K,
                                                      uint32_t logN, uint32_t logS, uint32_t L,
                                                      double delta, const uint64_t* __restrict__ cdt,
                                                      int T, Key8 key, uint64_t g0,
                                                      const TowerConst* __restrict__ tcs,
                                                      const uint64_t* __restrict__ tw,
                                                      const uint64_t* __restrict__ twp,
                                                      uint64_t* __restrict__ out,
                                                      GenFlag flag, uint32_t t_split,
                                                      const uint64_t* __restrict__ enc_tab) {
  constexpr int R = 1 << LOGR, IS = 16 / R, G = R / 4;
  constexpr int NTW = TS ? 4 : 1;  // towers with their own LDS tables in one workgroup
  static_assert(LOGR == 3 || LOGR == 4, "a column is 8 or 16 rows of one sample group");
  static_assert(!VT || (LOGR == 4 && TAB && !TS), "v tables: 16-row columns, one column per thread");
  static_assert(!X5 || (LOGR == 4 && TAB && !TS && !VT), "the exchanged stage: 16-row columns, one per thread");
  constexpr int NTWL = X5 ? 2 << LOGR : 1 << LOGR;  // column-stage twiddles psi_rev[1 .. NTWL)
  __shared__ uint32_t thi[64], tlo[64];
  __shared__ uint64_t tabs_all[NTW][kEncTab];  // the tower's DeviceTables::enc_tab slice
  __shared__ ulonglong2 twl_all[NTW][NTWL];  // TWL: the tower's {w, w'} for column stages (index m + i)
  __shared__ uint64_t xch[X5 ? 8 * 256 : 1];   // X5: the 8 rows a thread trades, [row][thread]
  static_assert(!TWL || TAB, "LDS twiddles ride on the table path's per-tower barrier");
  const uint32_t wave = TS ? (threadIdx.x >> 6) : 0u, tid = TS ? (threadIdx.x & 63u) : threadIdx.x;
  uint64_t* tabs = tabs_all[wave];
  ulonglong2* twl = twl_all[wave];
  // TS: each wave's tables are its own, so ordering its LDS writes before its reads needs no barrier
  const auto tower_sync = [] {
    if (TS)
      wave_lds_sync();
    else
      __syncthreads();
  };
  load_cdt32(cdt, T, thi, tlo);
  __syncthreads();
  const uint32_t N = 1u << logN, BLK = N >> LOGR, N16 = N >> 4, V0 = N >> 6;
  const uint64_t gid = TS ? (uint64_t)blockIdx.x * 64 + tid : (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t k = gid >> (logN - LOGR);
  if (k >= K) return;  // workgroup-uniform (BLK is a multiple of 256)
  // X5: workgroup wi of a ciphertext holds column pairs (wi 128 + l, wi 128 + l + BLK/2), l < 128
  const uint32_t c = X5 ? (((uint32_t)(gid & (BLK - 1)) >> 8) << 7) + (threadIdx.x & 127u) +
                              ((threadIdx.x >> 7) ? (BLK >> 1) : 0u)
                        : (uint32_t)(gid & (BLK - 1));
  const uint32_t h = c & (N16 - 1), i0 = c >> (logN - 4);
  const uint64_t nonce = (1ull << 56) | (g0 + k);
  const uint32_t S = 1u << logS, gapLog = logN - 1 - logS;
  const double invS = 1.0 / (double)S;  // a power of two: x * (1/S) == x / S exactly
  const double lim = 2305843009213693952.0;  // 2^61: beyond, the call is redone by launch_encrypt_approx
  const uint64_t LN = (uint64_t)L << logN;
  // columns stages of one polynomial of tower t (values x[r] < q) and its lazy store
  // (towers with q < kNoRedQ run unreduced (NORED, fwd_set_ct): no stage reductions, no
  // store reduction; the blocks pass knows)
  // (first: the stage the values enter at; the small polynomials skip stages their tables did)
  auto cols = [&](uint64_t (&x)[R], uint32_t t, const TowerConst& cst, int poly, auto nored, auto first)
                  __attribute__((always_inline)) {
    constexpr bool NR = decltype(nored)::value;
    const uint64_t q = cst.q;
    const uint64_t* __restrict__ w = tw + ((uint64_t)t << logN);
    const uint64_t* __restrict__ wp = twp + ((uint64_t)t << logN);
#pragma unroll
    for (int s = decltype(first)::value; s < LOGR; ++s) {
      const int m = 1 << s, tr = R >> (s + 1);
#pragma unroll
      for (int i = 0; i < m; ++i) {
        uint64_t W, Wp;
        if constexpr (TWL) {
          const ulonglong2 T2 = twl[m + i];
          W = T2.x;
          Wp = T2.y;
        } else {
          W = w[m + i];
          Wp = wp[m + i];
        }
#pragma unroll
        for (int jj = 0; jj < tr; ++jj) {
          const int r0 = 2 * i * tr + jj, r1 = r0 + tr;
          if (!NR && fwd_red_at(s))
            ct_bfly_s<true>(x[r0], x[r1], W, Wp, q, cst.n8q);
          else
            ct_bfly_s<false>(x[r0], x[r1], W, Wp, q, cst.n8q);
        }
      }
    }
    uint64_t* __restrict__ o = out + (k * 3 + poly) * LN + ((uint64_t)t << logN) + c;
    if constexpr (X5) {
      // stage LOGR: row r of column c (low thread) with row r of c + BLK/2 (high thread), twiddle
      // psi_rev[R + r]; each keeps 8 rows of both columns
      const bool lo = threadIdx.x < 128;  // wave-uniform
      __syncthreads();                    // the previous exchange's reads are done
      // (explicit wave-uniform branches: a select between two register elements becomes a select
      // of addresses, which puts the array in scratch)
      if (lo) {
#pragma unroll
        for (int r = 0; r < R / 2; ++r) xch[r * 256 + threadIdx.x] = x[R / 2 + r];
      } else {
#pragma unroll
        for (int r = 0; r < R / 2; ++r) xch[r * 256 + threadIdx.x] = x[r];
      }
      __syncthreads();
      uint64_t y[R / 2];
#pragma unroll
      for (int r = 0; r < R / 2; ++r) y[r] = xch[r * 256 + (threadIdx.x ^ 128u)];
      constexpr bool RD = fwd_red_at(LOGR);
      const uint32_t rb = lo ? 0u : (uint32_t)(R / 2);  // this thread's rows rb .. rb + 7
      const int64_t dpart = lo ? (int64_t)(BLK >> 1) : -(int64_t)(BLK >> 1);  // the partner column
#pragma unroll
      for (int r = 0; r < R / 2; ++r) {
        uint64_t W, Wp;
        if constexpr (TWL) {
          const ulonglong2 T2 = twl[R + rb + r];
          W = T2.x;
          Wp = T2.y;
        } else {
          W = w[R + rb + r];
          Wp = wp[R + rb + r];
        }
        // low: (x[r], y[r]) = (c, c + BLK/2) at row r; high: (y[r], x[8 + r]) = (c - BLK/2, c) at row 8 + r
        // (wave-uniform branches with static register indices)
        if (lo)
          ct_bfly_s<!NR && RD>(x[r], y[r], W, Wp, q, cst.n8q);
        else
          ct_bfly_s<!NR && RD>(y[r], x[R / 2 + r], W, Wp, q, cst.n8q);
      }
      const auto fin = [&](uint64_t v) { return (!NR && fwd_bound(LOGR + 1) > 8) ? csub_neg(v, cst.n8q) : v; };
      if (lo) {
#pragma unroll
        for (int r = 0; r < R / 2; ++r) {
          o[(uint64_t)r * BLK] = fin(x[r]);          // own column
          o[(uint64_t)r * BLK + dpart] = fin(y[r]);  // the partner's column
        }
      } else {
#pragma unroll
        for (int r = 0; r < R / 2; ++r) {
          o[(uint64_t)(R / 2 + r) * BLK] = fin(x[R / 2 + r]);
          o[(uint64_t)(R / 2 + r) * BLK + dpart] = fin(y[r]);
        }
      }
      return;
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
      o[(uint64_t)r * BLK] = (!NR && fwd_bound(LOGR) > 8) ? csub_neg(x[r], cst.n8q) : x[r];
  };
  // phase 1: v (16 digits of a 128-bit word group) and e1, packed (e1 << 8) | (uint8) v
  {
    int32_t sv[R];
    {
      // block h/4 is shared by the quad of lanes h & ~3 .. h | 3 (h mod 4 = lane mod 4)
      uint32_t u[4];
      chacha20_quad(key, h >> 2, nonce, u);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int32_t d = (int32_t)trit_next(u) - 1;
        if (IS == 1) {
          sv[i] = d & 0xFF;
        } else if ((i % IS) == 0) {
          if (i0 == 0) sv[i / IS] = d & 0xFF;
        } else if (i0 == 1) {
          sv[i / IS] = d & 0xFF;
        }
      }
    }
    {
      uint32_t we[16];
      chacha20_block32(key, V0 + N16 + h, nonce, we);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint32_t i = IS == 1 ? (uint32_t)r : i0 + IS * r;
        const uint32_t wi = IS == 1 ? we[r] : (i0 ? we[IS * r + 1] : we[IS * r]);  // no dynamic register index
        sv[r] |= (int32_t)gauss32(wi, thi, tlo, [&] { return chacha20_word(key, V0 + 3 * N16 + h, nonce, i); }) << 8;
      }
    }
    // v's first two column stages are table lookups: rows g, g + R/4, g + R/2, g + 3R/4 (g < R/4)
    // form a radix-4 group whose 4 outputs depend only on its 4 ternary inputs (81 patterns,
    // DeviceTables::enc_tab, canonical); e1's stage 0 reads W0 e from the table (|e| <= 63).
    // The canonical ciphertext is the same; only lazy intermediates differ (smaller bounds).
    uint32_t vidx[G];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const auto tr = [&](int r) { return (uint32_t)((int32_t)(int8_t)(sv[r] & 0xFF) + 1); };
      vidx[g] = tr(g) + 3 * tr(g + G) + 9 * tr(g + 2 * G) + 27 * tr(g + 3 * G);
    }
    if constexpr (VT)
      reinterpret_cast<uint32_t*>(out + k * 3 * LN)[c] = vidx[0] | (vidx[1] << 7) | (vidx[2] << 14) | (vidx[3] << 21);
    // towers [0, t_split) reduced, [t_split, L) unreduced (q < kNoRedQ; the blocks pass knows)
    const auto small_polys = [&](uint32_t ta, uint32_t tb, auto nored) __attribute__((always_inline)) {
#pragma unroll 1
      for (uint32_t t = ta; t < tb; ++t) {
        if (TS && t != wave) continue;  // wave-uniform
        const TowerConst cst = tcs[t];
        if constexpr (!TAB) {  // A/B reference: every stage as butterflies (SHELFI_ENC_TAB=0)
#pragma unroll 1
          for (int poly = 0; poly < 3; poly += 2) {
            uint64_t x[R];
#pragma unroll
            for (int r = 0; r < R; ++r)
              x[r] = small_mod(poly == 0 ? (int32_t)(int8_t)(sv[r] & 0xFF) : (sv[r] >> 8), cst.q);
            cols(x, t, cst, poly, nored, std::integral_constant<int, 0>{});
          }
          continue;
        }
        tower_sync();  // the previous tower's lookups are done (every thread runs every tower)
        for (uint32_t i = tid; i < (uint32_t)kEncTab; i += (TS ? 64u : 256u)) tabs[i] = enc_tab[(size_t)t * kEncTab + i];
        if constexpr (TWL) {
          if (tid < (uint32_t)NTWL)
            twl[tid] = make_ulonglong2(tw[((uint64_t)t << logN) + tid], twp[((uint64_t)t << logN) + tid]);
        }
        tower_sync();
        if constexpr (!VT) {
          uint64_t x[R];
#pragma unroll
          for (int g = 0; g < G; ++g)
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) x[g + kk * G] = tabs[kk * 81 + vidx[g]];
          cols(x, t, cst, 0, nored, std::integral_constant<int, 2>{});
        }
        {
          uint64_t x[R];
#pragma unroll
          for (int r = 0; r < R / 2; ++r) {
            const uint64_t xa = small_mod(sv[r] >> 8, cst.q);
            const uint64_t tt = tabs[kEncVTab + 64 + (sv[r + R / 2] >> 8)];  // W0 e mod q
            x[r] = xa + tt;                   // < 2q
            x[r + R / 2] = xa + cst.q - tt;   // (0, 2q)
          }
          cols(x, t, cst, 2, nored, std::integral_constant<int, 1>{});
        }
      }
    };
    small_polys(0, t_split, std::false_type{});
    small_polys(t_split, L, std::true_type{});
  }
  // phase 2: m + e0; rows r and r + R/2 are the real and imaginary parts of one slot
  int64_t me[R];
  {
    uint32_t we[16];
    chacha20_block32(key, V0 + h, nonce, we);
#pragma unroll
    for (int r = 0; r < R / 2; ++r) {
      const uint32_t jj = c + BLK * r;  // < N/2
      int64_t mre = 0, mim = 0;
      if ((jj & ((1u << gapLog) - 1)) == 0) {
        const double2 cv = fbuf[k * S + bitrev_dev(jj >> gapLog, logS)];
        const double vr = __dmul_rn(__dmul_rn(cv.x, invS), delta);
        const double vi = __dmul_rn(__dmul_rn(cv.y, invS), delta);
        if (!(fabs(vr) <= lim) || !(fabs(vi) <= lim)) {
          gen_flag_set(flag, 0);
          if (!isfinite(vr) || !isfinite(vi)) gen_flag_set(flag, 1);
        }
        mre = round_half_away(vr);
        mim = round_half_away(vi);
      }
#pragma unroll
      for (int part = 0; part < 2; ++part) {
        const int rr = r + part * (R / 2);
        const uint32_t i = IS == 1 ? (uint32_t)rr : i0 + IS * rr;
        const uint32_t wi = IS == 1 ? we[rr] : (i0 ? we[IS * rr + 1] : we[IS * rr]);
        me[rr] = (part ? mim : mre) +
                 gauss32(wi, thi, tlo, [&] { return chacha20_word(key, V0 + 2 * N16 + h, nonce, i); });
      }
    }
  }
  // The first columns stage pairs rows r and r + R/2 and reads the upper row only through its
  // lazy Shoup product, which takes any 64-bit multiplicand: rows >= R/2 enter as
  // u = m + e0 + floor(2^62 / q) q (in [0, 2^63), congruent), and only rows < R/2 are reduced
  // (red_any, q >= 2^40).  The canonical ciphertext is the same; only lazy intermediates differ.
  const auto message_poly = [&](uint32_t ta, uint32_t tb, auto nored) __attribute__((always_inline)) {
#pragma unroll 1
    for (uint32_t t = ta; t < tb; ++t) {
      if (TS && t != wave) continue;  // wave-uniform
      if constexpr (TWL) {
        tower_sync();  // every thread runs every tower
        if (tid < (uint32_t)NTWL)
          twl[tid] = make_ulonglong2(tw[((uint64_t)t << logN) + tid], twp[((uint64_t)t << logN) + tid]);
        tower_sync();
      }
      const TowerConst cst = tcs[t];
      uint64_t x[R];
      if (cst.red_ok) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint64_t u = (uint64_t)me[r] + cst.bq62;
          x[r] = r < R / 2 ? red_any(u, cst) : u;
        }
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          x[r] = mod_signed_dev(me[r], cst);
          if ((r & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // bound reductions in flight
        }
      }
      cols(x, t, cst, 1, nored, std::integral_constant<int, 0>{});
    }
  };
  message_poly(0, t_split, std::false_type{});
  message_poly(t_split, L, std::true_type{});
}

// enc_cols_fused's tower-split form up to this many ciphertexts per call: K = 4 21.1 vs 24.6 us/ct,
// K = 16 6.7 vs 7.3, but K = 64 4.1 vs 3.3 and K = 714 3.5 vs 2.6 (profiles/r04u/ts_k*.txt)
constexpr uint64_t kEncTsMaxK = 24;

size_t encrypt_scratch_bytes(const Params& p, uint64_t K) {
  // FFT buffer | pbuf [K][3][L][N] | me0 [K][N] int64 | ve [K][N] int16 | the large-value path's
  // per-ciphertext max, exponent and 2^logApprox mod q_t (launch_encrypt_approx)
  return K * (uint64_t)p.batch * sizeof(double2) + K * 3ull * p.L * p.N * sizeof(uint64_t) +
         K * (uint64_t)p.N * (sizeof(int64_t) + sizeof(int16_t)) + K * (8 + 8 + 16ull * p.L) + 64;
}

// encode's FFTSpecialInv of K slot vectors (x: n doubles, zero-padded) into fbuf [K][S] (complex)
static void launch_encode_fft(const Params& p, const DeviceTables& dt, const double* x, uint64_t n, uint64_t K,
                              double2* fbuf, hipStream_t s) {
  const uint32_t logS = __builtin_ctz(p.batch);
  const uint32_t blkLog = fft_block_log(logS);
  const int logR = (int)(logS - blkLog);
  const size_t lds = sizeof(double2) << blkLog;
  if (logS == kFftWholeLogS && K >= kFftWholeMinK && switches().fft_whole) {  // a workgroup per vector
    hipLaunchKernelGGL(fft_inv_whole, dim3((uint32_t)K), dim3(1024), 0, s, x, n, fbuf, dt.fft_inv);
  } else if (logR > 0) {
    const uint64_t nb = K * ((p.batch >> logR) / 256);
    FFT_DISPATCH(logR, fft_inv_cols, dim3((uint32_t)nb), dim3(256), 0, s, x, n, fbuf, logS,
                 dt.fft_inv);
    const bool fct = switches().fft_ct;
    if (fct && blkLog == 10)
      hipLaunchKernelGGL((fft_inv_blocks_ct<10, 3, 3, 2, 2>), dim3((uint32_t)(K << logR)), dim3(128), 0, s, fbuf,
                         logS, dt.fft_inv);
    else if (fct && blkLog == 11)
      hipLaunchKernelGGL((fft_inv_blocks_ct<11, 3, 3, 3, 2>), dim3((uint32_t)(K << logR)), dim3(256), 0, s, fbuf,
                         logS, dt.fft_inv);
    else
      hipLaunchKernelGGL(fft_inv_blocks, dim3((uint32_t)(K << logR)), dim3(256), lds, s, x, n, fbuf,
                         logS, blkLog, 0, dt.fft_inv);
  } else {
    hipLaunchKernelGGL(fft_inv_blocks, dim3((uint32_t)K), dim3(256), lds, s, x, n, fbuf, logS,
                       blkLog, 1, dt.fft_inv);
  }
  SHELFI_HIP(hipGetLastError());
}

void launch_encrypt(const Params& p, const DeviceTables& dt, const DeviceKeys& dk, const double* x,
                    uint64_t n, uint64_t K, uint64_t* ct, void* scratch, const uint32_t key[8],
                    uint64_t g0, GenFlag flag, hipStream_t s) {
  if (!K) return;
  const uint32_t logS = __builtin_ctz(p.batch);
  double2* fbuf = reinterpret_cast<double2*>(scratch);
  uint64_t* pbuf = reinterpret_cast<uint64_t*>(fbuf + K * (uint64_t)p.batch);
  // 1. FFTSpecialInv of each ciphertext's slot vector
  launch_encode_fft(p, dt, x, n, K, fbuf, s);
  Key8 k8;
  for (int i = 0; i < 8; ++i) k8.k[i] = key[i];
  const Switches& sw = switches();
  const uint32_t nblkLog = ntt_block_log(p.logN);
  const int nlogR = (int)(p.logN - nblkLog);
  // nlogR = 5 (2^16 over 2^11 blocks, 2^17): the 16-row kernel with the exchanged fifth stage (X5)
  const bool fused = (nlogR == 3 || nlogR == 4 || (nlogR == 5 && sw.enc_tab && sw.enc_x5)) && dt.enc_tab &&
                     sw.enc_fused;
  int64_t* me0 = reinterpret_cast<int64_t*>(pbuf + K * 3ull * p.L * p.N);
  int16_t* ve = reinterpret_cast<int16_t*>(me0 + K * (uint64_t)p.N);
  // NORED towers (fwd_set_ct): q < kNoRedQ, run unreduced through both passes — only with the
  // persistent blocks pass, and only as a suffix of the chain (q_0 the 60-bit tower, the rest
  // near 2^scale_bits); t_split = L turns it off
  const bool pp = fused && nblkLog == 11 && dt.red_ok && sw.enc_pp;
  uint32_t t_split = 0;
  while (t_split < p.L && p.q[t_split] >= kNoRedQ) ++t_split;
  for (uint32_t t = t_split; t < p.L; ++t)
    if (p.q[t] >= kNoRedQ) t_split = p.L;
  // the two tower classes take one blocks-pass launch each, in series; below kEncNoredMinK ciphertexts a
  // call is latency-bound and one launch over every tower (all reduced) is faster: K = 4 / 16 / 64 / 128
  // encrypt 18.7 / 6.5 / 3.67 / 3.23 vs 21.2 / 6.9 / 3.76 / 3.28 us/ct, K = 256 2.92 vs 2.88
  // (profiles/r05zc/nored_k.txt; tests/test_gpu_switches.py checks both paths bit for bit at K = 200)
  // At 2^16 (nlogR = 5, X5 columns) the split is slower at every K measured: K = 256 / 512 encrypt 8.91 / 8.50
  // us/ct in one reduced launch vs 9.00 / 8.74 split, while 2^15 K = 714 gains 2.75 vs 2.88 (profiles/r06f/nr_*)
  if (!pp || !sw.enc_nored || K < kEncNoredMinK || nlogR == 5) t_split = p.L;
  bool vt = false;  // NTT(v)'s columns pass as enc_vtab sums in the blocks pass (round 5)
  if (fused) {
    // 2+3a. encode + sampling + columns pass of v, m + e0, e1 for every tower
    const uint64_t nb = (K << (p.logN - (nlogR == 5 ? 4 : nlogR))) / 256;
    const bool tab = sw.enc_tab;
    // LDS column twiddles at 3 waves/SIMD with the tables (no SGPR / VGPR spills): enc_cols_fused 578 ->
    // 534 us per 714 cts (probes/r03_enc_cols_twl.txt; the scalar-loaded form was removed in round 5)
#define ENC_COLS(LR, TB, ...)                                                                                   \
  hipLaunchKernelGGL((enc_cols_fused<LR, TB, ##__VA_ARGS__>), dim3((uint32_t)nb), dim3(256), 0, s, fbuf, K, p.logN, logS, p.L, \
                     p.delta, dt.cdt, dt.cdt_len, k8, g0, dt.tc, dt.psi_rev, dt.psi_rev_sh, pbuf, flag, t_split,  \
                     dt.enc_tab)
    // small calls (K <= kEncTsMaxK at 4 towers): one wave per tower (TS), so a call of a few
    // ciphertexts spreads over 4x the waves; SHELFI_ENC_TS=0 / 1 forces either (A/B switch)
    const bool ts = nlogR == 4 && tab && p.L == 4 && (sw.enc_ts >= 0 ? sw.enc_ts == 1 : K <= kEncTsMaxK);
    vt = pp && tab && !ts && nlogR == 4 && dt.enc_vtab && sw.enc_vt && ntt_wave_local();
    // X5: 16 register rows + the exchanged fifth stage (10 VGPRs spilled at 3 waves / SIMD; the
    // spill-free 2-wave build ran 3-4% slower, profiles/r06b)
    if (nlogR == 5)
      ENC_COLS(4, true, 3, true, false, false, true);
    else if (vt)  // v's columns pass left to the blocks pass (enc_vtab sums)
      ENC_COLS(4, true, 3, true, false, true);
    else if (ts)
      hipLaunchKernelGGL((enc_cols_fused<4, true, 3, true, true>), dim3((uint32_t)(nb * 4)), dim3(256), 0, s, fbuf, K,
                         p.logN, logS, p.L, p.delta, dt.cdt, dt.cdt_len, k8, g0, dt.tc, dt.psi_rev, dt.psi_rev_sh,
                         pbuf, flag, t_split, dt.enc_tab);
    else if (nlogR == 3 && tab)
      ENC_COLS(3, true);
    else if (nlogR == 3)
      ENC_COLS(3, false);
    else if (tab)  // 164 VGPRs without spills at 3 waves (4 would spill 36)
      ENC_COLS(4, true, 3, true);
    else
      ENC_COLS(4, false);
#undef ENC_COLS
    SHELFI_HIP(hipGetLastError());
  } else {
    // 2. encode (scale/round) + sampling -> compact record
    const uint64_t threads = K * (p.N / 16);  // one per v2 sample group
    hipLaunchKernelGGL(enc_prep_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s, fbuf,
                       K, p.logN, logS, p.delta, dt.cdt, dt.cdt_len, k8, g0, me0, ve, flag);
    SHELFI_HIP(hipGetLastError());
  }
  // 3. NTT of v, m + e0, e1 per tower (columns pass expands the record), then the
  // blocks pass fused with the public-key combine writes the ciphertexts
  if (nlogR > 0 && !fused) {
    const uint64_t nb = K * ((p.N >> nlogR) / 256);
#define COLS_ENC(LR)                                                                          \
  hipLaunchKernelGGL((ntt_fwd_cols_enc<LR, 0>), dim3((uint32_t)nb), dim3(256), 0, s, me0, ve, K,  \
                     p.logN, p.L, dt.tc, dt.psi_rev, dt.psi_rev_sh, pbuf);                       \
  hipLaunchKernelGGL((ntt_fwd_cols_enc<LR, 1>), dim3((uint32_t)nb), dim3(256), 0, s, me0, ve, K,  \
                     p.logN, p.L, dt.tc, dt.psi_rev, dt.psi_rev_sh, pbuf);                       \
  hipLaunchKernelGGL((ntt_fwd_cols_enc<LR, 2>), dim3((uint32_t)nb), dim3(256), 0, s, me0, ve, K,  \
                     p.logN, p.L, dt.tc, dt.psi_rev, dt.psi_rev_sh, pbuf);
    switch (nlogR) {
      case 1: COLS_ENC(1) break;
      case 2: COLS_ENC(2) break;
      case 3: COLS_ENC(3) break;
      case 4: COLS_ENC(4) break;
      case 5: COLS_ENC(5) break;
      case 6: COLS_ENC(6) break;
      default: throw Error{SHELFI_ERR_ARG, "unsupported ring dimension"};
    }
#undef COLS_ENC
    SHELFI_HIP(hipGetLastError());
  }
  const uint64_t nbb = K * p.L << nlogR;
  if (nbb > 0x7FFFFFFFull) throw Error{SHELFI_ERR_ARG, "encrypt batch too large"};
  const uint32_t xg = xcd_combos(p.L << nlogR);
  if (pp) {  // one launch per tower class, each spread over all CUs
    const bool wl = ntt_wave_local();
    const auto launch_pp = [&](uint32_t ta, uint32_t nt, bool nr) {
      const uint32_t ncombo = nt << nlogR;
      const uint32_t pc = pp_per_combo(ncombo, K, 3);
#define ENC_PP(NR, WL, VT)                                                                                       \
  hipLaunchKernelGGL((ntt_fwd_blocks_enc_pp<11, 3, 3, 3, 2, NR, WL, VT>), dim3(ncombo * pc), dim3(256), 0, s, pbuf, \
                     p.L, p.logN, dt.tw_fwd_blk, dt.tc, dk.pk, dk.pk_sh, ct, (uint32_t)K, pc, ta, nt, dt.enc_vtab)
      if (nr && wl && vt) ENC_PP(true, true, true);
      else if (nr && wl) ENC_PP(true, true, false);
      else if (nr) ENC_PP(true, false, false);
      else if (wl && vt) ENC_PP(false, true, true);
      else if (wl) ENC_PP(false, true, false);
      else ENC_PP(false, false, false);
#undef ENC_PP
    };
    if (t_split > 0) launch_pp(0u, t_split, false);
    if (t_split < p.L) launch_pp(t_split, p.L - t_split, true);
  } else if (nlogR > 0 && nblkLog == 11 && dt.red_ok)
    hipLaunchKernelGGL((ntt_fwd_blocks_enc_ct<11, 3, 3, 3, 2>), dim3((uint32_t)nbb), dim3(256), 0, s,
                       pbuf, p.L, p.logN, dt.tw_fwd_blk, dt.tc, dk.pk, dk.pk_sh, ct, 0u, xg);
  else if (nlogR > 0 && nblkLog == 12 && dt.red_ok)
    hipLaunchKernelGGL((ntt_fwd_blocks_enc_ct<12, 3, 3, 3, 3>), dim3((uint32_t)nbb), dim3(256), 0, s,
                       pbuf, p.L, p.logN, dt.tw_fwd_blk, dt.tc, dk.pk, dk.pk_sh, ct, 0u, xg);
  else if (nblkLog > 11)
    hipLaunchKernelGGL(ntt_fwd_blocks_enc<8>, dim3((uint32_t)nbb), dim3(256), sizeof(uint64_t) << nblkLog, s,
                     pbuf, p.L, p.logN, (uint32_t)nlogR, dt.psi_rev, dt.psi_rev_sh, dt.tc, dk.pk,
                     dk.pk_sh, ct, nlogR > 0 ? (const int64_t*)nullptr : me0,
                     nlogR > 0 ? (const int16_t*)nullptr : ve);
  else
    hipLaunchKernelGGL(ntt_fwd_blocks_enc<4>, dim3((uint32_t)nbb), dim3(256), sizeof(uint64_t) << nblkLog, s,
                     pbuf, p.L, p.logN, (uint32_t)nlogR, dt.psi_rev, dt.psi_rev_sh, dt.tc, dk.pk,
                     dk.pk_sh, ct, nlogR > 0 ? (const int64_t*)nullptr : me0,
                     nlogR > 0 ? (const int16_t*)nullptr : ve);
  SHELFI_HIP(hipGetLastError());
}

// ---------------------------------------------- encode's large-value path ----
// PALISADE 1.11 CKKSPackedEncoding::Encode (ckks.cpp:80) scales a slot vector down before rounding when
// its largest coefficient would not fit a 62-bit word [PALISADE-1.11, restated in
// oracle/ckks_oracle.c or_encode_coeffs_ex; parity with PALISADE unpinned]:
//   logc = max over nonzero v_i = FFTSpecialInv(x)_i * Delta of ceil(log2 |v_i|);
//   logApprox = max(0, logc - 62); r_i = llround(v_i / 2^logApprox), wrapped as FitToNativeVector
//   does with Max64BitValue() = 2^63 - 513 (enc_fit_wrap); residue_t = r_i * 2^logApprox mod q_t.
// The fast encrypt kernels handle |v| <= 2^61 (logApprox = 0, no wrap) and flag anything larger;
// the call is then redone here: per-ciphertext max |v| on the device, logApprox from glibc's log2 on
// the host (the function PALISADE calls; one exponent per ciphertext), then the coefficients,
// samples and the 2^logApprox factor written as canonical residues [K][3][L][N], the generic NTT,
// and the public-key combine.  Same ChaCha20 streams as the fast path, so only the message
// coefficients can differ, and only where the fast path refused.
__device__ __forceinline__ int64_t enc_fit_wrap(int64_t r) {
  constexpr int64_t kMax64 = 9223372036854775295LL;  // PALISADE Max64BitValue(): 2^63 - 513
  constexpr int64_t hf = kMax64 >> 1;
  if (r > hf) return r - kMax64;
  if (r < 0 && kMax64 + r <= hf) return r + kMax64;
  return r;
}

// per ciphertext: max |Re|, |Im| of its FFTSpecialInv output, as the bits of a positive double
__global__ __launch_bounds__(256) void enc_maxabs_kernel(const double2* __restrict__ fbuf, uint32_t logS,
                                                         uint64_t* __restrict__ amax) {
  const uint32_t S = 1u << logS;
  const double2* __restrict__ f = fbuf + (uint64_t)blockIdx.x * S;
  uint64_t m = 0;
  for (uint32_t i = threadIdx.x; i < S; i += 256) {
    const double2 v = f[i];
    const uint64_t a = (uint64_t)__double_as_longlong(fabs(v.x)), b = (uint64_t)__double_as_longlong(fabs(v.y));
    m = max(m, max(a, b));
  }
  __shared__ uint64_t red[256];
  red[threadIdx.x] = m;
  __syncthreads();
  for (uint32_t w = 128; w; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) amax[blockIdx.x] = red[0];
}

// thread = sample group h of ciphertext k (enc_prep_kernel's mapping and streams): v, m + e0, e1 as
// canonical residues of every tower into pbuf [K][3][L][N] (COEFFICIENT domain)
__global__ __launch_bounds__(256) void enc_expand_approx_kernel(
    const double2* __restrict__ fbuf, uint64_t K, uint32_t logN, uint32_t logS, uint32_t L, double delta,
    const uint64_t* __restrict__ cdt, int T, Key8 key, uint64_t g0, const TowerConst* __restrict__ tcs,
    const int32_t* __restrict__ log_approx, const uint64_t* __restrict__ pw, uint64_t* __restrict__ pbuf) {
  const uint32_t N = 1u << logN, S = 1u << logS, N16 = N >> 4, V0 = N >> 6;
  __shared__ uint32_t thi[64], tlo[64];
  load_cdt32(cdt, T, thi, tlo);
  __syncthreads();
  const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t k = gid >> (logN - 4);
  if (k >= K) return;
  const uint32_t h = (uint32_t)(gid & (N16 - 1));
  const uint64_t nonce = (1ull << 56) | (g0 + k);
  const uint32_t half = N >> 1, gapLog = logN - 1 - logS;
  const double dS = (double)S;
  const double approx = ldexp(1.0, log_approx[k]);
  uint32_t w[16];
  chacha20_block32(key, h >> 2, nonce, w);
  uint32_t u[4] = {w[4 * (h & 3)], w[4 * (h & 3) + 1], w[4 * (h & 3) + 2], w[4 * (h & 3) + 3]};
  int32_t vv[16], e0[16], e1[16];
  int64_t mm[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) vv[i] = (int32_t)trit_next(u) - 1;
  chacha20_block32(key, V0 + h, nonce, w);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t j = h + N16 * i;
    const uint32_t jj = j < half ? j : j - half;
    int64_t m = 0;
    if ((jj & ((1u << gapLog) - 1)) == 0) {
      const double2 cv = fbuf[k * S + bitrev_dev(jj >> gapLog, logS)];
      const double val = __dmul_rn(__ddiv_rn(j < half ? cv.x : cv.y, dS), delta);
      m = enc_fit_wrap(round_half_away(__ddiv_rn(val, approx)));
    }
    mm[i] = m;
    e0[i] = (int32_t)gauss32(w[i], thi, tlo, [&] { return chacha20_word(key, V0 + 2 * N16 + h, nonce, i); });
  }
  chacha20_block32(key, V0 + N16 + h, nonce, w);
#pragma unroll
  for (int i = 0; i < 16; ++i)
    e1[i] = (int32_t)gauss32(w[i], thi, tlo, [&] { return chacha20_word(key, V0 + 3 * N16 + h, nonce, i); });
  const uint64_t LN = (uint64_t)L << logN;
  for (uint32_t t = 0; t < L; ++t) {
    const TowerConst cst = tcs[t];
    const uint64_t q = cst.q, P = pw[(k * L + t) * 2], Psh = pw[(k * L + t) * 2 + 1];
    uint64_t* __restrict__ o = pbuf + k * 3 * LN + ((uint64_t)t << logN) + h;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint64_t j = (uint64_t)N16 * i;
      o[j] = small_mod(vv[i], q);
      o[LN + j] = addmod(shoup_mul(mod_signed_dev(mm[i], cst), P, Psh, q), small_mod(e0[i], q), q);
      o[2 * LN + j] = small_mod(e1[i], q);
    }
  }
}

// c0 = NTT(v) b + NTT(m + e0), c1 = NTT(v) a + NTT(e1) from canonical EVALUATION residues
__global__ __launch_bounds__(256) void enc_combine_kernel(const uint64_t* __restrict__ pbuf, uint64_t K,
                                                          uint32_t logN, uint32_t L,
                                                          const TowerConst* __restrict__ tcs,
                                                          const uint64_t* __restrict__ pk,
                                                          const uint64_t* __restrict__ pk_sh,
                                                          uint64_t* __restrict__ ct) {
  const uint64_t LN = (uint64_t)L << logN;
  const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (gid >= K * LN) return;
  const uint64_t k = gid / LN, r = gid - k * LN;
  const uint64_t q = tcs[r >> logN].q;
  const uint64_t* __restrict__ b = pbuf + k * 3 * LN;
  const uint64_t V = b[r], M = b[LN + r], E = b[2 * LN + r];
  ct[k * 2 * LN + r] = addmod(shoup_mul(V, pk[r], pk_sh[r], q), M, q);
  ct[k * 2 * LN + LN + r] = addmod(shoup_mul(V, pk[LN + r], pk_sh[LN + r], q), E, q);
}

static uint64_t host_powmod2(uint32_t e, uint64_t q) {
  unsigned __int128 r = 1 % q, b = 2 % q;
  for (; e; e >>= 1) {
    if (e & 1) r = r * b % q;
    b = b * b % q;
  }
  return (uint64_t)r;
}

void launch_encrypt_approx(const Params& p, const DeviceTables& dt, const DeviceKeys& dk, const double* x,
                           uint64_t n, uint64_t K, uint64_t* ct, void* scratch, const uint32_t key[8],
                           uint64_t g0, hipStream_t s) {
  if (!K) return;
  const uint32_t logS = __builtin_ctz(p.batch);
  double2* fbuf = reinterpret_cast<double2*>(scratch);
  uint64_t* pbuf = reinterpret_cast<uint64_t*>(fbuf + K * (uint64_t)p.batch);
  // aux region after me0 / ve (encrypt_scratch_bytes): amax [K] u64 | log_approx [K] i32 (8-aligned) |
  // pw [K][L][2] u64
  uint8_t* aux = reinterpret_cast<uint8_t*>(pbuf + K * 3ull * p.L * p.N) + K * (uint64_t)p.N * 10;
  uint64_t* amax = reinterpret_cast<uint64_t*>(aux);
  int32_t* la_dev = reinterpret_cast<int32_t*>(amax + K);
  uint64_t* pw_dev = amax + K + (K + 1) / 2;
  launch_encode_fft(p, dt, x, n, K, fbuf, s);
  hipLaunchKernelGGL(enc_maxabs_kernel, dim3((uint32_t)K), dim3(256), 0, s, fbuf, logS, amax);
  SHELFI_HIP(hipGetLastError());
  std::vector<uint64_t> hm(K);
  SHELFI_HIP(hipMemcpyAsync(hm.data(), amax, K * 8, hipMemcpyDeviceToHost, s));
  SHELFI_HIP(hipStreamSynchronize(s));
  std::vector<int32_t> la(K);
  std::vector<uint64_t> pw(K * p.L * 2);
  for (uint64_t k = 0; k < K; ++k) {
    double M;
    std::memcpy(&M, &hm[k], 8);
    const double v = (M / (double)p.batch) * p.delta;  // the kernels' (c / S) * Delta, monotone in c
    int logc = 0;
    if (v != 0) logc = std::max(0, (int)std::ceil(std::log2(v)));  // glibc, as Encode calls it
    la[k] = logc > 62 ? logc - 62 : 0;
    for (uint32_t t = 0; t < p.L; ++t) {
      const uint64_t q = p.q[t], w = host_powmod2((uint32_t)la[k], q);
      pw[(k * p.L + t) * 2] = w;
      pw[(k * p.L + t) * 2 + 1] = (uint64_t)(((unsigned __int128)w << 64) / q);
    }
  }
  SHELFI_HIP(hipMemcpyAsync(la_dev, la.data(), K * 4, hipMemcpyHostToDevice, s));
  SHELFI_HIP(hipMemcpyAsync(pw_dev, pw.data(), pw.size() * 8, hipMemcpyHostToDevice, s));
  Key8 k8;
  for (int i = 0; i < 8; ++i) k8.k[i] = key[i];
  const uint64_t threads = K * (p.N / 16);
  hipLaunchKernelGGL(enc_expand_approx_kernel, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s, fbuf, K,
                     p.logN, logS, p.L, p.delta, dt.cdt, dt.cdt_len, k8, g0, dt.tc, la_dev, pw_dev, pbuf);
  SHELFI_HIP(hipGetLastError());
  launch_ntt(pbuf, K * 3ull * p.L, p.L, p.logN, false, dt, s);
  const uint64_t tot = K * (uint64_t)p.L * p.N;
  hipLaunchKernelGGL(enc_combine_kernel, dim3((uint32_t)((tot + 255) / 256)), dim3(256), 0, s, pbuf, K, p.logN, p.L,
                     dt.tc, dk.pk, dk.pk_sh, ct);
  SHELFI_HIP(hipGetLastError());
  SHELFI_HIP(hipStreamSynchronize(s));  // the host tables above are uploaded from pageable memory
}

// One coefficient of the centred CRT over the decode's towers: y(t) in [0, q_t) are
// b_t (Q/q_t)^-1 mod q_t for the L <= 7 towers; X = sum_t y_t (Q/q_t) - k Q with k = round(sum_t
// y_t / q_t), then (double)X * (1/scale) (PALISADE Decode: ConvertToDouble * scalingFactorPre *
// 2^-p), X read as a signed 128-bit integer: (double)|X|_hi 2^64 + (double)|X|_lo with its sign
// (the oracle's or_mw_to_double restricted to two words).
//
// The sum runs in NC 30-bit limb columns (y_t = a + b 2^30; every column is a sum of <= 2L
// products below 2^60 plus k times a 30-bit limb, below 2^64 without carries: one v_mad_u64_u32
// per product), then one carry pass.  NC (DeviceTables::crt_nc) is chosen so that the columns
// hold X' = sum_t y_t (Q/q_t) - k Q exactly in two's complement (|X'| < L Q): whatever k's binary32
// estimate gave, X' is a representative of X mod Q, and it is the centred one exactly when it lies
// in (-2^127, 2^127) -- the value range of this path (round 6).  Bits 127 .. 30 NC - 1 of X' all
// equal is therefore the exact test of "this output is right": otherwise *wide is set and the
// caller redoes the call through crt_exact_kernel over every tower (any |X| <= (Q - 1) / 2, as
// PALISADE's BigInteger decode).  No X in the old range sets it: over the prefix decode_towers keeps
// (Q > 2^130), |X| < 2^127 puts sum_t y_t / q_t within 2^-3 of k, and the binary32 estimate errs by
// at most ~L 2^-21 (terms (y_t >> s_t) * (2^s_t / q_t), y_t >> s_t < 2^32, TowerConst::crt_sh), so
// k is exact and the output bits are the round-5 ones.
template <int NC, class YF>
__device__ __forceinline__ double crt_value(YF yf, uint32_t L, const TowerConst* __restrict__ tcs,
                                            double inv_scale, bool& wide) {
  static_assert(NC >= 5 && NC <= 7, "crt columns");
  constexpr uint32_t M30 = (1u << 30) - 1;
  uint64_t sc[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) sc[j] = 0;
  float f = 0.f;
#pragma unroll 1
  for (uint32_t t = 0; t < L; ++t) {
    const TowerConst& c = tcs[t];
    const uint64_t y = yf(t);
    const uint32_t ytop = __builtin_amdgcn_alignbit((uint32_t)(y >> 32), (uint32_t)y, c.crt_sh);
    f = __fadd_rn(f, __fmul_rn((float)ytop, c.inv_q32));
    const uint32_t a = (uint32_t)y & M30, b = (uint32_t)(y >> 30);
    sc[0] += (uint64_t)a * c.crt30[0];
#pragma unroll
    for (int j = 1; j < NC; ++j) sc[j] += (uint64_t)a * c.crt30[j] + (uint64_t)b * c.crt30[j - 1];
  }
  const uint32_t kk = (uint32_t)__fadd_rn(f, 0.5f);  // <= L
  const uint32_t* nq = tcs[0].nq30;
  sc[0] += (uint64_t)kk * nq[0];
#pragma unroll
  for (int j = 1; j < NC; ++j) sc[j] += (uint64_t)kk * nq[j] + (sc[j - 1] >> 30);
  uint64_t xlo = (sc[0] & M30) | ((sc[1] & M30) << 30) | (sc[2] << 60);
  uint64_t xhi = ((sc[2] & M30) >> 4) | ((sc[3] & M30) << 26) | (sc[4] << 56);
  // bits 127 .. 30 NC - 1 must be X's sign
  const bool neg = (int64_t)xhi < 0;
  const uint32_t ext = neg ? M30 : 0u;
  bool bad = (((uint32_t)sc[4] & M30) >> 7) != (ext >> 7);
#pragma unroll
  for (int j = 5; j < NC; ++j) bad |= ((uint32_t)sc[j] & M30) != ext;
  wide |= bad;
  // sign-magnitude -> double (the oracle's or_i128_to_double)
  if (neg) {
    xlo = ~xlo + 1;
    xhi = ~xhi + (xlo == 0 ? 1 : 0);
  }
  double v = __dadd_rn(__dmul_rn((double)xhi, 18446744073709551616.0), (double)xlo);
  if (neg) v = -v;
  return __dmul_rn(v, inv_scale);
}

// Bits [pos, pos + 64) of a little-endian 30-bit-limb integer of NL limbs.
__device__ __forceinline__ uint64_t mw30_bits64(const uint64_t* a, uint32_t NL, uint32_t pos) {
  uint64_t r = 0;
#pragma unroll 1
  for (uint32_t l = pos / 30; l < NL && 30 * l < pos + 64; ++l) {
    const int sh = (int)(30 * l) - (int)pos;
    r |= sh >= 0 ? (a[l] << sh) : (a[l] >> -sh);
  }
  return r;
}

// a += m * b (mod 2^(30 NL)), a normalised to 30-bit limbs
__device__ __forceinline__ void mw30_addmul(uint64_t* a, const uint32_t* b, uint64_t m, uint32_t NL) {
  constexpr uint64_t M30 = (1u << 30) - 1;
  uint64_t carry = 0;
#pragma unroll 1
  for (uint32_t j = 0; j < NL; ++j) {
    const uint64_t v = a[j] + m * b[j] + carry;
    a[j] = v & M30;
    carry = v >> 30;
  }
}

// compare two NL-limb magnitudes: -1, 0, 1
__device__ __forceinline__ int mw30_cmp(const uint64_t* a, const uint32_t* b, uint32_t NL) {
#pragma unroll 1
  for (int j = (int)NL - 1; j >= 0; --j)
    if (a[j] != b[j]) return a[j] < b[j] ? -1 : 1;
  return 0;
}

__device__ __forceinline__ void mw30_negate(uint64_t* a, uint32_t NL) {
  constexpr uint64_t M30 = (1u << 30) - 1;
  uint64_t carry = 1;
#pragma unroll 1
  for (uint32_t j = 0; j < NL; ++j) {
    const uint64_t v = ((~a[j]) & M30) + carry;
    a[j] = v & M30;
    carry = v >> 30;
  }
}

// The exact centred CRT over any tower set (round 6; PALISADE's CRTInterpolate to a BigInteger and
// centring mod Q before Decode, ckks.cpp:189): X in [-(Q - 1) / 2, (Q - 1) / 2]
// from V = sum_t y_t (Q/q_t) (< L Q) in NL 30-bit limbs (DeviceTables::crt_mw), k = round(sum_t
// y_t / q_t) in binary64, X' = V - k Q in two's complement, then at most two corrections by Q
// against (Q - 1) / 2 (exact comparisons), so k's estimate only has to be within 1.  |X| becomes
// NW 64-bit words w and (double) by Horner from the top, d = d 2^64 + (double)w_i, the oracle's
// or_mw_to_double; leading zero words leave d unchanged, so below 2^127 this is crt_value's
// two-word conversion bit for bit.  A slow path: limbs live in scratch (private memory).
template <class YF>
__device__ __forceinline__ double crt_exact_value(YF yf, uint32_t L, const TowerConst* __restrict__ tcs,
                                                  const uint32_t* __restrict__ mw, double inv_scale) {
  constexpr uint64_t M30 = (1u << 30) - 1;
  const uint32_t NL = mw[0], NW = mw[1];
  const uint32_t* qh = mw + 4;
  const uint32_t* nQ = qh + (size_t)L * NL;
  const uint32_t* half = nQ + NL;
  uint64_t acc[kCrtMwMaxLimbs];
#pragma unroll 1
  for (uint32_t j = 0; j < NL; ++j) acc[j] = 0;
  double f = 0.0;
#pragma unroll 1
  for (uint32_t t = 0; t < L; ++t) {
    const uint64_t y = yf(t);
    f = __dadd_rn(f, __dmul_rn((double)y, tcs[t].inv_q));
    const uint64_t a = y & M30, b = y >> 30;
    const uint32_t* h = qh + (size_t)t * NL;
    uint64_t carry = 0;
#pragma unroll 1
    for (uint32_t j = 0; j < NL; ++j) {
      const uint64_t v = acc[j] + a * h[j] + (j ? b * h[j - 1] : 0) + carry;
      acc[j] = v & M30;
      carry = v >> 30;
    }
  }
  mw30_addmul(acc, nQ, (uint64_t)__dadd_rn(f, 0.5), NL);  // X' = V - k Q
#pragma unroll 1
  for (int it = 0; it < 2; ++it) {
    const bool neg = (acc[NL - 1] >> 29) & 1;
    if (!neg) {
      if (mw30_cmp(acc, half, NL) <= 0) break;
      mw30_addmul(acc, nQ, 1, NL);  // X' - Q
    } else {
      mw30_negate(acc, NL);
      const bool over = mw30_cmp(acc, half, NL) > 0;
      mw30_negate(acc, NL);
      if (!over) break;
      // X' + Q = X' - (2^(30 NL) - Q) mod 2^(30 NL)
      mw30_negate(acc, NL);
      mw30_addmul(acc, nQ, 1, NL);
      mw30_negate(acc, NL);
    }
  }
  const bool neg = (acc[NL - 1] >> 29) & 1;
  if (neg) mw30_negate(acc, NL);
  double d = (double)mw30_bits64(acc, NL, 64 * (NW - 1));
#pragma unroll 1
  for (int w = (int)NW - 2; w >= 0; --w)
    d = __dadd_rn(__dmul_rn(d, 18446744073709551616.0), (double)mw30_bits64(acc, NL, 64 * (uint32_t)w));
  if (neg) d = -d;
  return __dmul_rn(d, inv_scale);
}

// -------------------------------------------------------------- decrypt ----
// Centred CRT: y_t = b_t (Q/q_t)^-1 mod q_t; X = sum y_t (Q/q_t) - k Q with k = round(sum y_t / q_t)
// (crt_value: NC exact columns, *wide set when X is outside the 128-bit range); then (double)X *
// (1/scale) (PALISADE Decode: ConvertToDouble * scalingFactorPre * 2^-p).  Written at bitrev(i) for
// FFTSpecial.  EXACT: crt_exact_kernel's arithmetic (crt_exact_value, every |X| <= (Q - 1) / 2).
template <int NC, bool EXACT = false>
__global__ __launch_bounds__(256) void crt_decode_kernel(const uint64_t* __restrict__ dbuf,
                                                         uint64_t K, uint32_t logN, uint32_t logS,
                                                         uint32_t L,
                                                         const TowerConst* __restrict__ tcs,
                                                         const uint32_t* __restrict__ mw,
                                                         double inv_scale,
                                                         double2* __restrict__ fbuf,
                                                         GenFlag wide_flag) {
  const uint32_t N = 1u << logN, S = 1u << logS;
  // S >= 256: a block owns the 256 slots i = hi.2^(logS-4) | mid.16 | lo (hi, lo < 16) of one
  // middle value, so the tower reads (16 consecutive i) and, after a transpose through LDS,
  // the bit-reversed stores (16 consecutive outputs, 256 B) are both contiguous.
  const bool tiled = logS >= 8;
  uint64_t k;
  uint32_t i, mid = 0;
  if (tiled) {
    k = blockIdx.x >> (logS - 8);
    mid = blockIdx.x & ((1u << (logS - 8)) - 1);
    i = ((threadIdx.x >> 4) << (logS - 4)) | (mid << 4) | (threadIdx.x & 15);
  } else {
    const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    k = gid >> logS;
    i = (uint32_t)(gid & (S - 1));
  }
  if (k >= K) return;  // block-uniform when tiled (the grid is exact)
  const uint32_t gapLog = logN - 1 - logS;
  const uint64_t* __restrict__ d = dbuf + k * ((uint64_t)L << logN);
  double res[2];
  bool wide = false;
#pragma unroll
  for (int part = 0; part < 2; ++part) {
    const uint32_t j = (part ? (N >> 1) : 0) + (i << gapLog);
    const auto yf = [&](uint32_t t) {
      const TowerConst& c = tcs[t];
      return shoup_mul(d[((uint64_t)t << logN) + j], c.qhat_inv, c.qhat_inv_shoup, c.q);
    };
    if constexpr (EXACT)
      res[part] = crt_exact_value(yf, L, tcs, mw, inv_scale);
    else
      res[part] = crt_value<NC>(yf, L, tcs, inv_scale, wide);
  }
  if (wide) gen_flag_set(wide_flag, 2);
  if (!tiled) {
    fbuf[k * S + bitrev_dev(i, logS)] = make_double2(res[0], res[1]);
    return;
  }
  // bitrev(i) = bitrev4(lo).2^(logS-4) | bitrev(mid).16 | bitrev4(hi): slot (lo, hi) goes to
  // tile row bitrev4(lo), column bitrev4(hi); rows padded to 17 entries (conflict-free).
  __shared__ double2 tile[16][17];
  tile[bitrev_dev(threadIdx.x & 15, 4)][bitrev_dev(threadIdx.x >> 4, 4)] = make_double2(res[0], res[1]);
  __syncthreads();
  const uint32_t a = threadIdx.x >> 4, b = threadIdx.x & 15;
  fbuf[k * S + ((a << (logS - 4)) | (bitrev_dev(mid, logS - 8) << 4) | b)] = tile[a][b];
}

// Decrypt's last INTT pass fused with the exact CRT decode (ntt_inv_cols + crt_decode_kernel
// without the round trip of the [K][L][N] residues through HBM).  A workgroup owns 64
// columns (coefficients j = c + BLK r, r < R) of one ciphertext for every tower: wave w
// runs the top LOGR stages of towers t = w, w + 4, ... and leaves y_t = b_t (N^-1 (Q/q_t)^-1)
// mod q_t in LDS; then each (real, imaginary) coefficient pair (r, r + R/2) is
// CRT-reconstructed exactly as crt_decode_kernel does (same operation order) and stored
// at bitrev(slot).  Needs L R 512 B of LDS <= kCrtFuseLds and gap = N / 2S <= 64.
// LDS rows: the CRT loop reads ys[t][r][u] with r fastest (8 consecutive lanes = 8 rows, 4
// consecutive u per 32-lane ds_read_b64 group); rows of 64 u64 would put those 8 rows on one bank.
// Round 5: column u is stored at u ^ 4 (r mod 8) -- 32 distinct banks per group in L R 512 B (32 KiB
// at 2^15 / L4, 5 workgroups per CU; the round-4 rows padded to 68 u64 ran the same, 0.960 vs 0.959
// us per decrypted ciphertext, profiles/r05d).
constexpr size_t kCrtFuseLds = 48 << 10;
template <int LOGR, int NC>
__global__ __launch_bounds__(256) void ntt_inv_cols_crt(const uint64_t* __restrict__ dbuf, uint32_t L,
                                                        uint32_t logN, uint32_t logS,
                                                        const uint64_t* __restrict__ tw,
                                                        const uint64_t* __restrict__ twp,
                                                        const TowerConst* __restrict__ tcs, double inv_scale,
                                                        double2* __restrict__ fbuf,
                                                        GenFlag wide_flag) {
  constexpr int R = 1 << LOGR, CW = 64, CWP = 64;
  extern __shared__ uint64_t ys_flat[];  // [L][R][CWP]
  uint64_t(*ys)[R][CWP] = reinterpret_cast<uint64_t(*)[R][CWP]>(ys_flat);
  const auto ucol = [](uint32_t r, uint32_t u) { return u ^ ((r & 7u) << 2); };
  const uint32_t N = 1u << logN, BLK = N >> LOGR, S = 1u << logS;
  const uint32_t cpb = BLK / CW;
  const uint64_t k = blockIdx.x / cpb;
  const uint32_t c0 = (blockIdx.x % cpb) * CW;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll 1
  for (uint32_t t = wv; t < L; t += 4) {
    const TowerConst& c = tcs[t];
    const uint64_t q = c.q;
    const uint64_t* __restrict__ w = tw + ((uint64_t)t << logN);
    const uint64_t* __restrict__ wp = twp + ((uint64_t)t << logN);
    const uint64_t* __restrict__ a = dbuf + ((k * L + t) << logN) + c0 + lane;
    uint64_t x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = a[(uint64_t)r * BLK];
#pragma unroll
    for (int v = 0; v < LOGR - 1; ++v) {
      const int tr = 1 << v, h = R >> (v + 1);
#pragma unroll
      for (int i = 0; i < h; ++i) {
        const uint64_t W = w[h + i], Wp = wp[h + i];
#pragma unroll
        for (int jj = 0; jj < tr; ++jj) {
          if (gs_in8<true>(v, jj))
            gs_bfly_b<true>(x[2 * i * tr + jj], x[2 * i * tr + jj + tr], W, Wp, q, c.n8q);
          else
            gs_bfly_b<false>(x[2 * i * tr + jj], x[2 * i * tr + jj + tr], W, Wp, q, c.n8q);
        }
      }
    }
    // the last stage (one twiddle, w[1]) fused with the scale N^-1 (Q/q_t)^-1 (round 5): X = (x + y) c,
    // Y = (x + B - y) (w[1] c) -- two products per pair instead of the butterfly's one and the scale's two
    constexpr int TR = R / 2;
#pragma unroll
    for (int jj = 0; jj < TR; ++jj) {
      const uint64_t xv = x[jj], yv = x[jj + TR];
      const uint64_t B = gs_in8<true>(LOGR - 1, jj) ? (q << 3) : (q << 2);  // the butterfly's input bound
      ys[t][jj][ucol(jj, lane)] = canon4(shoup_lazy(xv + yv, c.ninv_qhat, c.ninv_qhat_shoup, q), q);
      ys[t][jj + TR][ucol(jj + TR, lane)] =
          canon4(shoup_lazy(xv + B - yv, c.ninv_qhat_w1, c.ninv_qhat_w1_shoup, q), q);
    }
  }
  __syncthreads();
  const uint32_t gapLog = logN - 1 - logS, gap = 1u << gapLog;
  bool wide = false;
  // pair p -> half-row r (< R/2) fastest, so 8 consecutive threads store 8 consecutive
  // bit-reversed slots (one 128-byte segment)
#pragma unroll 1
  for (uint32_t p = threadIdx.x; p < (uint32_t)(R / 2) * CW; p += 256) {
    const uint32_t r = p % (R / 2), u = p / (R / 2);
    const uint32_t col = c0 + u;
    if (col & (gap - 1)) continue;  // coefficient not on a slot
    double res[2];
#pragma unroll
    for (int part = 0; part < 2; ++part) {
      const uint32_t rr = r + part * (R / 2);
      res[part] = crt_value<NC>([&](uint32_t t) { return ys[t][rr][ucol(rr, u)]; }, L, tcs, inv_scale, wide);
    }
    const uint32_t i = (col + BLK * r) >> gapLog;
    fbuf[k * S + bitrev_dev(i, logS)] = make_double2(res[0], res[1]);
  }
  if (wide) gen_flag_set(wide_flag, 2);
}

// ------------------------------------------------- decode noise flooding ----
// PALISADE 1.11 CKKSPackedEncoding::Decode, on the coefficient
// pairs v_i = (c[i gap], c[N/2 + i gap]) / scale that crt_decode_kernel wrote at
// bitrev(i).  m(X^-1) in this packing is conj_0 = (re_0, -im_0),
// conj_i = (-im_{S-i}, -re_{S-i}); the anti-symmetric part u = v - conj has S
// independent components (i = 0: 2 im_0; 0 < i < S/2: both; i = S/2: one), whose
// sample stddev / 2 estimates the decryption error sigma.  In 2^p units (p = scale
// bits, PALISADE's plaintext modulus): fail if log2 sigma > p - 5; sigma >= sqrt(N)/8;
// stddev = sqrt(M+1) sigma; each output becomes (v + conj)/2 + 2^-p N(0, stddev);
// logError = round(log2(stddev sqrt(2 S))).  One block per ciphertext.
__device__ __forceinline__ double block_sum_1024(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x < 64) {
    s = threadIdx.x < (blockDim.x >> 6) ? red[threadIdx.x] : 0.0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if (threadIdx.x == 0) red[16] = s;
  }
  __syncthreads();
  s = red[16];
  __syncthreads();
  return s;
}

// Box-Muller pair from two 32-bit stream words: u1 = (a + 1) 2^-32 in (0, 1], u2 = b 2^-32
// in [0, 1) (revolutions; the top 24 bits are used).  The transcendental functions run
// in binary32 (one instruction each): the normals scale noise ~1e-13 of the decoded
// values, so their 2^-24 relative error moves an output by < 1e-20 (the oracle
// evaluates them in binary64).
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, double& z0, double& z1) {
  const float u1 = (float)fma((double)a, 0x1.0p-32, 0x1.0p-32);
  const float u2 = (float)(b >> 8) * 0x1.0p-24f;
  const float r = __fsqrt_rn(-2.0f * __logf(u1));
  float sn, cs;
  __sincosf(6.2831853071795864f * u2, &sn, &cs);
  z0 = (double)(r * cs);
  z1 = (double)(r * sn);
}
// (re, im) normals of FFT-input position P: ChaCha20 block P >> 3 (nonce (3 << 56) | g),
// stream words 2 (P mod 8) and 2 (P mod 8) + 1 (one u64 of chacha20_block's output).
__device__ __forceinline__ void flood_pair(uint64_t w, double& z0, double& z1) {
  box_muller((uint32_t)w, (uint32_t)(w >> 32), z0, z1);
}

__global__ __launch_bounds__(1024) void decode_flood_kernel(double2* __restrict__ fbuf, uint32_t logS,
                                                            uint32_t logN, double two_p,
                                                            double p_bits, double m_factor,
                                                            Key8 key, uint64_t g0,
                                                            uint32_t* __restrict__ flags, GenFlag fail) {
  __shared__ double red[17];
  const uint32_t S = 1u << logS, half = S >> 1;
  double2* __restrict__ f = fbuf + (uint64_t)blockIdx.x * S;
  // u components of pair index i in [0, S/2]
  auto comps = [&](uint32_t i, double& a, double& b) -> int {
    const double2 x = f[bitrev_dev(i, logS)];
    if (i == 0) {
      a = 2.0 * x.y;
      return 1;
    }
    if (i == half) {
      a = x.x + x.y;
      return 1;
    }
    const double2 y = f[bitrev_dev(S - i, logS)];
    a = x.x + y.y;
    b = x.y + y.x;
    return 2;
  };
  double sigma;
  if (S == 1) {
    sigma = fabs(f[0].y);  // PALISADE StdDev: vec[0].imag() for one slot
  } else {
    double s1 = 0.0;
    for (uint32_t i = threadIdx.x; i <= half; i += blockDim.x) {
      double a = 0.0, b = 0.0;
      const int c = comps(i, a, b);
      s1 += a + (c == 2 ? b : 0.0);
    }
    const double mean = block_sum_1024(s1, red) / (double)S;
    double s2 = 0.0;
    for (uint32_t i = threadIdx.x; i <= half; i += blockDim.x) {
      double a = 0.0, b = 0.0;
      const int c = comps(i, a, b);
      s2 += (a - mean) * (a - mean) + (c == 2 ? (b - mean) * (b - mean) : 0.0);
    }
    const double var = block_sum_1024(s2, red) / (double)(S - 1);
    sigma = 0.5 * sqrt(var);
  }
  double sigma_p = sigma * two_p;  // PALISADE works at scale 2^p
  const double logstd = log2(sigma_p);
  if (!(logstd <= p_bits - 5.0)) {
    if (threadIdx.x == 0) gen_flag_set(fail, 3);  // decode precision failure
  }
  const double floor_sd = 0.125 * sqrt((double)(1u << logN));
  if (sigma_p < floor_sd) sigma_p = floor_sd;
  const double stddev_p = sqrt(m_factor + 1.0) * sigma_p;
  if (threadIdx.x == 0) {
    const double le = rint(log2(stddev_p * sqrt(2.0 * (double)S)));
    atomicMax((int*)&flags[2], (int)le);
  }
  const double nsd = stddev_p / two_p;  // noise stddev in output units
  const uint64_t nonce = (3ull << 56) | (g0 + blockIdx.x);
  // the normals of the slot at FFT-input position P: block P >> 1, pair P & 1
  auto noise = [&](uint32_t P, double& za, double& zb) {
    uint64_t w[8];
    chacha20_block(key, P >> 3, nonce, w);
    flood_pair(w[P & 7], za, zb);
  };
  __syncthreads();  // every thread has read its pairs before any is overwritten
  for (uint32_t i = threadIdx.x; i <= half; i += blockDim.x) {
    const uint32_t pi = bitrev_dev(i, logS);
    const double2 x = f[pi];
    double z0, z1;
    noise(pi, z0, z1);
    if (i == 0) {
      f[pi] = make_double2(x.x + nsd * z0, nsd * z1);
      if (S == 1) continue;
    } else if (i == half) {
      f[pi] = make_double2(0.5 * (x.x - x.y) + nsd * z0, 0.5 * (x.y - x.x) + nsd * z1);
    } else {
      const uint32_t pj = bitrev_dev(S - i, logS);
      const double2 y = f[pj];
      double z2, z3;
      noise(pj, z2, z3);
      f[pi] = make_double2(0.5 * (x.x - y.y) + nsd * z0, 0.5 * (x.y - y.x) + nsd * z1);
      f[pj] = make_double2(0.5 * (y.x - x.y) + nsd * z2, 0.5 * (y.y - x.x) + nsd * z3);
    }
  }
}

// Flooding at 2^11 slots and more, in two steps that stream the slots once each:
//  1. decode_stats_kernel: per ciphertext G = S/2048 workgroups sum the anti-symmetric
//     components u (decode_flood_kernel's, over pairs (i, S - i)) and their squares;
//  2. fft_fwd_blocks adds the noise while it loads its block (FloodArgs): sigma from
//     the G partial sums (one-pass variance (sum u^2 - (sum u)^2 / S) / (S - 1)), the
//     normals of position P from ChaCha20 block P >> 3 (a thread loads positions 8m ..
//     8m + 7: one block, eight Box-Muller pairs).
// The symmetrization (v + conj)/2 is left out: conj contributes only the imaginary part
// of each decoded slot (m(1/zeta) = conj m(zeta) for real coefficients) and decrypt
// keeps real parts, so the output is the same up to rounding (oracle tolerance 1e-14).
// Slot i sits at FFT-input position P = bitrev(i); its conjugate partner S - i sits at
// P ^ (2^h - 1), h = the index of P's leading bit (complementing i's bits above its
// lowest set bit complements P's bits below its highest): the octave [2^h, 2^(h+1))
// mirrored.  Pair m (0 <= m < S/2 - 1) is P = 2^h + o with m + 1 = 2^(h-1) + o, partner
// 2^(h+1) - 1 - o: consecutive m read two contiguous runs (one backwards).  Positions 0
// (slot 0) and 1 (slot S/2) are their own partners.
constexpr uint32_t kFloodPairsPerWg = 1024;
__global__ __launch_bounds__(256) void decode_stats_kernel(const double2* __restrict__ fbuf, uint32_t logS,
                                                           uint32_t G, double2* __restrict__ part,
                                                           uint32_t* __restrict__ reset_flags) {
  __shared__ double red[2][4];
  // the call's precision / logError flags, reset here (the FFT pass that sets them runs after this
  // kernel on the same stream) instead of by a separate fill launch
  if (reset_flags && blockIdx.x == 0 && threadIdx.x < 2) reset_flags[1 + threadIdx.x] = 0;
  const uint32_t S = 1u << logS, half = S >> 1;
  const uint64_t k = blockIdx.x / G;
  const uint32_t wg = blockIdx.x % G;
  const double2* __restrict__ f = fbuf + k * S;
  double s1 = 0.0, s2 = 0.0;
  const uint32_t m1 = min(half - 1, (wg + 1) * kFloodPairsPerWg);
  for (uint32_t m = wg * kFloodPairsPerWg + threadIdx.x; m < m1; m += 256) {
    const uint32_t hb = 31 - __clz(m + 1);  // h - 1
    const uint32_t o = m + 1 - (1u << hb);
    const double2 x = f[(2u << hb) + o], y = f[(4u << hb) - 1 - o];
    const double a = x.x + y.y, b = x.y + y.x;
    s1 += a + b;
    s2 += a * a + b * b;
  }
  if (wg == 0 && threadIdx.x == 0) {
    const double2 x0 = f[0], xh = f[1];  // slot 0: 2 im; slot S/2: re + im
    const double a = 2.0 * x0.y, c = xh.x + xh.y;
    s1 += a + c;
    s2 += a * a + c * c;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_down(s1, o, 64);
    s2 += __shfl_down(s2, o, 64);
  }
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wave] = s1;
    red[1][wave] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    part[blockIdx.x] = make_double2((red[0][0] + red[0][1]) + (red[0][2] + red[0][3]),
                                    (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]));
}

struct FloodArgs {
  const double2* part;  // [K][G] (sum u, sum u^2) of decode_stats_kernel
  uint32_t G, logN;
  double two_p, p_bits, m_factor;
  Key8 key;
  uint64_t g0;
  uint32_t* flags;  // [2] = max logError
  GenFlag fail;     // word 3: precision failure
};

// Ciphertext k's flooding scale from decode_stats_kernel's partial sums: the noise's standard
// deviation in slot units (the first block of each ciphertext records the precision failure and
// logError).
__device__ __forceinline__ double flood_nsd_sums(const FloodArgs& fa, double s1, double s2, uint32_t b, uint32_t S) {
  const double var = (s2 - s1 * (s1 / (double)S)) / (double)(S - 1);
  double sigma_p = 0.5 * sqrt(var > 0.0 ? var : 0.0) * fa.two_p;
  const bool fail = !(log2(sigma_p) <= fa.p_bits - 5.0);
  const double floor_sd = 0.125 * sqrt((double)(1u << fa.logN));
  if (sigma_p < floor_sd) sigma_p = floor_sd;
  const double stddev_p = sqrt(fa.m_factor + 1.0) * sigma_p;
  if (b == 0 && threadIdx.x == 0) {
    if (fail) gen_flag_set(fa.fail, 3);
    atomicMax((int*)&fa.flags[2], (int)rint(log2(stddev_p * sqrt(2.0 * (double)S))));
  }
  return stddev_p / fa.two_p;
}
__device__ __forceinline__ double flood_nsd(const FloodArgs& fa, uint64_t k, uint32_t b, uint32_t S) {
  double s1 = 0.0, s2 = 0.0;
  for (uint32_t g = 0; g < fa.G; ++g) {
    const double2 v = fa.part[k * fa.G + g];
    s1 += v.x;
    s2 += v.y;
  }
  return flood_nsd_sums(fa, s1, s2, b, S);
}

// FFTSpecial first pass (decode): input already bit-reversed by the CRT's scatter; DIT
// stages len = 2..blk with twiddle ffwd[len/2 + (x mod len)] in LDS blocks; the top LOGR
// stages follow on register columns (fft_fwd_cols).  A single pass writes the real parts
// of the first `n` slots straight into the caller's output vector; FLOOD adds the decode
// noise there, in the output domain (as fft_fwd_cols).
template <bool FLOOD>
__global__ __launch_bounds__(256) void fft_fwd_blocks(double2* __restrict__ buf, uint32_t logS,
                                                      uint32_t blkLog, const double2* __restrict__ tw,
                                                      double* __restrict__ out, uint64_t n,
                                                      int final_pass, FloodArgs fa) {
  extern __shared__ __attribute__((aligned(16))) double2 smc[];
  const uint32_t S = 1u << logS, blk = 1u << blkLog;
  const uint32_t sh = logS - blkLog;
  const uint64_t k = blockIdx.x >> sh;
  const uint32_t b = blockIdx.x & ((1u << sh) - 1);
  const uint64_t off = k * S + ((uint64_t)b << blkLog);
  for (uint32_t i = threadIdx.x; i < blk; i += 256) smc[i] = buf[off + i];
  __syncthreads();
  for (uint32_t len = 2; len <= blk; len <<= 1) {
    const uint32_t lenh = len >> 1;
    for (uint32_t p = threadIdx.x; p < blk / 2; p += 256) {
      const uint32_t j = p & (lenh - 1);
      const uint32_t i0 = (p - j) * 2 + j;
      const double2 W = tw[lenh + j];
      const double2 u = smc[i0];
      const double2 v = cmul(smc[i0 + lenh], W);
      smc[i0] = cadd(u, v);
      smc[i0 + lenh] = csub(u, v);
    }
    __syncthreads();
  }
  if (final_pass) {  // (one block per ciphertext: b == 0, blk == S)
    double nso = 0.0;
    uint64_t nonce = 0;
    if (FLOOD) {
      nso = flood_nsd(fa, k, b, S) * sqrt((double)S);
      nonce = (3ull << 56) | (fa.g0 + k);
    }
    for (uint32_t i = threadIdx.x; i < blk; i += 256) {
      const uint64_t gi = off + i;
      double v = smc[i].x;
      if (FLOOD) {  // fft_fwd_cols's output-domain stream: normal (i div S/16) of block (i mod S/16)
        const uint32_t S16 = S >> 4, nidx = i / S16;
        uint64_t w[8];
        chacha20_block(fa.key, i & (S16 - 1), nonce, w);
        double z0, z1;
        flood_pair(w[nidx >> 1], z0, z1);
        v = __dadd_rn(v, __dmul_rn(nso, (nidx & 1) ? z1 : z0));
      }
      if (gi < n) out[gi] = v;
    }
  } else {
    for (uint32_t i = threadIdx.x; i < blk; i += 256) buf[off + i] = smc[i];
  }
}

// FFTSpecial's first pass (decode, not the final pass): block b of ciphertext k, DIT half-sizes
// 1 .. 2^(BL-1).  (Until round 4 the flooding noise was added here, on load; it now lands on the
// output in fft_fwd_cols.)
template <int BL, int K1, int K2, int K3, int K4, bool SWZ = true>
__global__ __launch_bounds__(1 << (BL - 3)) void fft_fwd_blocks_ct(double2* __restrict__ buf, uint32_t logS,
                                                                  const double2* __restrict__ tw) {
  static_assert(K1 + K2 + K3 + K4 == BL, "chunk plan");
  __shared__ __attribute__((aligned(16))) double2 sm[1 << BL];
  const uint32_t S = 1u << logS, sh = logS - BL;
  const uint64_t k = blockIdx.x >> sh;
  const uint32_t b = blockIdx.x & ((1u << sh) - 1);
  double2* __restrict__ g = buf + k * S + ((uint64_t)b << BL);
  const auto lds_ld = [&](uint32_t j) { return sm[fft_swz<SWZ>(j)]; };
  const auto lds_st = [&](uint32_t j, double2 v) { sm[fft_swz<SWZ>(j)] = v; };
  fft_chunk<BL, K1, 0, true>(tw, [&](uint32_t j) { return g[j]; }, lds_st);
  __syncthreads();
  fft_chunk<BL, K2, K1, true>(tw, lds_ld, lds_st);
  __syncthreads();
  fft_chunk<BL, K3, K1 + K2, true>(tw, lds_ld, lds_st);
  __syncthreads();
  fft_chunk<BL, K4, K1 + K2 + K3, true>(tw, lds_ld, [&](uint32_t j, double2 v) { g[j] = v; });
}

// FFTSpecial's last pass (decode): the top LOGR stages on register columns; writes the real parts
// of the first `n` slots straight into the caller's output vector.  FLOOD (round 5): PALISADE's
// decode noise in the output domain -- N(0, sd sqrt(S)) added to each decoded real part, the same
// distribution as N(0, sd) on every FFT input (FFTSpecial's F F^H = S I; oracle or_decrypt_flood):
// slot i takes normal (i div S/16) of ChaCha20 block (i mod S/16), so a thread's 2^LOGR rows share
// 2^max(0, LOGR-4) blocks.
template <int LOGR, bool FLOOD = false>
__global__ __launch_bounds__(256) void fft_fwd_cols(const double2* __restrict__ buf, uint32_t logS,
                                                    const double2* __restrict__ tw,
                                                    double* __restrict__ out, uint64_t n, FloodArgs fa) {
  constexpr int R = 1 << LOGR;
  const uint32_t S = 1u << logS;
  const uint32_t BLK = S >> LOGR;
  const uint32_t bpp = BLK / 256;
  const uint64_t k = blockIdx.x / bpp;
  const uint32_t col = (blockIdx.x % bpp) * 256 + threadIdx.x;
  double2 v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) v[r] = buf[k * S + col + (uint64_t)r * BLK];
#pragma unroll
  for (int s = 0; s < LOGR; ++s) {
    const uint32_t lenh = BLK << s;
    const int tr = 1 << s;
#pragma unroll
    for (int r0 = 0; r0 < R; ++r0) {
      if ((r0 >> s) & 1) continue;
      const int r1 = r0 + tr;
      const uint32_t j = col + (uint32_t)(r0 & ((2 << s) - 1)) * BLK;  // (col + r0 BLK) mod len
      const double2 W = tw[lenh + j];
      const double2 u = v[r0];
      const double2 w = cmul(v[r1], W);
      v[r0] = cadd(u, w);
      v[r1] = csub(u, w);
    }
  }
  if (FLOOD) {
    const double nso = flood_nsd(fa, k, blockIdx.x % bpp, S) * sqrt((double)S);
    const uint64_t nonce = (3ull << 56) | (fa.g0 + k);
    const uint32_t S16 = S >> 4;
    constexpr int LO = LOGR > 4 ? LOGR - 4 : 0;  // ChaCha blocks per thread: 2^LO
#pragma unroll
    for (int rl = 0; rl < (1 << LO); ++rl) {
      uint64_t w[8];
      chacha20_block(fa.key, (col + BLK * (uint32_t)rl) & (S16 - 1), nonce, w);
      if (LOGR >= 4) {  // the thread's rows use all 16 normals of the block
        double z[16];
#pragma unroll
        for (int m = 0; m < 8; ++m) flood_pair(w[m], z[2 * m], z[2 * m + 1]);
#pragma unroll
        for (int r = rl; r < R; r += (1 << LO)) {
          const uint32_t nidx = (col + BLK * (uint32_t)r) / S16;  // < 16
          double zr = 0.0;
#pragma unroll
          for (int m = 0; m < 16; ++m) zr = (uint32_t)m == nidx ? z[m] : zr;  // no dynamic register index
          v[r].x = __dadd_rn(v[r].x, __dmul_rn(nso, zr));
        }
      } else {  // rows 2^(4-LOGR) normals apart: one Box-Muller pair per row, half of it used
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint32_t nidx = (col + BLK * (uint32_t)r) / S16;
          uint64_t wr = 0;
#pragma unroll
          for (int m = 0; m < 8; ++m) wr = (uint32_t)m == (nidx >> 1) ? w[m] : wr;
          double z0, z1;
          flood_pair(wr, z0, z1);
          v[r].x = __dadd_rn(v[r].x, __dmul_rn(nso, (nidx & 1) ? z1 : z0));
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t gi = k * S + col + (uint64_t)r * BLK;
    if (gi < n) out[gi] = v[r].x;
  }
}

// decode_stats_kernel's sums inside the whole-vector decode (round 5): a[i] holds FFT-input position
// P = 1024 w + 4 (l + 64 (i >> 2)) + (i & 3); pair (P, P ^ (2^h - 1)) (h = P's leading bit, P in the
// lower half of its octave) contributes a = x.re + y.im and b = x.im + y.re, positions 0 and 1 their
// own terms.  The partners' components come through LDS (real parts, then imaginary), the sums by a
// wave shuffle and LDS reduction; every thread returns (sum, sum of squares).
__device__ __forceinline__ double2 fft_whole_flood_stats(const double2 (&a)[16], double* __restrict__ lds) {
  const uint32_t T = threadIdx.x, w = T >> 6, l = T & 63;
  double s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int part = 0; part < 2; ++part) {
#pragma unroll
    for (int i = 0; i < 16; ++i) lds[w * kFftWholeRow + fft_wt1(l, i)] = part ? a[i].y : a[i].x;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t P = 1024 * w + 4 * (l + 64 * (i >> 2)) + (i & 3);
      if (P < 2) continue;
      const uint32_t h = 31 - __clz(P);
      if ((P >> (h - 1)) & 1) continue;  // upper half of the octave: counted by its partner
      const uint32_t Q = P ^ ((1u << h) - 1);
      const double y = lds[(Q >> 10) * kFftWholeRow + fft_wpad(Q & 1023)];
      const double v = part ? a[i].x + y : a[i].y + y;  // part 0: b = x.im + y.re; part 1: a = x.re + y.im
      s1 += v;
      s2 += v * v;
    }
    __syncthreads();
  }
  if (T == 0) {  // slot 0: 2 im; slot S/2: re + im (positions 0 and 1)
    const double a0 = 2.0 * a[0].y, c = a[1].x + a[1].y;
    s1 += a0 + c;
    s2 += a0 * a0 + c * c;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_down(s1, o, 64);
    s2 += __shfl_down(s2, o, 64);
  }
  if (l == 0) {
    lds[2 * w] = s1;
    lds[2 * w + 1] = s2;
  }
  __syncthreads();
  double t1 = 0.0, t2 = 0.0;
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    t1 += lds[2 * v];
    t2 += lds[2 * v + 1];
  }
  __syncthreads();  // the LDS is the block exchanges' next
  return make_double2(t1, t2);
}

// FFTSpecial (decode) of one 2^14-slot vector per workgroup (see fft_inv_whole): buf [K][S] (bit-reversed
// by the CRT's scatter) -> the real parts of the first n slots in out.  STATS (flooded decrypts): the
// workgroup also sums decode_stats_kernel's statistics of its vector (fft_whole_flood_stats) into
// part[k]; flood_add_kernel then adds the noise to out (adding it here, beside the 16 values per thread,
// spilled under the 128-VGPR cap and ran slower than the extra pass).
template <bool STATS>
__global__ __launch_bounds__(1024) void fft_fwd_whole(const double2* __restrict__ buf, const double2* __restrict__ tw,
                                                      double* __restrict__ out, uint64_t n,
                                                      double2* __restrict__ part) {
  constexpr uint32_t S = 1u << kFftWholeLogS, BLK = 1024;
  constexpr int R = 16;
  __shared__ double lds[16 * kFftWholeRow];
  const uint64_t k = blockIdx.x;
  const uint32_t T = threadIdx.x, w = T >> 6, l = T & 63;
  double2 a[R];
  // block w: DIT half-sizes 1 .. 2 on sets l + 64 q (elements 4 (l + 64 q) + m), loaded from HBM
  const double2* __restrict__ g = buf + k * S + (uint64_t)w * BLK;
#pragma unroll
  for (int i = 0; i < R; ++i) a[i] = g[4 * (l + 64 * (i >> 2)) + (i & 3)];
  if (STATS) {
    const double2 st = fft_whole_flood_stats(a, lds);
    if (T == 0) part[k] = st;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    double2 c[4] = {a[4 * q], a[4 * q + 1], a[4 * q + 2], a[4 * q + 3]};
    fft_dit_set<2, 0>(c, 0u, tw);
#pragma unroll
    for (int m = 0; m < 4; ++m) a[4 * q + m] = c[m];
  }
  double* Ls = lds + w * kFftWholeRow;
  // (the empty asm statements keep each phase's twiddle loads in that phase: hoisted to the kernel
  // entry, 33 twiddles would not fit beside the data under the 128-VGPR cap)
  fft_wave_xch(a, Ls, [&](int m) { return fft_xa1(l, m); }, [&](int m) { return fft_xa2(l, m); });
  asm volatile("" ::: "memory");
  fft_dit_set<4, 2>(a, l & 3, tw);  // half-sizes 4 .. 32
  fft_wave_xch(a, Ls, [&](int m) { return fft_xb2(l, m); }, [&](int m) { return fft_xb3(l, m); });
  asm volatile("" ::: "memory");
  fft_dit_set<4, 6>(a, l, tw);  // half-sizes 64 .. 512
  asm volatile("" ::: "memory");
  fft_whole_transpose<false>(a, lds);
  // columns: DIT half-sizes 1024 .. 4096 on column T (fft_fwd_cols<4>); the last stage (8192) computes
  // only the real parts decrypt returns and stores each pair as it is done (with every output held to the
  // end, the column pass spilled under the 128-VGPR cap)
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    asm volatile("" ::: "memory");
    const uint32_t lenh = BLK << s;
    const int tr = 1 << s;
#pragma unroll
    for (int r0 = 0; r0 < R; ++r0) {
      if ((r0 >> s) & 1) continue;
      const int r1 = r0 + tr;
      const double2 W = tw[lenh + T + (uint32_t)(r0 & ((2 << s) - 1)) * BLK];
      const double2 u = a[r0];
      const double2 v = cmul(a[r1], W);
      a[r0] = cadd(u, v);
      a[r1] = csub(u, v);
    }
  }
  // uniform base + 32-bit offsets (16 precomputed 64-bit addresses would not fit)
  double* __restrict__ ok = out + k * S;
  const uint32_t rem = n > k * S ? (uint32_t)std::min<uint64_t>(n - k * S, S) : 0u;
#pragma unroll
  for (int r0 = 0; r0 < R / 2; ++r0) {
    asm volatile("" ::: "memory");
    const int r1 = r0 + R / 2;
    const double2 W = tw[(BLK << 3) + T + (uint32_t)r0 * BLK];
    const double vx = __dsub_rn(__dmul_rn(a[r1].x, W.x), __dmul_rn(a[r1].y, W.y));  // cmul(a[r1], W).x
    const uint32_t i0 = T + (uint32_t)r0 * BLK, i1 = T + (uint32_t)r1 * BLK;
    if (i0 < rem) ok[i0] = __dadd_rn(a[r0].x, vx);
    if (i1 < rem) ok[i1] = __dsub_rn(a[r0].x, vx);
  }
}

// The decode noise of a flooded whole-vector decode, added to the decoded outputs (fft_fwd_cols<LOGR,
// true>'s stream: slot i takes normal i div S/16 of ChaCha20 block i mod S/16): one thread per (ciphertext,
// block), 16 outputs each; sigma from the workgroup sums of fft_fwd_whole<true> (FloodArgs::part, G = 1).
__global__ __launch_bounds__(256) void flood_add_kernel(double* __restrict__ out, uint64_t n, uint32_t logS,
                                                        uint64_t K, FloodArgs fa) {
  const uint32_t S = 1u << logS, S16 = S >> 4;
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= K * S16) return;
  const uint64_t k = t / S16;
  const uint32_t b = (uint32_t)(t % S16);
  const double nso = flood_nsd(fa, k, b == 0 ? 0u : 1u, S) * sqrt((double)S);  // b == 0 records the flags
  uint64_t wd[8];
  chacha20_block(fa.key, b, (3ull << 56) | (fa.g0 + k), wd);
  double* __restrict__ ok = out + k * S;
  const uint32_t rem = n > k * S ? (uint32_t)std::min<uint64_t>(n - k * S, S) : 0u;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    double z0, z1;
    flood_pair(wd[m], z0, z1);
    const uint32_t i0 = b + S16 * (2 * m), i1 = i0 + S16;
    if (i0 < rem) ok[i0] = __dadd_rn(ok[i0], __dmul_rn(nso, z0));
    if (i1 < rem) ok[i1] = __dadd_rn(ok[i1], __dmul_rn(nso, z1));
  }
}

static uint32_t flood_groups(uint32_t S) {
  const uint32_t half = S / 2;
  return half >= kFloodPairsPerWg ? half / kFloodPairsPerWg : 1;
}

size_t decrypt_scratch_bytes(const Params& p, uint64_t K) {
  // dbuf [K][L][N] | fbuf [K][S] | flooding partial sums [K][G]
  return K * (uint64_t)p.L * p.N * sizeof(uint64_t) + K * (uint64_t)p.batch * sizeof(double2) +
         K * (uint64_t)flood_groups(p.batch) * sizeof(double2) + 64;
}

void launch_decrypt(const Params& p, const DeviceTables& dt, const DeviceKeys& dk,
                    const uint64_t* ct, uint64_t K, double scale, uint64_t n, double* out,
                    void* scratch, hipStream_t s, const DecodeNoise* dn, bool sum_in, uint32_t ct_L,
                    GenFlag crt_flag, bool exact) {
  if (!K) return;
  if (!ct_L) ct_L = p.L;
  if (ct_L < p.L) throw Error{SHELFI_ERR_ARG, "decrypt: fewer ciphertext towers than decoded towers"};
  exact = exact || dt.crt_nc == 0;  // towers too wide for crt_value's columns: always exact
  if (exact && !dt.crt_mw) throw Error{SHELFI_ERR_STATE, "decrypt: no exact CRT table for these towers"};
  if (!exact && !crt_flag.p) throw Error{SHELFI_ERR_STATE, "decrypt: the fast CRT needs a range flag"};
  const uint32_t logS = __builtin_ctz(p.batch);
  uint64_t* dbuf = reinterpret_cast<uint64_t*>(scratch);
  double2* fbuf = reinterpret_cast<double2*>(dbuf + K * (uint64_t)p.L * p.N);
  // c0 + c1*s formed in the first INTT pass (ntt_inv_blocks reading the ciphertexts); the
  // last pass fused with the CRT decode where its shape allows
  const uint32_t blkLog = ntt_block_log(p.logN);
  const int logR = (int)(p.logN - blkLog);
  const size_t fuse_lds = (size_t)p.L * 64 * sizeof(uint64_t) << (logR > 0 ? logR : 0);
  const bool fuse = !exact && logR > 0 && fuse_lds <= kCrtFuseLds && p.gap <= 64 &&
                    ((p.N >> logR) % 64) == 0;
  {
    const uint64_t P = K * p.L, nbBlocks = P << logR, nbCols = P * ((p.N >> logR) / 256);
    if (nbBlocks > 0x7FFFFFFFull) throw Error{SHELFI_ERR_ARG, "decrypt batch too large"};
    const uint32_t xg = xcd_combos(p.L << (logR > 0 ? logR : 0));
    // the persistent pass from kDecPpMinItems (ciphertext, tower, block) items: below, its per-workgroup
    // prologue is not amortised and the one-shot pass is faster (same dbuf bits)
    const bool pp = logR > 0 && blkLog == 11 && dt.red_ok && switches().dec_pp &&
                    K * ((uint64_t)p.L << logR) >= kDecPpMinItems;
    if (pp) {
      const uint32_t ncombo = p.L << logR;
      const uint32_t pc = pp_per_combo(ncombo, K, 3);
      if (sum_in)
        hipLaunchKernelGGL((ntt_inv_blocks_dec_pp<11, 2, 3, 3, 3, true>), dim3(ncombo * pc), dim3(256), 0, s, dbuf,
                           p.L, p.logN, dt.tw_inv_blk, dt.tc, ct, dk.sk, dk.sk_sh, (uint32_t)K, pc, ct_L);
      else if (ntt_wave_local())
        hipLaunchKernelGGL((ntt_inv_blocks_dec_pp<11, 2, 3, 3, 3, false, true>), dim3(ncombo * pc), dim3(256), 0, s,
                           dbuf, p.L, p.logN, dt.tw_inv_blk, dt.tc, ct, dk.sk, dk.sk_sh, (uint32_t)K, pc, ct_L);
      else
        hipLaunchKernelGGL((ntt_inv_blocks_dec_pp<11, 2, 3, 3, 3, false>), dim3(ncombo * pc), dim3(256), 0, s, dbuf,
                           p.L, p.logN, dt.tw_inv_blk, dt.tc, ct, dk.sk, dk.sk_sh, (uint32_t)K, pc, ct_L);
    } else if (logR > 0 && blkLog == 11 && dt.red_ok && !sum_in)
      hipLaunchKernelGGL((ntt_inv_blocks_dec_ct<11, 2, 3, 3, 3>), dim3((uint32_t)nbBlocks), dim3(256), 0,
                         s, dbuf, p.L, p.logN, dt.tw_inv_blk, dt.tc, ct, dk.sk, dk.sk_sh, xg, ct_L);
    else if (logR > 0 && blkLog == 11 && dt.red_ok)
      hipLaunchKernelGGL((ntt_inv_blocks_dec_ct<11, 2, 3, 3, 3, true>), dim3((uint32_t)nbBlocks), dim3(256), 0,
                         s, dbuf, p.L, p.logN, dt.tw_inv_blk, dt.tc, ct, dk.sk, dk.sk_sh, xg, ct_L);
    else if (logR > 0 && blkLog == 12 && dt.red_ok && !sum_in)
      hipLaunchKernelGGL((ntt_inv_blocks_dec_ct<12, 3, 3, 3, 3>), dim3((uint32_t)nbBlocks), dim3(256), 0,
                         s, dbuf, p.L, p.logN, dt.tw_inv_blk, dt.tc, ct, dk.sk, dk.sk_sh, xg, ct_L);
    else if (logR > 0 && blkLog == 12 && dt.red_ok)
      hipLaunchKernelGGL((ntt_inv_blocks_dec_ct<12, 3, 3, 3, 3, true>), dim3((uint32_t)nbBlocks), dim3(256), 0,
                         s, dbuf, p.L, p.logN, dt.tw_inv_blk, dt.tc, ct, dk.sk, dk.sk_sh, xg, ct_L);
    else
      hipLaunchKernelGGL(ntt_inv_blocks, dim3((uint32_t)nbBlocks), dim3(256), sizeof(uint64_t) << blkLog,
                         s, dbuf, p.L, p.logN, blkLog, dt.ipsi_rev, dt.ipsi_rev_sh, dt.tc,
                         logR == 0 ? 1 : 0, ct, dk.sk, dk.sk_sh, sum_in ? 1 : 0, ct_L);
    if (logR > 0 && fuse) {
      const uint64_t nbf = K * ((p.N >> logR) / 64);
#define CRT_FUSED(LR, NCC)                                                                                    \
  hipLaunchKernelGGL((ntt_inv_cols_crt<LR, NCC>), dim3((uint32_t)nbf), dim3(256), fuse_lds, s, dbuf, p.L, p.logN, \
                     logS, dt.ipsi_rev, dt.ipsi_rev_sh, dt.tc, 1.0 / scale, fbuf, crt_flag)
#define CRT_FUSED_NC(LR)                                  \
  if (dt.crt_nc == 5) CRT_FUSED(LR, 5);                   \
  else if (dt.crt_nc == 6) CRT_FUSED(LR, 6);              \
  else CRT_FUSED(LR, 7);
      switch (logR) {
        case 1: CRT_FUSED_NC(1) break;
        case 2: CRT_FUSED_NC(2) break;
        case 3: CRT_FUSED_NC(3) break;
        case 4: CRT_FUSED_NC(4) break;
        case 5: CRT_FUSED_NC(5) break;
        default: throw Error{SHELFI_ERR_ARG, "unsupported ring dimension"};
      }
#undef CRT_FUSED_NC
#undef CRT_FUSED
    } else if (logR > 0) {
      NTT_DISPATCH(logR, ntt_inv_cols, dim3((uint32_t)nbCols), dim3(256), 0, s, dbuf, p.L, p.logN,
                   dt.ipsi_rev, dt.ipsi_rev_sh, dt.tc);
    }
    SHELFI_HIP(hipGetLastError());
  }
  const uint64_t slots = K * (uint64_t)p.batch;
  if (!fuse) {
    const dim3 cg((uint32_t)((slots + 255) / 256));
    if (exact)
      hipLaunchKernelGGL((crt_decode_kernel<5, true>), cg, dim3(256), 0, s, dbuf, K, p.logN, logS, p.L, dt.tc,
                         dt.crt_mw, 1.0 / scale, fbuf, crt_flag);
    else if (dt.crt_nc == 5)
      hipLaunchKernelGGL((crt_decode_kernel<5>), cg, dim3(256), 0, s, dbuf, K, p.logN, logS, p.L, dt.tc,
                         dt.crt_mw, 1.0 / scale, fbuf, crt_flag);
    else if (dt.crt_nc == 6)
      hipLaunchKernelGGL((crt_decode_kernel<6>), cg, dim3(256), 0, s, dbuf, K, p.logN, logS, p.L, dt.tc,
                         dt.crt_mw, 1.0 / scale, fbuf, crt_flag);
    else
      hipLaunchKernelGGL((crt_decode_kernel<7>), cg, dim3(256), 0, s, dbuf, K, p.logN, logS, p.L, dt.tc,
                         dt.crt_mw, 1.0 / scale, fbuf, crt_flag);
  }
  SHELFI_HIP(hipGetLastError());
  const uint32_t fblkLog = fft_block_log(logS);
  const int flogR = (int)(logS - fblkLog);
  const size_t lds = sizeof(double2) << fblkLog;
  FloodArgs fa{};
  bool fused_flood = false;
  const bool whole = logS == kFftWholeLogS && K >= kFftWholeMinK && switches().fft_whole;  // fft_fwd_whole
  if (dn && dn->enabled) {
    for (int i = 0; i < 8; ++i) fa.key.k[i] = dn->key[i];
    fa.two_p = ldexp(1.0, (int)dn->p_bits);
    fa.p_bits = (double)dn->p_bits;
    fa.m_factor = dn->m_factor;
    fa.g0 = dn->g0;
    fa.flags = dn->flags;
    fa.fail = dn->fail;
    fa.logN = p.logN;
    fused_flood = p.batch >= 64;  // decode_flood_kernel below 2^6 slots
    if (fused_flood && whole) {  // fft_fwd_whole<true> sums its own statistics
      if (dn->reset) SHELFI_HIP(hipMemsetAsync(dn->flags + 1, 0, 8, s));
    } else if (fused_flood) {
      fa.G = flood_groups(p.batch);
      double2* part = fbuf + K * (uint64_t)p.batch;
      fa.part = part;
      hipLaunchKernelGGL(decode_stats_kernel, dim3((uint32_t)(K * fa.G)), dim3(256), 0, s, fbuf, logS, fa.G,
                         part, dn->reset ? dn->flags : (uint32_t*)nullptr);
    } else {
      if (dn->reset) SHELFI_HIP(hipMemsetAsync(dn->flags + 1, 0, 8, s));
      hipLaunchKernelGGL(decode_flood_kernel, dim3((uint32_t)K), dim3(1024), 0, s, fbuf, logS, p.logN,
                         fa.two_p, fa.p_bits, fa.m_factor, fa.key, fa.g0, fa.flags, fa.fail);
    }
    SHELFI_HIP(hipGetLastError());
  }
  if (whole) {  // one workgroup per vector, no HBM intermediate
    if (fused_flood) {
      double2* part = fbuf + K * (uint64_t)p.batch;  // [K] sums (G = 1)
      fa.part = part;
      fa.G = 1;
      hipLaunchKernelGGL(fft_fwd_whole<true>, dim3((uint32_t)K), dim3(1024), 0, s, fbuf, dt.fft_fwd, out, n, part);
      SHELFI_HIP(hipGetLastError());
      const uint64_t th = K * (p.batch >> 4);
      hipLaunchKernelGGL(flood_add_kernel, dim3((uint32_t)((th + 255) / 256)), dim3(256), 0, s, out, n, logS, K, fa);
    } else {
      hipLaunchKernelGGL(fft_fwd_whole<false>, dim3((uint32_t)K), dim3(1024), 0, s, fbuf, dt.fft_fwd, out, n,
                         (double2*)nullptr);
    }
    SHELFI_HIP(hipGetLastError());
    return;
  }
  const bool fct = flogR > 0 && (fblkLog == 10 || fblkLog == 11) && switches().fft_ct;
  const dim3 fg((uint32_t)(K << flogR));
  // the flooding noise lands on the pass that writes the output (fft_fwd_cols, or the single pass)
  if (fct && fblkLog == 10)
    hipLaunchKernelGGL((fft_fwd_blocks_ct<10, 3, 3, 2, 2>), fg, dim3(128), 0, s, fbuf, logS, dt.fft_fwd);
  else if (fct)
    hipLaunchKernelGGL((fft_fwd_blocks_ct<11, 3, 3, 3, 2>), fg, dim3(256), 0, s, fbuf, logS, dt.fft_fwd);
  else if (fused_flood && flogR == 0)
    hipLaunchKernelGGL(fft_fwd_blocks<true>, fg, dim3(256), lds, s, fbuf, logS, fblkLog, dt.fft_fwd, out, n, 1, fa);
  else
    hipLaunchKernelGGL(fft_fwd_blocks<false>, fg, dim3(256), lds, s, fbuf, logS,
                       fblkLog, dt.fft_fwd, out, n, flogR == 0 ? 1 : 0, fa);
  SHELFI_HIP(hipGetLastError());
  if (flogR > 0) {
    const uint64_t nb = K * ((p.batch >> flogR) / 256);
#define COLS_FWD(LR)                                                                                          \
  if (fused_flood)                                                                                            \
    hipLaunchKernelGGL((fft_fwd_cols<LR, true>), dim3((uint32_t)nb), dim3(256), 0, s, fbuf, logS, dt.fft_fwd, out, \
                       n, fa);                                                                                 \
  else                                                                                                        \
    hipLaunchKernelGGL((fft_fwd_cols<LR, false>), dim3((uint32_t)nb), dim3(256), 0, s, fbuf, logS, dt.fft_fwd,     \
                       out, n, fa);
    switch (flogR) {
      case 1: COLS_FWD(1) break;
      case 2: COLS_FWD(2) break;
      case 3: COLS_FWD(3) break;
      case 4: COLS_FWD(4) break;
      case 5: COLS_FWD(5) break;
      case 6: COLS_FWD(6) break;
      default: throw Error{SHELFI_ERR_ARG, "unsupported batch size"};
    }
#undef COLS_FWD
    SHELFI_HIP(hipGetLastError());
  }
}

// --------------------------------------------------------------- keygen ----
// s ternary (nonce 2<<56, words [0,N)), e Gaussian (words [N,2N)), a_t uniform
// (nonce (2<<56)|(1+t), word pair (2j, 2j+1) -> 128-bit value mod q_t).
__global__ __launch_bounds__(256) void keygen_sample_kernel(uint32_t logN, uint32_t L,
                                                            const TowerConst* __restrict__ tcs,
                                                            const uint64_t* __restrict__ cdt, int T,
                                                            Key8 key, uint64_t* __restrict__ se,
                                                            uint64_t* __restrict__ a_out) {
  const uint32_t N = 1u << logN;
  const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
  if (gid >= (N >> 3)) return;
  const uint32_t j0 = gid * 8;
  const uint64_t nonce = 2ull << 56;
  uint64_t rs[8], re[8];
  chacha20_block(key, j0 >> 3, nonce, rs);
  chacha20_block(key, (N >> 3) + (j0 >> 3), nonce, re);
  int64_t sv[8], ev[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    sv[u] = ternary_sample(rs[u]);
    ev[u] = gauss_sample(re[u], cdt, T);
  }
  for (uint32_t t = 0; t < L; ++t) {
    const TowerConst c = tcs[t];
    uint64_t ra[16];
    chacha20_block(key, j0 >> 2, nonce | (1 + t), ra);
    chacha20_block(key, (j0 >> 2) + 1, nonce | (1 + t), ra + 8);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      se[((uint64_t)0 * L + t) * N + j0 + u] = mod_signed_dev(sv[u], c);
      se[((uint64_t)1 * L + t) * N + j0 + u] = mod_signed_dev(ev[u], c);
      const uint64_t lo = ra[2 * u], hi = ra[2 * u + 1];
      a_out[(uint64_t)t * N + j0 + u] =
          addmod(shoup_mul(red64(hi, c.q, c.one_shoup), c.r64, c.r64_shoup, c.q),
                 red64(lo, c.q, c.one_shoup), c.q);
    }
  }
}

// sk = NTT(s); b = NTT(e) - a * NTT(s)
__global__ __launch_bounds__(256) void keygen_combine_kernel(const uint64_t* __restrict__ se,
                                                             uint32_t logN, uint32_t L,
                                                             const TowerConst* __restrict__ tcs,
                                                             uint64_t* __restrict__ sk,
                                                             uint64_t* __restrict__ pk) {
  const uint64_t LN = (uint64_t)L << logN;
  const uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= LN) return;
  const uint32_t t = (uint32_t)(e >> logN);
  const TowerConst c = tcs[t];
  const uint64_t s = se[e], er = se[LN + e], a = pk[LN + e];
  sk[e] = s;
  pk[e] = submod(er, mulmod_generic(a, s, c), c.q);
}

size_t keygen_scratch_bytes(const Params& p) { return 2ull * p.L * p.N * sizeof(uint64_t); }

void launch_keygen(const Params& p, const DeviceTables& dt, const uint32_t key[8], uint64_t* sk,
                   uint64_t* pk, void* scratch, hipStream_t s) {
  Key8 k8;
  for (int i = 0; i < 8; ++i) k8.k[i] = key[i];
  uint64_t* se = reinterpret_cast<uint64_t*>(scratch);
  const uint32_t th = p.N / 8;
  hipLaunchKernelGGL(keygen_sample_kernel, dim3((th + 255) / 256), dim3(256), 0, s, p.logN, p.L,
                     dt.tc, dt.cdt, dt.cdt_len, k8, se, pk + (uint64_t)p.L * p.N);
  SHELFI_HIP(hipGetLastError());
  launch_ntt(se, 2ull * p.L, p.L, p.logN, false, dt, s);
  const uint64_t LN = (uint64_t)p.L * p.N;
  hipLaunchKernelGGL(keygen_combine_kernel, dim3((uint32_t)((LN + 255) / 256)), dim3(256), 0, s,
                     se, p.logN, p.L, dt.tc, sk, pk);
  SHELFI_HIP(hipGetLastError());
}

}  // namespace shelfi

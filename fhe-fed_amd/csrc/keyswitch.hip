// keyswitch.hip — SURVEY §8 f4 on gfx950: ciphertext x ciphertext EvalMult with HYBRID
// relinearization, ModReduce (rescale), and EvalMultKeyGen.
//
// PALISADE 1.11 (the reference's library; ckks.cpp:28 builds its contexts with
// genCryptoContextCKKS, whose serialized parameters read ks = HYBRID, rs = EXACTRESCALE,
// dnum = 2: cryptocontext.txt@2514, key-eval-mult.txt@2699):
//   EvalMult(ct, ct')  c0 = a0 b0, c1 = a0 b1 + a1 b0, c2 = a1 b1, then KeySwitch(c2):
//     ModUp     digit j = towers [j alpha, (j+1) alpha) of Q_l, extended to every other
//               tower of Q_l u P by the fast basis conversion (ApproxSwitchCRTBasis):
//               y_t = sum_i [c_i (Q_j/q_i)^-1]_{q_i} (Q_j/q_i) mod t
//     inner     (u0, u1) = sum_j digit_j * (b_j, a_j)           over Q_l u P
//     ModDown   u - ApproxSwitchCRTBasis(P -> Q_l)(u_P), times P^-1 mod q_t
//     (c0, c1) += (u0, u1)
//   ModReduce  (DCRTPoly::DropLastElementAndScale) c_t <- (c_t - [c_l]) q_l^-1 mod q_t,
//              [c_l] = the last tower's coefficients lifted centred (NativeVector::
//              SwitchModulus), i.e. round(c / q_l).
//   EvalMultKeyGen (KeySwitchHYBRID::KeySwitchGen, s' = s^2):
//     b_j = -a_j s + e_j + [t in digit j] (P mod q_t) s^2,  a_j uniform over Q u P.
//
// Every kernel is elementwise or a per-coefficient basis conversion (no twiddles): one
// thread per coefficient, one block per 256 coefficients of one row, rows tower-uniform
// so the tower constants are scalar loads.  The NTTs in between are launch_ntt's.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dev_common.h"
#include "shelfi_internal.h"

namespace shelfi {

typedef unsigned __int128 du128;

#define NTT_DISPATCH_KS(LOGRV, KERNEL, ...)                                               \
  switch (LOGRV) {                                                                       \
    case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break;                           \
    case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;                           \
    case 3: hipLaunchKernelGGL(KERNEL<3>, __VA_ARGS__); break;                           \
    case 4: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;                           \
    case 5: hipLaunchKernelGGL(KERNEL<5>, __VA_ARGS__); break;                           \
    case 6: hipLaunchKernelGGL(KERNEL<6>, __VA_ARGS__); break;                           \
    default: throw Error{SHELFI_ERR_ARG, "EvalMult: unsupported ring dimension"};        \
  }

// sum of products (< 2^124) -> [0, q)
__device__ __forceinline__ uint64_t red128(du128 acc, const TowerConst& c) {
  const uint64_t hi = (uint64_t)(acc >> 64), lo = (uint64_t)acc;
  return addmod(shoup_mul(hi, c.r64, c.r64_shoup, c.q), red64(lo, c.q, c.one_shoup), c.q);
}
__device__ __forceinline__ du128 mul128(uint64_t a, uint64_t b) { return (du128)a * b; }

// Digit j of a level owns towers [j alpha, j alpha + cnt) of Q_l; its "foreign" towers (the
// rest of Q_l, then P) are the ones ModUp must produce, stored in that order (index u =
// t < s ? t : t - cnt) so every NTT over them is a plain batch with per-digit tables.
__device__ __forceinline__ void digit_span(const KsArgs& a, uint32_t j, uint32_t& s, uint32_t& cnt) {
  s = j * a.alpha;
  cnt = min(a.alpha, a.Ll - s);
}
__device__ __forceinline__ uint64_t ext_base(const KsArgs& a, uint32_t j, uint64_t K) {
  uint64_t base = 0;
  for (uint32_t i = 0; i < j; ++i) {
    uint32_t s, cnt;
    digit_span(a, i, s, cnt);
    base += (uint64_t)(a.T - cnt) * K;  // in polynomials
  }
  return base << a.logN;
}

// ------------------------------------------------ tensor + first INTT pass ----
// One workgroup per (ct, tower, block): c0 = a0 b0 and c1 = a0 b1 + a1 b0 go to `out`,
// c2 = a1 b1 to d2e (EVALUATION, kept for the digits' own towers) and into LDS, where the
// first inverse stages run; the lazy block goes to d2c for the columns pass (or, for a
// single-block ring, the scaled canonical coefficients).
// (x, y and out may alias: each element is read before it is written, by the same thread)
__global__ __launch_bounds__(256) void ks_tensor_intt_kernel(const uint64_t* x, const uint64_t* y, uint32_t Ll,
                                                             uint32_t logN, uint32_t blkLog,
                                                             const uint64_t* __restrict__ itw,
                                                             const uint64_t* __restrict__ itwp,
                                                             const TowerConst* __restrict__ tq, uint64_t* out,
                                                             uint64_t* __restrict__ d2e,
                                                             uint64_t* __restrict__ d2c) {
  extern __shared__ __attribute__((aligned(16))) uint64_t sm[];
  const uint32_t N = 1u << logN, blk = 1u << blkLog, sh = logN - blkLog;
  const uint64_t row = blockIdx.x >> sh;  // k * Ll + t
  const uint32_t b = blockIdx.x & ((1u << sh) - 1);
  const uint64_t k = row / Ll;
  const uint32_t t = (uint32_t)(row % Ll);
  const TowerConst c = tq[t];
  const uint64_t q = c.q;
  const uint64_t off = ((uint64_t)t << logN) + ((uint64_t)b << blkLog);
  const uint64_t i0 = ((k * 2 * Ll) << logN) + off, i1 = (((k * 2 + 1) * Ll) << logN) + off;
  const uint64_t id = (row << logN) + ((uint64_t)b << blkLog);
  const ulonglong2* A0 = reinterpret_cast<const ulonglong2*>(x + i0);
  const ulonglong2* A1 = reinterpret_cast<const ulonglong2*>(x + i1);
  const ulonglong2* B0 = reinterpret_cast<const ulonglong2*>(y + i0);
  const ulonglong2* B1 = reinterpret_cast<const ulonglong2*>(y + i1);
  ulonglong2* O0 = reinterpret_cast<ulonglong2*>(out + i0);
  ulonglong2* O1 = reinterpret_cast<ulonglong2*>(out + i1);
  ulonglong2* E2 = reinterpret_cast<ulonglong2*>(d2e + id);
  for (uint32_t p = threadIdx.x; p < blk / 2; p += 256) {
    const ulonglong2 a0 = A0[p], a1 = A1[p], b0 = B0[p], b1 = B1[p];
    const ulonglong2 r0 = make_ulonglong2(mulmod_generic(a0.x, b0.x, c), mulmod_generic(a0.y, b0.y, c));
    const ulonglong2 r1 =
        make_ulonglong2(addmod(mulmod_generic(a0.x, b1.x, c), mulmod_generic(a1.x, b0.x, c), q),
                        addmod(mulmod_generic(a0.y, b1.y, c), mulmod_generic(a1.y, b0.y, c), q));
    const ulonglong2 r2 = make_ulonglong2(mulmod_generic(a1.x, b1.x, c), mulmod_generic(a1.y, b1.y, c));
    O0[p] = r0;
    O1[p] = r1;
    E2[p] = r2;
    lds_put2(sm, p, r2);
  }
  __syncthreads();
  ntt_inv_block_stages(sm, blkLog, b, logN, itw + (uint64_t)t * N, itwp + (uint64_t)t * N, q);
  ulonglong2* D = reinterpret_cast<ulonglong2*>(d2c + id);
  if (sh == 0) {
    for (uint32_t p = threadIdx.x; p < blk / 2; p += 256) {
      const ulonglong2 v = lds_get2(sm, p);
      D[p] = make_ulonglong2(canon4(shoup_lazy(v.x, c.ninv, c.ninv_shoup, q), q),
                             canon4(shoup_lazy(v.y, c.ninv, c.ninv_shoup, q), q));
    }
  } else {  // lazy values in [0, 4q): the columns pass canonicalises
    for (uint32_t p = threadIdx.x; p < blk / 2; p += 256) D[p] = lds_get2(sm, p);
  }
}

// ----------------------------------------------------------------- ModUp ----
// c [K][Ll][N] (COEFFICIENT) -> digit j's foreign towers ext_j [K][T - cnt][N]
// (COEFFICIENT) by the fast basis conversion.
__global__ __launch_bounds__(256) void modup_kernel(const uint64_t* __restrict__ c, uint64_t K,
                                                    KsArgs a, uint64_t* __restrict__ ext) {
  const uint32_t N = 1u << a.logN, bpr = N >> 8;
  const uint64_t row = blockIdx.x / bpr;  // j * K + k
  const uint32_t n = (blockIdx.x % bpr) * 256 + threadIdx.x;
  const uint32_t j = (uint32_t)(row / K);
  const uint64_t k = row % K;
  uint32_t s, cnt;
  digit_span(a, j, s, cnt);
  uint64_t yv[kMaxTowers];
  for (uint32_t i = 0; i < cnt; ++i) {
    const TowerConst ci = a.tq[s + i];
    yv[i] = shoup_mul(c[((k * a.Ll + s + i) << a.logN) + n], a.mu_inv[j * a.alpha + i],
                      a.mu_inv_sh[j * a.alpha + i], ci.q);
  }
  const uint32_t Tf = a.T - cnt;
  uint64_t* __restrict__ o = ext + ext_base(a, j, K) + ((k * Tf) << a.logN) + n;
  for (uint32_t u = 0; u < Tf; ++u) {
    const uint32_t t = u < s ? u : u + cnt;
    du128 acc = 0;
    const uint64_t* __restrict__ h = a.mu_hat + (uint64_t)j * a.alpha * a.T + t;
    for (uint32_t i = 0; i < cnt; ++i) acc += mul128(yv[i], h[(uint64_t)i * a.T]);
    o[(uint64_t)u << a.logN] = red128(acc, a.te[t]);
  }
}

// ModUp fused with the first NTT stages (rings with a columns pass): one thread per
// (digit, ct, column of R = 2^LOGR rows).  It converts its R coefficients of the digit's
// towers once (y_i = [c_i (Q_j/q_i)^-1]_{q_i}, kept in registers), then for every foreign
// tower forms the column by the basis conversion, runs the LOGR register stages with that
// tower's twiddles and writes the lazy column — the coefficient-domain extension never
// round-trips through HBM.  (Recomputing y per tower instead, to drop to 97 VGPRs / 4 waves,
// measured slower: 11.7 vs 11.0 us per product at 2^15/L4.)
template <int LOGR>
__global__ __launch_bounds__(256) void modup_cols_kernel(const uint64_t* __restrict__ c, uint64_t K, KsArgs a,
                                                         const uint64_t* __restrict__ tw,
                                                         const uint64_t* __restrict__ twp,
                                                         uint64_t* __restrict__ ext) {
  constexpr int R = 1 << LOGR;
  const uint32_t N = 1u << a.logN, BLK = N >> LOGR, bpp = BLK / 256;
  const uint64_t row = blockIdx.x / bpp;  // j * K + k
  const uint32_t col = (blockIdx.x % bpp) * 256 + threadIdx.x;
  const uint32_t j = (uint32_t)(row / K);
  const uint64_t k = row % K;
  uint32_t s, cnt;
  digit_span(a, j, s, cnt);
  // the digit's converted coefficients, [i][r] (cnt <= 2 here: launch_eval_mult checks)
  uint64_t y[2][R];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if ((uint32_t)i < cnt) {
      const TowerConst ci = a.tq[s + i];
      const uint64_t w = a.mu_inv[j * a.alpha + i], wp = a.mu_inv_sh[j * a.alpha + i];
      const uint64_t* __restrict__ src = c + ((k * a.Ll + s + i) << a.logN) + col;
#pragma unroll
      for (int r = 0; r < R; ++r) y[i][r] = shoup_mul(src[(uint64_t)r * BLK], w, wp, ci.q);
    }
  }
  const uint32_t Tf = a.T - cnt;
  uint64_t* __restrict__ o = ext + ext_base(a, j, K) + ((k * Tf) << a.logN) + col;
  for (uint32_t u = 0; u < Tf; ++u) {
    const uint32_t t = u < s ? u : u + cnt;
    const TowerConst ct = a.te[t];
    const uint64_t h0 = a.mu_hat[(uint64_t)j * a.alpha * a.T + t];
    const uint64_t h1 = cnt > 1 ? a.mu_hat[((uint64_t)j * a.alpha + 1) * a.T + t] : 0;
    uint64_t x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      du128 acc = mul128(y[0][r], h0);
      if (cnt > 1) acc += mul128(y[1][r], h1);
      x[r] = red128(acc, ct);
    }
    const uint64_t* __restrict__ w = tw + (uint64_t)t * N;
    const uint64_t* __restrict__ wp = twp + (uint64_t)t * N;
#pragma unroll
    for (int st = 0; st < LOGR; ++st) {
      const int m = 1 << st, tr = R >> (st + 1);
#pragma unroll
      for (int i = 0; i < m; ++i) {
        const uint64_t W = w[m + i], Wp = wp[m + i];
#pragma unroll
        for (int jj = 0; jj < tr; ++jj) {
          const int r0 = 2 * i * tr + jj, r1 = r0 + tr;
          ct_bfly(x[r0], x[r1], W, Wp, ct.q);
        }
      }
    }
    uint64_t* __restrict__ ou = o + ((uint64_t)u << a.logN);
#pragma unroll
    for (int r = 0; r < R; ++r) ou[(uint64_t)r * BLK] = x[r];
  }
}

// ModDown's P -> Q_l conversion fused with z's first NTT stages: one thread per (ct, poly,
// column), y_m of the special towers in registers (kP <= 2 here), then per target tower the
// conversion, the LOGR register stages and the lazy write.
template <int LOGR>
__global__ __launch_bounds__(256) void moddown_cols_kernel(const uint64_t* __restrict__ accP, KsArgs a,
                                                           const uint64_t* __restrict__ tw,
                                                           const uint64_t* __restrict__ twp,
                                                           uint64_t* __restrict__ z) {
  constexpr int R = 1 << LOGR;
  const uint32_t N = 1u << a.logN, BLK = N >> LOGR, bpp = BLK / 256;
  const uint64_t row = blockIdx.x / bpp;  // k * 2 + poly
  const uint32_t col = (blockIdx.x % bpp) * 256 + threadIdx.x;
  uint64_t y[2][R];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    if ((uint32_t)m < a.kP) {
      const TowerConst cp = a.te[a.Ll + m];
      const uint64_t* __restrict__ src = accP + ((row * a.kP + m) << a.logN) + col;
#pragma unroll
      for (int r = 0; r < R; ++r) y[m][r] = shoup_mul(src[(uint64_t)r * BLK], a.md_inv[m], a.md_inv_sh[m], cp.q);
    }
  }
  for (uint32_t t = 0; t < a.Ll; ++t) {
    const TowerConst ct = a.tq[t];
    const uint64_t h0 = a.md_hat[t], h1 = a.kP > 1 ? a.md_hat[(uint64_t)a.Ll + t] : 0;
    uint64_t x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      du128 acc = mul128(y[0][r], h0);
      if (a.kP > 1) acc += mul128(y[1][r], h1);
      x[r] = red128(acc, ct);
    }
    const uint64_t* __restrict__ w = tw + (uint64_t)t * N;
    const uint64_t* __restrict__ wp = twp + (uint64_t)t * N;
#pragma unroll
    for (int st = 0; st < LOGR; ++st) {
      const int m = 1 << st, tr = R >> (st + 1);
#pragma unroll
      for (int i = 0; i < m; ++i) {
        const uint64_t W = w[m + i], Wp = wp[m + i];
#pragma unroll
        for (int jj = 0; jj < tr; ++jj) {
          const int r0 = 2 * i * tr + jj, r1 = r0 + tr;
          ct_bfly(x[r0], x[r1], W, Wp, ct.q);
        }
      }
    }
    uint64_t* __restrict__ ot = z + ((row * a.Ll + t) << a.logN) + col;
#pragma unroll
    for (int r = 0; r < R; ++r) ot[(uint64_t)r * BLK] = x[r];
  }
}

// ------------------------------------- last NTT pass + key inner product ----
// One workgroup per (ct, tower t of Q_l u P, block): every digit j's block of tower t in
// EVALUATION — straight from d2e when t is one of the digit's own towers, else the foreign
// block after its last NTT stages in LDS slot j — is multiplied by the key (b_j, a_j) and
// summed; (u0, u1) go to accQ / accP.  The extended polynomials never return to HBM in
// EVALUATION form.  All digits' blocks sit in LDS together (dn x 16 KiB at 2^11 blocks), so
// the products are formed in one pass with nothing held in registers across digits.
__global__ __launch_bounds__(256) void ks_inner_blocks_kernel(const uint64_t* __restrict__ d2e,
                                                              const uint64_t* __restrict__ ext, uint64_t K,
                                                              KsArgs a, uint32_t blkLog,
                                                              const uint64_t* __restrict__ tw,
                                                              const uint64_t* __restrict__ twp,
                                                              const uint64_t* __restrict__ evk,
                                                              const uint64_t* __restrict__ evk_sh,
                                                              uint64_t* __restrict__ accQ,
                                                              uint64_t* __restrict__ accP) {
  extern __shared__ __attribute__((aligned(16))) uint64_t sm[];
  const uint32_t N = 1u << a.logN, blk = 1u << blkLog, sh = a.logN - blkLog;
  const uint64_t row = blockIdx.x >> sh;  // k * T + t
  const uint32_t b = blockIdx.x & ((1u << sh) - 1);
  const uint64_t k = row / a.T;
  const uint32_t t = (uint32_t)(row % a.T);
  const TowerConst c = a.te[t];
  const uint64_t q = c.q;
  const uint32_t TF = a.Lfull + a.kP;
  const uint32_t tk = t < a.Ll ? t : a.Lfull + (t - a.Ll);  // the key's tower
  const uint64_t boff = (uint64_t)b << blkLog;
  uint32_t own_mask = 0;
  for (uint32_t j = 0; j < a.dn; ++j) {
    uint32_t s, cnt;
    digit_span(a, j, s, cnt);
    if (t >= s && t < s + cnt) {
      own_mask |= 1u << j;
      continue;
    }
    const uint32_t u = t < s ? t : t - cnt;
    const ulonglong2* src = reinterpret_cast<const ulonglong2*>(
        ext + ext_base(a, j, K) + ((k * (a.T - cnt) + u) << a.logN) + boff);
    for (uint32_t p = threadIdx.x; p < blk / 2; p += 256) lds_put2(sm + ((uint64_t)j << blkLog), p, src[p]);
  }
  __syncthreads();
  for (uint32_t j = 0; j < a.dn; ++j)
    if (!(own_mask & (1u << j)))
      ntt_fwd_block_stages(sm + ((uint64_t)j << blkLog), blkLog, b, a.logN, tw + (uint64_t)t * N,
                           twp + (uint64_t)t * N, q);
  const ulonglong2* own_src = reinterpret_cast<const ulonglong2*>(d2e + ((k * a.Ll + t) << a.logN) + boff);
  ulonglong2 *o0, *o1;
  if (t < a.Ll) {
    o0 = reinterpret_cast<ulonglong2*>(accQ + ((((k * 2 + 0) * a.Ll + t)) << a.logN) + boff);
    o1 = reinterpret_cast<ulonglong2*>(accQ + ((((k * 2 + 1) * a.Ll + t)) << a.logN) + boff);
  } else {
    const uint32_t m = t - a.Ll;
    o0 = reinterpret_cast<ulonglong2*>(accP + ((((k * 2 + 0) * a.kP + m)) << a.logN) + boff);
    o1 = reinterpret_cast<ulonglong2*>(accP + ((((k * 2 + 1) * a.kP + m)) << a.logN) + boff);
  }
  for (uint32_t p = threadIdx.x; p < blk / 2; p += 256) {
    ulonglong2 u0 = make_ulonglong2(0, 0), u1 = make_ulonglong2(0, 0);
    for (uint32_t j = 0; j < a.dn; ++j) {
      ulonglong2 v;
      if (own_mask & (1u << j)) {
        v = own_src[p];
      } else {
        v = lds_get2(sm + ((uint64_t)j << blkLog), p);
        v = make_ulonglong2(canon8(v.x, q), canon8(v.y, q));
      }
      const uint64_t kb = ((((uint64_t)j * TF + tk)) << a.logN) + boff + 2ull * p;
      const uint64_t ka = ((((uint64_t)(a.dnFull + j) * TF + tk)) << a.logN) + boff + 2ull * p;
      const ulonglong2 bv = *reinterpret_cast<const ulonglong2*>(evk + kb);
      const ulonglong2 bs = *reinterpret_cast<const ulonglong2*>(evk_sh + kb);
      const ulonglong2 av = *reinterpret_cast<const ulonglong2*>(evk + ka);
      const ulonglong2 as = *reinterpret_cast<const ulonglong2*>(evk_sh + ka);
      u0.x = addmod(u0.x, shoup_mul(v.x, bv.x, bs.x, q), q);
      u0.y = addmod(u0.y, shoup_mul(v.y, bv.y, bs.y, q), q);
      u1.x = addmod(u1.x, shoup_mul(v.x, av.x, as.x, q), q);
      u1.y = addmod(u1.y, shoup_mul(v.y, av.y, as.y, q), q);
    }
    o0[p] = u0;
    o1[p] = u1;
  }
}

// The same inner product at compile-time shape: every foreign digit's block runs its last
// stages through fwd_block_pass_ct (first chunk straight from ext, per-block twiddle slices of
// the extended basis) and leaves canonical residues in its own padded LDS slot; then the key
// products are summed as above.  Dynamic LDS: dn slots of lpad_size(BL) u64.
template <int BL, int K1, int K2, int K3, int K4>
__global__ __launch_bounds__(256) void ks_inner_blocks_ct(const uint64_t* __restrict__ d2e,
                                                          const uint64_t* __restrict__ ext, uint64_t K, KsArgs a,
                                                          const ulonglong2* __restrict__ twb,
                                                          const uint64_t* __restrict__ evk,
                                                          const uint64_t* __restrict__ evk_sh,
                                                          uint64_t* __restrict__ accQ, uint64_t* __restrict__ accP) {
  extern __shared__ __attribute__((aligned(16))) uint64_t sm[];
  constexpr uint32_t SL = lpad_size(BL);
  const uint32_t sh = a.logN - BL;
  const uint64_t row = blockIdx.x >> sh;  // k * T + t
  const uint32_t b = blockIdx.x & ((1u << sh) - 1);
  const uint64_t k = row / a.T;
  const uint32_t t = (uint32_t)(row % a.T);
  const TowerConst& c = a.te[t];
  const uint64_t q = c.q;
  const uint32_t TF = a.Lfull + a.kP;
  const uint32_t tk = t < a.Ll ? t : a.Lfull + (t - a.Ll);  // the key's tower
  const uint64_t boff = (uint64_t)b << BL;
  const ulonglong2* __restrict__ tb = twb + ((uint64_t)t << a.logN) + boff;
  uint32_t own_mask = 0;
  for (uint32_t j = 0; j < a.dn; ++j) {
    uint32_t s, cnt;
    digit_span(a, j, s, cnt);
    if (t >= s && t < s + cnt) {
      own_mask |= 1u << j;
      continue;
    }
    const uint32_t u = t < s ? t : t - cnt;
    uint64_t* slot = sm + (uint64_t)j * SL;
    fwd_block_pass_ct<BL, K1, K2, K3, K4>(ext + ext_base(a, j, K) + ((k * (a.T - cnt) + u) << a.logN) + boff, tb,
                                          q, c.n8q, slot, [&](uint32_t j0, auto& x) {
                                            const uint32_t pj0 = lpad(j0);
#pragma unroll
                                            for (int m = 0; m < (1 << K4); ++m) slot[pj0 + m] = red_any(x[m], c);
                                          });
  }
  __syncthreads();
  const ulonglong2* own_src = reinterpret_cast<const ulonglong2*>(d2e + ((k * a.Ll + t) << a.logN) + boff);
  ulonglong2 *o0, *o1;
  if (t < a.Ll) {
    o0 = reinterpret_cast<ulonglong2*>(accQ + ((((k * 2 + 0) * a.Ll + t)) << a.logN) + boff);
    o1 = reinterpret_cast<ulonglong2*>(accQ + ((((k * 2 + 1) * a.Ll + t)) << a.logN) + boff);
  } else {
    const uint32_t m = t - a.Ll;
    o0 = reinterpret_cast<ulonglong2*>(accP + ((((k * 2 + 0) * a.kP + m)) << a.logN) + boff);
    o1 = reinterpret_cast<ulonglong2*>(accP + ((((k * 2 + 1) * a.kP + m)) << a.logN) + boff);
  }
  for (uint32_t p = threadIdx.x; p < (1u << BL) / 2; p += 256) {
    ulonglong2 u0 = make_ulonglong2(0, 0), u1 = make_ulonglong2(0, 0);
    for (uint32_t j = 0; j < a.dn; ++j) {
      const ulonglong2 v = (own_mask & (1u << j))
                               ? own_src[p]
                               : *reinterpret_cast<const ulonglong2*>(sm + (uint64_t)j * SL + lpad(2 * p));
      const uint64_t kb = ((((uint64_t)j * TF + tk)) << a.logN) + boff + 2ull * p;
      const uint64_t ka = ((((uint64_t)(a.dnFull + j) * TF + tk)) << a.logN) + boff + 2ull * p;
      const ulonglong2 bv = *reinterpret_cast<const ulonglong2*>(evk + kb);
      const ulonglong2 bs = *reinterpret_cast<const ulonglong2*>(evk_sh + kb);
      const ulonglong2 av = *reinterpret_cast<const ulonglong2*>(evk + ka);
      const ulonglong2 as = *reinterpret_cast<const ulonglong2*>(evk_sh + ka);
      u0.x = addmod(u0.x, shoup_mul(v.x, bv.x, bs.x, q), q);
      u0.y = addmod(u0.y, shoup_mul(v.y, bv.y, bs.y, q), q);
      u1.x = addmod(u1.x, shoup_mul(v.x, av.x, as.x, q), q);
      u1.y = addmod(u1.y, shoup_mul(v.y, av.y, as.y, q), q);
    }
    o0[p] = u0;
    o1[p] = u1;
  }
}

// --------------------------------------------------------------- ModDown ----
// accP [K][2][kP][N] (COEFFICIENT) -> z [K][2][Ll][N] (COEFFICIENT), P -> Q_l conversion
__global__ __launch_bounds__(256) void moddown_kernel(const uint64_t* __restrict__ accP, KsArgs a,
                                                      uint64_t* __restrict__ z) {
  const uint32_t N = 1u << a.logN, bpr = N >> 8;
  const uint64_t row = blockIdx.x / bpr;  // k * 2 + poly
  const uint32_t n = (blockIdx.x % bpr) * 256 + threadIdx.x;
  uint64_t yv[kMaxTowers];
  for (uint32_t m = 0; m < a.kP; ++m) {
    const TowerConst cp = a.te[a.Ll + m];
    yv[m] = shoup_mul(accP[(row * a.kP + m) * N + n], a.md_inv[m], a.md_inv_sh[m], cp.q);
  }
  for (uint32_t t = 0; t < a.Ll; ++t) {
    du128 acc = 0;
    for (uint32_t m = 0; m < a.kP; ++m) acc += mul128(yv[m], a.md_hat[(uint64_t)m * a.Ll + t]);
    z[(row * a.Ll + t) * N + n] = red128(acc, a.tq[t]);
  }
}

// ------------------------------------- last NTT pass of z + the ModDown finish ----
// out[k][poly][t] += (accQ - NTT(z)) P^-1 mod q_t, z's last stages in LDS
__global__ __launch_bounds__(256) void ks_finish_blocks_kernel(const uint64_t* __restrict__ z,
                                                               const uint64_t* __restrict__ accQ, KsArgs a,
                                                               uint32_t blkLog, const uint64_t* __restrict__ tw,
                                                               const uint64_t* __restrict__ twp,
                                                               uint64_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint64_t sm[];
  const uint32_t N = 1u << a.logN, blk = 1u << blkLog, sh = a.logN - blkLog;
  const uint64_t row = blockIdx.x >> sh;  // (k * 2 + poly) * Ll + t
  const uint32_t b = blockIdx.x & ((1u << sh) - 1);
  const uint32_t t = (uint32_t)(row % a.Ll);
  const TowerConst c = a.tq[t];
  const uint64_t q = c.q, pinv = a.pinv[t], pinv_sh = a.pinv_sh[t];
  const uint64_t off = (row << a.logN) + ((uint64_t)b << blkLog);
  const ulonglong2* Z = reinterpret_cast<const ulonglong2*>(z + off);
  for (uint32_t p = threadIdx.x; p < blk / 2; p += 256) lds_put2(sm, p, Z[p]);
  __syncthreads();
  ntt_fwd_block_stages(sm, blkLog, b, a.logN, tw + (uint64_t)t * N, twp + (uint64_t)t * N, q);
  const ulonglong2* AQ = reinterpret_cast<const ulonglong2*>(accQ + off);
  ulonglong2* O = reinterpret_cast<ulonglong2*>(out + off);
  for (uint32_t p = threadIdx.x; p < blk / 2; p += 256) {
    const ulonglong2 v = lds_get2(sm, p), aq = AQ[p], o = O[p];
    const uint64_t dx = submod(aq.x, canon8(v.x, q), q), dy = submod(aq.y, canon8(v.y, q), q);
    O[p] = make_ulonglong2(addmod(o.x, shoup_mul(dx, pinv, pinv_sh, q), q),
                           addmod(o.y, shoup_mul(dy, pinv, pinv_sh, q), q));
  }
}

// The same finish at compile-time shape (fwd_block_pass_ct over the per-block twiddle slices
// tw_fwd_blk; needs logN > BL and every q_t >= 2^40 for red_any): z's last stages run on the
// registers of the chunk passes and the finish reads them from registers.
template <int BL, int K1, int K2, int K3, int K4>
__global__ __launch_bounds__(256) void ks_finish_blocks_ct(const uint64_t* __restrict__ z,
                                                           const uint64_t* __restrict__ accQ, KsArgs a,
                                                           const ulonglong2* __restrict__ twb,
                                                           uint64_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint64_t sm[lpad_size(BL)];
  const uint32_t sh = a.logN - BL;
  const uint64_t row = blockIdx.x >> sh;  // (k * 2 + poly) * Ll + t
  const uint32_t b = blockIdx.x & ((1u << sh) - 1);
  const uint32_t t = (uint32_t)(row % a.Ll);
  const TowerConst& c = a.tq[t];
  const uint64_t q = c.q, pinv = a.pinv[t], pinv_sh = a.pinv_sh[t];
  const uint64_t off = (row << a.logN) + ((uint64_t)b << BL);
  const ulonglong2* __restrict__ tb = twb + ((uint64_t)t << a.logN) + ((uint64_t)b << BL);
  fwd_block_pass_ct<BL, K1, K2, K3, K4>(z + off, tb, q, c.n8q, sm, [&](uint32_t j0, auto& x) {
#pragma unroll
    for (int m = 0; m < (1 << K4); m += 2) {
      const ulonglong2 aq = *reinterpret_cast<const ulonglong2*>(accQ + off + j0 + m);
      ulonglong2* O = reinterpret_cast<ulonglong2*>(out + off + j0 + m);
      const ulonglong2 o = *O;
      const uint64_t dx = submod(aq.x, red_any(x[m], c), q), dy = submod(aq.y, red_any(x[m + 1], c), q);
      *O = make_ulonglong2(addmod(o.x, shoup_mul(dx, pinv, pinv_sh, q), q),
                           addmod(o.y, shoup_mul(dy, pinv, pinv_sh, q), q));
    }
  });
}

size_t ks_scratch_bytes(uint32_t Ll, uint32_t kP, uint32_t dn, uint32_t alpha, uint32_t N, uint64_t K) {
  const uint64_t T = Ll + kP;
  uint64_t ext = 0;
  for (uint32_t j = 0; j < dn; ++j) ext += T - std::min(alpha, Ll - j * alpha);
  // d2e | d2c | ext | accQ | accP | z
  return K * (uint64_t)N * 8 * (2ull * Ll + ext + 2ull * Ll + 2ull * kP + 2ull * Ll) + 64;
}

void launch_eval_mult(const KsArgs& a, const DeviceTables& dtq, const DeviceTables& dte,
                      const DeviceTables* dtf, const uint64_t* evk, const uint64_t* evk_sh, const uint64_t* x,
                      const uint64_t* y, uint64_t K, uint64_t* out, void* scratch, hipStream_t s) {
  if (!K) return;
  const uint32_t N = 1u << a.logN, bpr = N >> 8;
  const uint32_t blkLog = ntt_block_log(a.logN), sh = a.logN - blkLog;
  const size_t lds = sizeof(uint64_t) << blkLog;
  const uint64_t KN = K * N;
  uint64_t* d2e = reinterpret_cast<uint64_t*>(scratch);
  uint64_t* d2c = d2e + KN * a.Ll;
  uint64_t* ext = d2c + KN * a.Ll;
  uint64_t next = 0;
  for (uint32_t j = 0; j < a.dn; ++j) next += a.T - std::min(a.alpha, a.Ll - j * a.alpha);
  uint64_t* accQ = ext + KN * next;
  uint64_t* accP = accQ + KN * 2 * a.Ll;
  uint64_t* z = accP + KN * 2 * a.kP;
  auto grid = [&](uint64_t rows, uint32_t per_row) {
    const uint64_t b = rows * per_row;
    if (b > 0x7FFFFFFFull) throw Error{SHELFI_ERR_ARG, "EvalMult batch too large"};
    return dim3((uint32_t)b);
  };
  const uint32_t nb = 1u << sh;
  // tensor -> c0, c1 (out), c2 (EVALUATION) + first INTT pass; then the INTT columns pass
  hipLaunchKernelGGL(ks_tensor_intt_kernel, grid(K * a.Ll, nb), dim3(256), lds, s, x, y, a.Ll, a.logN, blkLog,
                     dtq.ipsi_rev, dtq.ipsi_rev_sh, a.tq, out, d2e, d2c);
  SHELFI_HIP(hipGetLastError());
  launch_ntt_cols(d2c, K * a.Ll, a.Ll, a.logN, true, dtq, s);
  // ModUp of every digit's foreign towers with their first NTT stages: fused when the ring has
  // a columns pass and digits / special primes have <= 2 towers; else modup_kernel, then a
  // columns pass per digit (none for a single-block ring, whose blocks pass runs every stage)
  const int logR = (int)sh;
  // (LOGR 5 would hold 2 x 32 converted rows + 32 lanes: 256 VGPRs, 1 wave/SIMD; unfused there)
  const bool fuse_cols = logR > 0 && logR <= 4 && a.alpha <= 2 && a.kP <= 2;
  if (fuse_cols) {
    const uint64_t rows = (uint64_t)a.dn * K, per = (N >> logR) / 256;
    NTT_DISPATCH_KS(logR, modup_cols_kernel, grid(rows, (uint32_t)per), dim3(256), 0, s, d2c, K, a, dte.psi_rev,
                    dte.psi_rev_sh, ext);
  } else {
    hipLaunchKernelGGL(modup_kernel, grid((uint64_t)a.dn * K, bpr), dim3(256), 0, s, d2c, K, a, ext);
    uint64_t* e = ext;
    for (uint32_t j = 0; j < a.dn && logR > 0; ++j) {
      const uint32_t Tf = a.T - std::min(a.alpha, a.Ll - j * a.alpha);
      launch_ntt_cols(e, K * Tf, Tf, a.logN, false, dtf[j], s);
      e += KN * Tf;
    }
  }
  SHELFI_HIP(hipGetLastError());
  // last NTT stages + the key inner product (one LDS block per digit; > 64 KiB only for
  // 2^12-element blocks with 3 digits, which a gfx950 workgroup may still declare)
  if (sh > 0 && blkLog == 11 && dte.red_ok) {
    hipLaunchKernelGGL((ks_inner_blocks_ct<11, 3, 3, 3, 2>), grid(K * a.T, nb), dim3(256),
                       sizeof(uint64_t) * lpad_size(11) * a.dn, s, d2e, ext, K, a, dte.tw_fwd_blk, evk, evk_sh, accQ,
                       accP);
  } else {
    if (lds * a.dn > 65536)
      SHELFI_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&ks_inner_blocks_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)(lds * a.dn)));
    hipLaunchKernelGGL(ks_inner_blocks_kernel, grid(K * a.T, nb), dim3(256), lds * a.dn, s, d2e, ext, K, a, blkLog,
                       dte.psi_rev, dte.psi_rev_sh, evk, evk_sh, accQ, accP);
  }
  SHELFI_HIP(hipGetLastError());
  // ModDown: INTT of the P part, P -> Q_l conversion, its NTT fused with the finish
  launch_ntt(accP, K * 2 * a.kP, a.kP, a.logN, true, tower_view(dte, a.Ll, N), s);
  if (fuse_cols) {
    NTT_DISPATCH_KS(logR, moddown_cols_kernel, grid(K * 2, (uint32_t)((N >> logR) / 256)), dim3(256), 0, s, accP, a,
                    dtq.psi_rev, dtq.psi_rev_sh, z);
  } else {
    hipLaunchKernelGGL(moddown_kernel, grid(K * 2, bpr), dim3(256), 0, s, accP, a, z);
    SHELFI_HIP(hipGetLastError());
    launch_ntt_cols(z, K * 2 * a.Ll, a.Ll, a.logN, false, dtq, s);
  }
  SHELFI_HIP(hipGetLastError());
  if (sh > 0 && blkLog == 11 && dtq.red_ok)
    hipLaunchKernelGGL((ks_finish_blocks_ct<11, 3, 3, 3, 2>), grid(K * 2 * a.Ll, nb), dim3(256), 0, s, z, accQ, a,
                       dtq.tw_fwd_blk, out);
  else if (sh > 0 && blkLog == 12 && dtq.red_ok)
    hipLaunchKernelGGL((ks_finish_blocks_ct<12, 3, 3, 3, 3>), grid(K * 2 * a.Ll, nb), dim3(256), 0, s, z, accQ, a,
                       dtq.tw_fwd_blk, out);
  else
    hipLaunchKernelGGL(ks_finish_blocks_kernel, grid(K * 2 * a.Ll, nb), dim3(256), lds, s, z, accQ, a, blkLog,
                       dtq.psi_rev, dtq.psi_rev_sh, out);
  SHELFI_HIP(hipGetLastError());
}

// -------------------------------------------------------------- ModReduce ----
// last [K][2][N] (COEFFICIENT of tower Ll-1) -> v [K][2][Lo][N]: the centred lift mod q_t
__global__ __launch_bounds__(256) void rescale_lift_kernel(const uint64_t* __restrict__ last, uint32_t Lo,
                                                           uint32_t logN, uint64_t ql,
                                                           const TowerConst* __restrict__ tq,
                                                           uint64_t* __restrict__ v) {
  const uint32_t N = 1u << logN, bpr = N >> 8;
  const uint64_t row = blockIdx.x / bpr;  // (k * 2 + poly) * Lo + t
  const uint32_t n = (blockIdx.x % bpr) * 256 + threadIdx.x;
  const uint32_t t = (uint32_t)(row % Lo);
  const TowerConst c = tq[t];
  const uint64_t x = last[(row / Lo) * N + n];
  uint64_t r;
  if (x > (ql >> 1)) {  // x - q_l < 0: q_t - ((q_l - x) mod q_t)
    const uint64_t m = red64(ql - x, c.q, c.one_shoup);
    r = m ? c.q - m : 0;
  } else {
    r = red64(x, c.q, c.one_shoup);
  }
  v[row * N + n] = r;
}

// v's last NTT stages in LDS, then out = (in - v) q_l^-1 mod q_t
__global__ __launch_bounds__(256) void rescale_finish_blocks_kernel(const uint64_t* __restrict__ in,
                                                                    const uint64_t* __restrict__ v, uint32_t Lo,
                                                                    uint32_t logN, uint32_t blkLog,
                                                                    const uint64_t* __restrict__ tw,
                                                                    const uint64_t* __restrict__ twp,
                                                                    const TowerConst* __restrict__ tq,
                                                                    RescaleConst rc, uint64_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint64_t sm[];
  const uint32_t N = 1u << logN, blk = 1u << blkLog, sh = logN - blkLog;
  const uint64_t row = blockIdx.x >> sh;  // (k * 2 + poly) * Lo + t
  const uint32_t b = blockIdx.x & ((1u << sh) - 1);
  const uint64_t kp = row / Lo;
  const uint32_t t = (uint32_t)(row % Lo);
  const uint64_t q = tq[t].q, w = rc.qlinv[t], wp = rc.qlinv_sh[t];
  const uint64_t boff = (uint64_t)b << blkLog;
  const ulonglong2* V = reinterpret_cast<const ulonglong2*>(v + (row << logN) + boff);
  for (uint32_t p = threadIdx.x; p < blk / 2; p += 256) lds_put2(sm, p, V[p]);
  __syncthreads();
  ntt_fwd_block_stages(sm, blkLog, b, logN, tw + (uint64_t)t * N, twp + (uint64_t)t * N, q);
  const ulonglong2* X = reinterpret_cast<const ulonglong2*>(in + ((kp * (Lo + 1) + t) << logN) + boff);
  ulonglong2* O = reinterpret_cast<ulonglong2*>(out + (row << logN) + boff);
  for (uint32_t p = threadIdx.x; p < blk / 2; p += 256) {
    const ulonglong2 y = lds_get2(sm, p), x = X[p];
    O[p] = make_ulonglong2(shoup_mul(submod(x.x, canon8(y.x, q), q), w, wp, q),
                           shoup_mul(submod(x.y, canon8(y.y, q), q), w, wp, q));
  }
}

size_t rescale_scratch_bytes(uint32_t Ll, uint32_t N, uint64_t K) {
  return K * 2ull * N * 8 * (1 + (uint64_t)(Ll - 1)) + 64;  // last | v
}

// The same finish at compile-time shape (see ks_finish_blocks_ct).
template <int BL, int K1, int K2, int K3, int K4>
__global__ __launch_bounds__(256) void rescale_finish_blocks_ct(const uint64_t* __restrict__ in,
                                                                const uint64_t* __restrict__ v, uint32_t Lo,
                                                                uint32_t logN, const ulonglong2* __restrict__ twb,
                                                                const TowerConst* __restrict__ tq, RescaleConst rc,
                                                                uint64_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint64_t sm[lpad_size(BL)];
  const uint32_t sh = logN - BL;
  const uint64_t row = blockIdx.x >> sh;  // (k * 2 + poly) * Lo + t
  const uint32_t b = blockIdx.x & ((1u << sh) - 1);
  const uint64_t kp = row / Lo;
  const uint32_t t = (uint32_t)(row % Lo);
  const TowerConst& c = tq[t];
  const uint64_t q = c.q, w = rc.qlinv[t], wp = rc.qlinv_sh[t];
  const uint64_t boff = (uint64_t)b << BL;
  const ulonglong2* __restrict__ tb = twb + ((uint64_t)t << logN) + boff;
  const uint64_t* __restrict__ X = in + ((kp * (Lo + 1) + t) << logN) + boff;
  uint64_t* __restrict__ O = out + (row << logN) + boff;
  fwd_block_pass_ct<BL, K1, K2, K3, K4>(v + (row << logN) + boff, tb, q, c.n8q, sm, [&](uint32_t j0, auto& y) {
#pragma unroll
    for (int m = 0; m < (1 << K4); m += 2) {
      const ulonglong2 x = *reinterpret_cast<const ulonglong2*>(X + j0 + m);
      *reinterpret_cast<ulonglong2*>(O + j0 + m) =
          make_ulonglong2(shoup_mul(submod(x.x, red_any(y[m], c), q), w, wp, q),
                          shoup_mul(submod(x.y, red_any(y[m + 1], c), q), w, wp, q));
    }
  });
}

void launch_rescale(const DeviceTables& dt, uint32_t Ll, uint32_t logN, const RescaleConst& rc,
                    const uint64_t* in, uint64_t K, uint64_t* out, void* scratch, hipStream_t s) {
  if (!K) return;
  const uint32_t N = 1u << logN, bpr = N >> 8, Lo = Ll - 1;
  uint64_t* last = reinterpret_cast<uint64_t*>(scratch);
  uint64_t* v = last + K * 2 * N;
  // the dropped tower of every (ct, poly): K * 2 rows of N words, pitch Ll * N
  SHELFI_HIP(hipMemcpy2DAsync(last, (size_t)N * 8, in + (uint64_t)Lo * N, (size_t)Ll * N * 8, (size_t)N * 8,
                              K * 2, hipMemcpyDeviceToDevice, s));
  launch_ntt(last, K * 2, 1, logN, true, tower_view(dt, Lo, N), s);
  const uint64_t rows = K * 2 * Lo;
  if (rows * bpr > 0x7FFFFFFFull) throw Error{SHELFI_ERR_ARG, "ModReduce batch too large"};
  hipLaunchKernelGGL(rescale_lift_kernel, dim3((uint32_t)(rows * bpr)), dim3(256), 0, s, last, Lo, logN, rc.ql,
                     dt.tc, v);
  SHELFI_HIP(hipGetLastError());
  launch_ntt_cols(v, rows, Lo, logN, false, dt, s);
  const uint32_t blkLog = ntt_block_log(logN);
  const dim3 nbf((uint32_t)(rows << (logN - blkLog)));
  if (logN > blkLog && blkLog == 11 && dt.red_ok)
    hipLaunchKernelGGL((rescale_finish_blocks_ct<11, 3, 3, 3, 2>), nbf, dim3(256), 0, s, in, v, Lo, logN,
                       dt.tw_fwd_blk, dt.tc, rc, out);
  else if (logN > blkLog && blkLog == 12 && dt.red_ok)
    hipLaunchKernelGGL((rescale_finish_blocks_ct<12, 3, 3, 3, 3>), nbf, dim3(256), 0, s, in, v, Lo, logN,
                       dt.tw_fwd_blk, dt.tc, rc, out);
  else
    hipLaunchKernelGGL(rescale_finish_blocks_kernel, nbf, dim3(256), sizeof(uint64_t) << blkLog, s, in, v, Lo,
                       logN, blkLog, dt.psi_rev, dt.psi_rev_sh, dt.tc, rc, out);
  SHELFI_HIP(hipGetLastError());
}

// --------------------------------------------------------- EvalMultKeyGen ----
// digit j: e_j (nonce (4 << 56) | (j << 16), words [0, N)), a_{j,t} uniform over tower t of
// Q u P (nonce (4 << 56) | (j << 16) | (1 + t), word pair (2i, 2i+1) -> 128 bits mod q_t)
__global__ __launch_bounds__(256) void evk_sample_kernel(uint32_t logN, uint32_t T0,
                                                         const TowerConst* __restrict__ te,
                                                         const uint64_t* __restrict__ cdt, int T, Key8 key,
                                                         uint32_t j, uint64_t* __restrict__ e_out,
                                                         uint64_t* __restrict__ a_out) {
  const uint32_t N = 1u << logN;
  const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
  if (gid >= (N >> 3)) return;
  const uint32_t j0 = gid * 8;
  const uint64_t nonce = (4ull << 56) | ((uint64_t)j << 16);
  uint64_t re[8];
  chacha20_block(key, j0 >> 3, nonce, re);
  int64_t ev[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) ev[u] = gauss_sample(re[u], cdt, T);
  for (uint32_t t = 0; t < T0; ++t) {
    const TowerConst c = te[t];
    uint64_t ra[16];
    chacha20_block(key, j0 >> 2, nonce | (1 + t), ra);
    chacha20_block(key, (j0 >> 2) + 1, nonce | (1 + t), ra + 8);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      e_out[(uint64_t)t * N + j0 + u] = mod_signed_dev(ev[u], c);
      const uint64_t lo = ra[2 * u], hi = ra[2 * u + 1];
      a_out[(uint64_t)t * N + j0 + u] =
          addmod(shoup_mul(red64(hi, c.q, c.one_shoup), c.r64, c.r64_shoup, c.q), red64(lo, c.q, c.one_shoup),
                 c.q);
    }
  }
}

// s over the special primes: the centred coefficients of s (tower 0, COEFFICIENT) mod p_m
__global__ __launch_bounds__(256) void evk_s_ext_kernel(const uint64_t* __restrict__ s0, uint64_t q0,
                                                        uint32_t logN, uint32_t kP,
                                                        const TowerConst* __restrict__ tp,
                                                        uint64_t* __restrict__ sp) {
  const uint32_t N = 1u << logN;
  const uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (uint64_t)kP * N) return;
  const uint32_t m = (uint32_t)(e >> logN);
  const TowerConst c = tp[m];
  const uint64_t x = s0[e & (N - 1)];
  const int64_t v = x > (q0 >> 1) ? -(int64_t)(q0 - x) : (int64_t)x;
  sp[e] = mod_signed_dev(v, c);
}

// b_j = e_j - a_j s + [t in digit j] (P mod q_t) s^2 (EVALUATION); evk[0][j] = b, evk[1][j] = a
__global__ __launch_bounds__(256) void evk_combine_kernel(const uint64_t* __restrict__ e_eval,
                                                          const uint64_t* __restrict__ a_eval,
                                                          const uint64_t* __restrict__ sk,
                                                          const uint64_t* __restrict__ sp,
                                                          const TowerConst* __restrict__ te, EvkGenConst g,
                                                          uint32_t j, uint64_t* __restrict__ evk) {
  const uint32_t N = 1u << g.logN, T0 = g.L + g.kP;
  const uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (uint64_t)T0 * N) return;
  const uint32_t t = (uint32_t)(e >> g.logN);
  const TowerConst c = te[t];
  const uint64_t st = t < g.L ? sk[e] : sp[e - (uint64_t)g.L * N];
  const uint64_t a = a_eval[e];
  uint64_t b = submod(e_eval[e], mulmod_generic(a, st, c), c.q);
  if (t < g.L && t >= j * g.alpha && t < (j + 1) * g.alpha)
    b = addmod(b, mulmod_generic(g.pmod[t], mulmod_generic(st, st, c), c), c.q);
  const uint64_t TN = (uint64_t)T0 * N;
  evk[(uint64_t)j * TN + e] = b;
  evk[((uint64_t)g.dnum + j) * TN + e] = a;
}

size_t evk_scratch_bytes(uint32_t L, uint32_t kP, uint32_t N) {
  return (uint64_t)N * 8 * (2ull * (L + kP) + kP + 1) + 64;  // e | a | s over P | s0
}

void launch_evk_keygen(const EvkGenConst& g, const DeviceTables& dtq, const DeviceTables& dte,
                       const uint64_t* cdt, int cdt_len, const uint32_t key[8], const uint64_t* sk,
                       uint64_t* evk, void* scratch, hipStream_t s) {
  const uint32_t N = 1u << g.logN, T0 = g.L + g.kP;
  uint64_t* eb = reinterpret_cast<uint64_t*>(scratch);
  uint64_t* ab = eb + (uint64_t)T0 * N;
  uint64_t* sp = ab + (uint64_t)T0 * N;
  uint64_t* s0 = sp + (uint64_t)g.kP * N;
  Key8 k8;
  for (int i = 0; i < 8; ++i) k8.k[i] = key[i];
  SHELFI_HIP(hipMemcpyAsync(s0, sk, (size_t)N * 8, hipMemcpyDeviceToDevice, s));
  launch_ntt(s0, 1, 1, g.logN, true, dtq, s);  // tower 0 of s -> COEFFICIENT
  const uint64_t kpn = (uint64_t)g.kP * N;
  hipLaunchKernelGGL(evk_s_ext_kernel, dim3((uint32_t)((kpn + 255) / 256)), dim3(256), 0, s, s0, g.q0, g.logN,
                     g.kP, dte.tc + g.L, sp);
  SHELFI_HIP(hipGetLastError());
  launch_ntt(sp, g.kP, g.kP, g.logN, false, tower_view(dte, g.L, N), s);
  const uint64_t tn = (uint64_t)T0 * N;
  for (uint32_t j = 0; j < g.dnum; ++j) {
    hipLaunchKernelGGL(evk_sample_kernel, dim3((N / 8 + 255) / 256), dim3(256), 0, s, g.logN, T0, dte.tc, cdt,
                       cdt_len, k8, j, eb, ab);
    SHELFI_HIP(hipGetLastError());
    launch_ntt(eb, T0, T0, g.logN, false, dte, s);
    hipLaunchKernelGGL(evk_combine_kernel, dim3((uint32_t)((tn + 255) / 256)), dim3(256), 0, s, eb, ab, sk, sp,
                       dte.tc, g, j, evk);
    SHELFI_HIP(hipGetLastError());
  }
}

}  // namespace shelfi

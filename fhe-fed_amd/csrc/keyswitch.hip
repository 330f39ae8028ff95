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

#include "dev_common.h"
#include "shelfi_internal.h"

namespace shelfi {

typedef unsigned __int128 du128;

// sum of products (< 2^124) -> [0, q)
__device__ __forceinline__ uint64_t red128(du128 acc, const TowerConst& c) {
  const uint64_t hi = (uint64_t)(acc >> 64), lo = (uint64_t)acc;
  return addmod(shoup_mul(hi, c.r64, c.r64_shoup, c.q), red64(lo, c.q, c.one_shoup), c.q);
}
__device__ __forceinline__ du128 mul128(uint64_t a, uint64_t b) { return (du128)a * b; }

// ---------------------------------------------------------------- tensor ----
// d0 = a0 b0 -> out[.][0], d1 = a0 b1 + a1 b0 -> out[.][1], d2 = a1 b1 -> d2[k][t]
__global__ __launch_bounds__(256) void tensor_kernel(const uint64_t* __restrict__ x,
                                                     const uint64_t* __restrict__ y, uint32_t Ll,
                                                     uint32_t logN, const TowerConst* __restrict__ tq,
                                                     uint64_t* __restrict__ out, uint64_t* __restrict__ d2) {
  const uint32_t N = 1u << logN, bpr = N >> 8;
  const uint64_t row = blockIdx.x / bpr;  // k * Ll + t
  const uint32_t n = (blockIdx.x % bpr) * 256 + threadIdx.x;
  const uint64_t k = row / Ll;
  const uint32_t t = (uint32_t)(row % Ll);
  const TowerConst c = tq[t];
  const uint64_t i0 = ((k * 2 + 0) * Ll + t) * N + n, i1 = i0 + (uint64_t)Ll * N;
  const uint64_t a0 = x[i0], a1 = x[i1], b0 = y[i0], b1 = y[i1];
  const uint64_t d0 = mulmod_generic(a0, b0, c);
  const uint64_t d1 = addmod(mulmod_generic(a0, b1, c), mulmod_generic(a1, b0, c), c.q);
  d2[row * N + n] = mulmod_generic(a1, b1, c);
  out[i0] = d0;
  out[i1] = d1;
}

// ----------------------------------------------------------------- ModUp ----
// c [K][Ll][N] (COEFFICIENT) -> ext [dn][K][T][N] (COEFFICIENT): digit j's own towers
// copied, every other tower of Q_l u P by the fast basis conversion.
__global__ __launch_bounds__(256) void modup_kernel(const uint64_t* __restrict__ c, uint64_t K,
                                                    KsArgs a, uint64_t* __restrict__ ext) {
  const uint32_t N = 1u << a.logN, bpr = N >> 8;
  const uint64_t row = blockIdx.x / bpr;  // j * K + k
  const uint32_t n = (blockIdx.x % bpr) * 256 + threadIdx.x;
  const uint32_t j = (uint32_t)(row / K);
  const uint64_t k = row % K;
  const uint32_t s = j * a.alpha, cnt = min(a.alpha, a.Ll - s);
  uint64_t x[kMaxTowers], yv[kMaxTowers];
  for (uint32_t i = 0; i < cnt; ++i) {
    const TowerConst ci = a.tq[s + i];
    x[i] = c[(k * a.Ll + s + i) * N + n];
    yv[i] = shoup_mul(x[i], a.mu_inv[j * a.alpha + i], a.mu_inv_sh[j * a.alpha + i], ci.q);
  }
  uint64_t* __restrict__ o = ext + row * a.T * N + n;
  for (uint32_t t = 0; t < a.T; ++t) {
    uint64_t v;
    if (t >= s && t < s + cnt) {
      v = x[t - s];
    } else {
      du128 acc = 0;
      const uint64_t* __restrict__ h = a.mu_hat + (uint64_t)j * a.alpha * a.T + t;
      for (uint32_t i = 0; i < cnt; ++i) acc += mul128(yv[i], h[(uint64_t)i * a.T]);
      v = red128(acc, a.te[t]);
    }
    o[(uint64_t)t * N] = v;
  }
}

// --------------------------------------------------------- inner product ----
// ext [dn][K][T][N] (EVALUATION) x key [2][dnFull][Lfull + kP][N] -> accQ [K][2][Ll][N],
// accP [K][2][kP][N]
__global__ __launch_bounds__(256) void ks_inner_kernel(const uint64_t* __restrict__ ext, uint64_t K,
                                                       KsArgs a, const uint64_t* __restrict__ evk,
                                                       const uint64_t* __restrict__ evk_sh,
                                                       uint64_t* __restrict__ accQ,
                                                       uint64_t* __restrict__ accP) {
  const uint32_t N = 1u << a.logN, bpr = N >> 8;
  const uint64_t row = blockIdx.x / bpr;  // k * T + t
  const uint32_t n = (blockIdx.x % bpr) * 256 + threadIdx.x;
  const uint64_t k = row / a.T;
  const uint32_t t = (uint32_t)(row % a.T);
  const TowerConst c = a.te[t];
  const uint32_t TF = a.Lfull + a.kP;
  const uint32_t tk = t < a.Ll ? t : a.Lfull + (t - a.Ll);  // the key's tower
  uint64_t u0 = 0, u1 = 0;
  for (uint32_t j = 0; j < a.dn; ++j) {
    const uint64_t xv = ext[((uint64_t)j * K + k) * a.T * N + (uint64_t)t * N + n];
    const uint64_t ib = ((uint64_t)j * TF + tk) * N + n;
    const uint64_t ia = ((uint64_t)(a.dnFull + j) * TF + tk) * N + n;
    u0 = addmod(u0, shoup_mul(xv, evk[ib], evk_sh[ib], c.q), c.q);
    u1 = addmod(u1, shoup_mul(xv, evk[ia], evk_sh[ia], c.q), c.q);
  }
  if (t < a.Ll) {
    accQ[((k * 2 + 0) * a.Ll + t) * N + n] = u0;
    accQ[((k * 2 + 1) * a.Ll + t) * N + n] = u1;
  } else {
    const uint32_t m = t - a.Ll;
    accP[((k * 2 + 0) * a.kP + m) * N + n] = u0;
    accP[((k * 2 + 1) * a.kP + m) * N + n] = u1;
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

// out[k][poly][t] += (accQ - z) P^-1 mod q_t   (all EVALUATION)
__global__ __launch_bounds__(256) void ks_finish_kernel(const uint64_t* __restrict__ accQ,
                                                        const uint64_t* __restrict__ z, KsArgs a,
                                                        uint64_t* __restrict__ out) {
  const uint32_t N = 1u << a.logN, bpr = N >> 8;
  const uint64_t row = blockIdx.x / bpr;  // (k * 2 + poly) * Ll + t
  const uint32_t n = (blockIdx.x % bpr) * 256 + threadIdx.x;
  const uint32_t t = (uint32_t)(row % a.Ll);
  const TowerConst c = a.tq[t];
  const uint64_t e = row * N + n;
  const uint64_t d = submod(accQ[e], z[e], c.q);
  out[e] = addmod(out[e], shoup_mul(d, a.pinv[t], a.pinv_sh[t], c.q), c.q);
}

size_t ks_scratch_bytes(uint32_t Ll, uint32_t kP, uint32_t dn, uint32_t N, uint64_t K) {
  const uint64_t T = Ll + kP;
  // [d2 | ext] (z reuses it: Ll + dn T >= 2 Ll) | accQ | accP
  return K * (uint64_t)N * 8 * (Ll + dn * T + 2ull * Ll + 2ull * kP) + 64;
}

void launch_eval_mult(const KsArgs& a, const DeviceTables& dtq, const DeviceTables& dte,
                      const uint64_t* evk, const uint64_t* evk_sh, const uint64_t* x, const uint64_t* y,
                      uint64_t K, uint64_t* out, void* scratch, hipStream_t s) {
  if (!K) return;
  const uint32_t N = 1u << a.logN, bpr = N >> 8;
  const uint64_t KN = K * N;
  uint64_t* d2 = reinterpret_cast<uint64_t*>(scratch);
  uint64_t* ext = d2 + KN * a.Ll;
  uint64_t* accQ = ext + KN * a.dn * a.T;
  uint64_t* accP = accQ + KN * 2 * a.Ll;
  uint64_t* z = d2;
  auto grid = [&](uint64_t rows) {
    const uint64_t b = rows * bpr;
    if (b > 0x7FFFFFFFull) throw Error{SHELFI_ERR_ARG, "EvalMult batch too large"};
    return dim3((uint32_t)b);
  };
  hipLaunchKernelGGL(tensor_kernel, grid(K * a.Ll), dim3(256), 0, s, x, y, a.Ll, a.logN, a.tq, out, d2);
  SHELFI_HIP(hipGetLastError());
  launch_ntt(d2, K * a.Ll, a.Ll, a.logN, true, dtq, s);  // c2 -> COEFFICIENT
  hipLaunchKernelGGL(modup_kernel, grid((uint64_t)a.dn * K), dim3(256), 0, s, d2, K, a, ext);
  SHELFI_HIP(hipGetLastError());
  launch_ntt(ext, (uint64_t)a.dn * K * a.T, a.T, a.logN, false, dte, s);
  hipLaunchKernelGGL(ks_inner_kernel, grid(K * a.T), dim3(256), 0, s, ext, K, a, evk, evk_sh, accQ, accP);
  SHELFI_HIP(hipGetLastError());
  launch_ntt(accP, K * 2 * a.kP, a.kP, a.logN, true, tower_view(dte, a.Ll, N), s);
  hipLaunchKernelGGL(moddown_kernel, grid(K * 2), dim3(256), 0, s, accP, a, z);
  SHELFI_HIP(hipGetLastError());
  launch_ntt(z, K * 2 * a.Ll, a.Ll, a.logN, false, dtq, s);
  hipLaunchKernelGGL(ks_finish_kernel, grid(K * 2 * a.Ll), dim3(256), 0, s, accQ, z, a, out);
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

__global__ __launch_bounds__(256) void rescale_finish_kernel(const uint64_t* __restrict__ in,
                                                             const uint64_t* __restrict__ v, uint32_t Lo,
                                                             uint32_t logN, const TowerConst* __restrict__ tq,
                                                             RescaleConst rc, uint64_t* __restrict__ out) {
  const uint32_t N = 1u << logN, bpr = N >> 8;
  const uint64_t row = blockIdx.x / bpr;  // (k * 2 + poly) * Lo + t
  const uint32_t n = (blockIdx.x % bpr) * 256 + threadIdx.x;
  const uint64_t kp = row / Lo;
  const uint32_t t = (uint32_t)(row % Lo);
  const TowerConst c = tq[t];
  const uint64_t xin = in[(kp * (Lo + 1) + t) * N + n];
  out[row * N + n] = shoup_mul(submod(xin, v[row * N + n], c.q), rc.qlinv[t], rc.qlinv_sh[t], c.q);
}

size_t rescale_scratch_bytes(uint32_t Ll, uint32_t N, uint64_t K) {
  return K * 2ull * N * 8 * (1 + (uint64_t)(Ll - 1)) + 64;  // last | v
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
  launch_ntt(v, rows, Lo, logN, false, dt, s);
  hipLaunchKernelGGL(rescale_finish_kernel, dim3((uint32_t)(rows * bpr)), dim3(256), 0, s, in, v, Lo, logN,
                     dt.tc, rc, out);
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

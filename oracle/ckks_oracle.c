/*
 * ckks_oracle.c — CPU restatement of the SHELFI_FHE / PALISADE-1.11 CKKS hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker (or the timed
 * CPU baseline).  The product (fhe-fed_amd/, libshelfi.so) never links, loads or
 * calls it.
 *
 * Every routine is written for obviousness, not speed (u128 `%` for every modmul),
 * except or_wavg_fast(), which is the Shoup-constant form used as the CPU baseline
 * and is itself cross-checked against or_wavg() in tests.
 *
 * Citations are to /root/reference (palisade_pybind/SHELFI_FHE/...) and to
 * PALISADE 1.11.7 behaviour, which is NOT vendored in the reference (see
 * SURVEY.md App. A/B); PALISADE-only facts are tagged [PALISADE-1.11].
 *
 * Parity pinning:
 *   - params (primes, minimal 2N-th roots) and NTT ordering are pinned by the
 *     committed PALISADE context/key files (tests/golden/palisade*): the KAT
 *     b + a*s == small e (test_oracle_kat.py) and the context's q/psi values;
 *   - encode/decode floating-point order and decrypt noise flooding are NOT
 *     pinned (PALISADE source absent) -> tolerance-level vs PALISADE;
 *   - aggregation (EvalMult-by-constant + EvalAdd) is exact integer arithmetic,
 *     pinned by construction once W = round((double)(float)w * q_last) is fixed.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;
typedef __int128 i128;

/* ------------------------------------------------------------------------ */
/* integer helpers                                                          */
/* ------------------------------------------------------------------------ */

static inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) {
  return (uint64_t)(((u128)a * b) % q);
}
static inline uint64_t addmod(uint64_t a, uint64_t b, uint64_t q) {
  uint64_t s = a + b;
  return s >= q ? s - q : s;
}
static inline uint64_t submod(uint64_t a, uint64_t b, uint64_t q) {
  return a >= b ? a - b : a + q - b;
}
uint64_t or_powmod(uint64_t a, uint64_t e, uint64_t q) {
  uint64_t r = 1 % q;
  a %= q;
  while (e) {
    if (e & 1) r = mulmod(r, a, q);
    a = mulmod(a, a, q);
    e >>= 1;
  }
  return r;
}
/* signed int64 -> [0,q) (v mod q).  Encode's own mapping, FitToNativeVector, agrees with it
 * for |v| < 2^62 - 256 and wraps beyond (or_fit_wrap below) [PALISADE-1.11]. */
uint64_t or_mod_signed(int64_t v, uint64_t q) {
  if (v >= 0) return (uint64_t)v % q;
  uint64_t m = (uint64_t)(-(v + 1)) + 1; /* |v| without overflow */
  m %= q;
  return m ? q - m : 0;
}
static uint64_t inv_mod(uint64_t a, uint64_t q) { return or_powmod(a, q - 2, q); }

static uint32_t bitrev(uint32_t x, int bits) {
  uint32_t r = 0;
  for (int i = 0; i < bits; ++i) {
    r = (r << 1) | (x & 1);
    x >>= 1;
  }
  return r;
}
static int ilog2(uint64_t n) {
  int l = 0;
  while ((1ull << l) < n) ++l;
  return l;
}

/* deterministic Miller-Rabin for all 64-bit n (bases = first 12 primes) */
int or_is_prime(uint64_t n) {
  static const uint64_t bases[12] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  if (n < 2) return 0;
  for (int i = 0; i < 12; ++i) {
    if (n == bases[i]) return 1;
    if (n % bases[i] == 0) return 0;
  }
  uint64_t d = n - 1;
  int s = 0;
  while ((d & 1) == 0) {
    d >>= 1;
    ++s;
  }
  for (int i = 0; i < 12; ++i) {
    uint64_t x = or_powmod(bases[i], d, n);
    if (x == 1 || x == n - 1) continue;
    int comp = 1;
    for (int r = 1; r < s; ++r) {
      x = mulmod(x, x, n);
      if (x == n - 1) {
        comp = 0;
        break;
      }
    }
    if (comp) return 0;
  }
  return 1;
}

/* ------------------------------------------------------------------------ */
/* parameter generation  (ckks.cpp:26-28 genCryptoContextCKKS(multDepth,...) */
/* -> PALISADE ParamsGen; prime rule recovered in SURVEY App. A)             */
/* ------------------------------------------------------------------------ */

/* PALISADE FirstPrime(nBits, m): smallest prime q > 2^nBits with q == 1 mod m
 * (m a power of two <= 2^nBits, so the search starts at 2^nBits + 1). */
uint64_t or_first_prime(uint32_t bits, uint64_t m) {
  uint64_t q = (1ull << bits) + 1;
  while (!or_is_prime(q)) q += m;
  return q;
}
uint64_t or_prev_prime(uint64_t q, uint64_t m) {
  do { q -= m; } while (!or_is_prime(q));
  return q;
}
uint64_t or_next_prime(uint64_t q, uint64_t m) {
  do { q += m; } while (!or_is_prime(q));
  return q;
}

/* PALISADE RootOfUnity(m, q): the MINIMUM primitive m-th root of unity
 * (it cycles a found root over all powers co-prime to m and keeps the
 * smallest) [PALISADE-1.11; verified against cryptocontext.txt@1935,@1984]. */
uint64_t or_min_root(uint64_t m, uint64_t q) {
  uint64_t r = 0;
  for (uint64_t g = 2;; ++g) {
    r = or_powmod(g, (q - 1) / m, q);
    if (or_powmod(r, m / 2, q) == q - 1) break; /* order exactly m (m = 2^k) */
  }
  uint64_t r2 = mulmod(r, r, q), x = r, best = r;
  for (uint64_t k = 1; k < m / 2; ++k) { /* x = r^(2k+1): all odd powers */
    x = mulmod(x, r2, q);
    if (x < best) best = x;
  }
  return best;
}

/* EXACTRESCALE chain: q[L-1] = FirstPrime(scaleBits, 2N); then alternately
 * PreviousPrime / NextPrime walking outwards; q[0] = PreviousPrime(
 * FirstPrime(firstModBits, 2N)).  Reproduces the committed 2-tower chain
 * (cryptocontext.txt@1927,@1976) and TCT1's 3-tower chain [SURVEY App. A]. */
int or_params_generate(uint32_t N, uint32_t L, uint32_t scale_bits, uint32_t first_mod_bits,
                       uint64_t* q, uint64_t* psi) {
  if (L < 1 || L > 16 || N < 8 || (N & (N - 1))) return -1;
  uint64_t m = 2ull * N;
  q[L - 1] = or_first_prime(scale_bits, m);
  uint64_t qprev = q[L - 1], qnext = q[L - 1];
  unsigned cnt = 0;
  for (int i = (int)L - 2; i >= 1; --i) {
    if ((cnt % 2) == 0) {
      qprev = or_prev_prime(qprev, m);
      q[i] = qprev;
    } else {
      qnext = or_next_prime(qnext, m);
      q[i] = qnext;
    }
    ++cnt;
  }
  if (L > 1) {
    if (first_mod_bits == scale_bits)
      q[0] = or_prev_prime(qprev, m);
    else
      q[0] = or_prev_prime(or_first_prime(first_mod_bits, m), m);
  }
  for (uint32_t i = 0; i < L; ++i) psi[i] = or_min_root(m, q[i]);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* negacyclic NTT, PALISADE convention (ChineseRemainderTransformFTT)        */
/* forward: out[i] = a(psi^(2*bitrev(i)+1)) (bit-reversed evaluation order), */
/* inverse: natural-order coefficients.  Pinned by the key KAT.              */
/* ------------------------------------------------------------------------ */

void or_ntt_fwd(uint64_t* a, uint32_t N, uint64_t q, uint64_t psi) {
  int logN = ilog2(N);
  uint64_t* tw = (uint64_t*)malloc(sizeof(uint64_t) * N);
  uint64_t p = 1;
  for (uint32_t i = 0; i < N; ++i) {
    tw[bitrev(i, logN)] = p;
    p = mulmod(p, psi, q);
  }
  uint32_t t = N;
  for (uint32_t m = 1; m < N; m <<= 1) {
    t >>= 1;
    for (uint32_t i = 0; i < m; ++i) {
      uint64_t S = tw[m + i];
      uint32_t j1 = 2 * i * t;
      for (uint32_t j = j1; j < j1 + t; ++j) {
        uint64_t U = a[j], V = mulmod(a[j + t], S, q);
        a[j] = addmod(U, V, q);
        a[j + t] = submod(U, V, q);
      }
    }
  }
  free(tw);
}

void or_ntt_inv(uint64_t* a, uint32_t N, uint64_t q, uint64_t psi) {
  int logN = ilog2(N);
  uint64_t psi_inv = inv_mod(psi, q);
  uint64_t* tw = (uint64_t*)malloc(sizeof(uint64_t) * N);
  uint64_t p = 1;
  for (uint32_t i = 0; i < N; ++i) {
    tw[bitrev(i, logN)] = p;
    p = mulmod(p, psi_inv, q);
  }
  uint32_t t = 1;
  for (uint32_t m = N; m > 1; m >>= 1) {
    uint32_t h = m >> 1, j1 = 0;
    for (uint32_t i = 0; i < h; ++i) {
      uint64_t S = tw[h + i];
      for (uint32_t j = j1; j < j1 + t; ++j) {
        uint64_t U = a[j], V = a[j + t];
        a[j] = addmod(U, V, q);
        a[j + t] = mulmod(submod(U, V, q), S, q);
      }
      j1 += 2 * t;
    }
    t <<= 1;
  }
  uint64_t ninv = inv_mod(N % q, q);
  for (uint32_t j = 0; j < N; ++j) a[j] = mulmod(a[j], ninv, q);
  free(tw);
}

/* ------------------------------------------------------------------------ */
/* CKKS special FFT (PALISADE DiscreteFourierTransform::FFTSpecial[Inv],     */
/* HEAAN layout).  M = 4*slots; ksi[j] = (cos 2pi j/M, sin 2pi j/M);          */
/* rotGroup[j] = 5^j mod M.  Complex products are (ac-bd, ad+bc) with no FMA */
/* contraction (built with -ffp-contract=off) — the product kernels follow   */
/* the identical operation order, which is what makes encode/decode bit-exact */
/* GPU-vs-oracle.  Oracle-vs-PALISADE float order: unpinned (tolerance).     */
/* ------------------------------------------------------------------------ */

/* Flat twiddle tables, index lenh + j (lenh = 1..slots/2, j < lenh):
 *   inv: ksi[(lenq - rot[j] % lenq) * (M/lenq)],  fwd: ksi[(rot[j] % lenq) * (M/lenq)]
 * with lenq = 4*len = 8*lenh.  Exported so the product library's tables can be
 * compared value-for-value in tests. */
void or_fft_twiddles(uint32_t slots, double* inv_re, double* inv_im, double* fwd_re,
                     double* fwd_im) {
  uint64_t M = 4ull * slots;
  uint64_t* rot = (uint64_t*)malloc(sizeof(uint64_t) * (slots > 0 ? slots : 1));
  uint64_t f = 1;
  for (uint32_t j = 0; j < slots; ++j) {
    rot[j] = f;
    f = (f * 5) % M;
  }
  inv_re[0] = inv_im[0] = fwd_re[0] = fwd_im[0] = 0.0;
  for (uint32_t lenh = 1; lenh < slots; lenh <<= 1) {
    uint64_t lenq = 8ull * lenh;
    uint64_t gap = M / lenq;
    for (uint32_t j = 0; j < lenh; ++j) {
      uint64_t ii = ((lenq - (rot[j] % lenq)) * gap) % M; /* ksi[M] == ksi[0] */
      uint64_t fi = ((rot[j] % lenq) * gap) % M;
      double ai = 2.0 * M_PI * (double)ii / (double)M;
      double af = 2.0 * M_PI * (double)fi / (double)M;
      inv_re[lenh + j] = cos(ai);
      inv_im[lenh + j] = sin(ai);
      fwd_re[lenh + j] = cos(af);
      fwd_im[lenh + j] = sin(af);
    }
  }
  free(rot);
}

static void bitrev_perm(double* re, double* im, uint32_t n) {
  int lg = ilog2(n);
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t r = bitrev(i, lg);
    if (r > i) {
      double t = re[i]; re[i] = re[r]; re[r] = t;
      t = im[i]; im[i] = im[r]; im[r] = t;
    }
  }
}

/* FFTSpecialInv: DIF stages len = n..2, BitReverse, then /n. */
void or_fft_special_inv(double* re, double* im, uint32_t n) {
  double *tr = malloc(sizeof(double) * n), *ti = malloc(sizeof(double) * n);
  double *fr = malloc(sizeof(double) * n), *fi = malloc(sizeof(double) * n);
  or_fft_twiddles(n, tr, ti, fr, fi);
  for (uint32_t len = n; len >= 2; len >>= 1) {
    uint32_t lenh = len >> 1;
    for (uint32_t i = 0; i < n; i += len) {
      for (uint32_t j = 0; j < lenh; ++j) {
        double ar = re[i + j], ai = im[i + j];
        double br = re[i + j + lenh], bi = im[i + j + lenh];
        double ur = ar + br, ui = ai + bi;
        double vr = ar - br, vi = ai - bi;
        double wr = tr[lenh + j], wi = ti[lenh + j];
        double xr = vr * wr - vi * wi;
        double xi = vr * wi + vi * wr;
        re[i + j] = ur; im[i + j] = ui;
        re[i + j + lenh] = xr; im[i + j + lenh] = xi;
      }
    }
  }
  bitrev_perm(re, im, n);
  double dn = (double)n;
  for (uint32_t i = 0; i < n; ++i) {
    re[i] /= dn;
    im[i] /= dn;
  }
  free(tr); free(ti); free(fr); free(fi);
}

/* FFTSpecial: BitReverse, then DIT stages len = 2..n. */
void or_fft_special(double* re, double* im, uint32_t n) {
  double *tr = malloc(sizeof(double) * n), *ti = malloc(sizeof(double) * n);
  double *fr = malloc(sizeof(double) * n), *fi = malloc(sizeof(double) * n);
  or_fft_twiddles(n, tr, ti, fr, fi);
  bitrev_perm(re, im, n);
  for (uint32_t len = 2; len <= n; len <<= 1) {
    uint32_t lenh = len >> 1;
    for (uint32_t i = 0; i < n; i += len) {
      for (uint32_t j = 0; j < lenh; ++j) {
        double ur = re[i + j], ui = im[i + j];
        double br = re[i + j + lenh], bi = im[i + j + lenh];
        double wr = fr[lenh + j], wi = fi[lenh + j];
        double vr = br * wr - bi * wi;
        double vi = br * wi + bi * wr;
        re[i + j] = ur + vr; im[i + j] = ui + vi;
        re[i + j + lenh] = ur - vr; im[i + j + lenh] = ui - vi;
      }
    }
  }
  free(tr); free(ti); free(fr); free(fi);
}

/* llround (ties away from zero) written so it is reproducible bit-for-bit by
 * the GPU kernels: t = trunc(x); |x - t| >= 0.5 -> step away from zero. */
int64_t or_round_half_away(double x) {
  double t = trunc(x);
  double d = x - t;
  if (d >= 0.5) t += 1.0;
  else if (d <= -0.5) t -= 1.0;
  return (int64_t)t;
}

/* ------------------------------------------------------------------------ */
/* encode  (ckks.cpp:80 MakeCKKSPackedPlaintext -> CKKSPackedEncoding::Encode)*/
/* ------------------------------------------------------------------------ */

/* The large-value path of CKKSPackedEncoding::Encode [PALISADE-1.11, restated; no reference
 * fixture exercises it, so parity with PALISADE is unpinned]:
 *   v_i = FFTSpecialInv(x)_i * Delta (real and imaginary parts);
 *   logc = max over nonzero v_i of ceil(log2|v_i|) (glibc log2), at least 0;
 *   logApprox = max(0, logc - MAX_BITS_IN_WORD), MAX_BITS_IN_WORD = 62;
 *   r_i = llround(v_i / 2^logApprox)   (|r_i| <= 2^62);
 *   FitToNativeVector: temp = r < 0 ? B + r : r with B = Max64BitValue() = 2^63 - 513, then
 *     temp > B >> 1 ? (temp - (B - q)) mod q : temp mod q
 *   (== r mod q for |r| <= 2^62 - 257, r - B or r + B beyond: or_fit_wrap);
 *   the residues are then multiplied by 2^logApprox mod q_t (CRTMult steps of <= 2^60 compose
 *   to exactly that) before the NTT.
 * For |v| <= 2^61 (logc <= 61) this is the plain llround encode. */
#define OR_MAX_BITS_IN_WORD 62
#define OR_MAX64_VALUE 9223372036854775295LL /* 2^63 - 513 */

int64_t or_fit_wrap(int64_t r) {
  const int64_t hf = OR_MAX64_VALUE >> 1; /* 2^62 - 257 */
  if (r > hf) return r - OR_MAX64_VALUE;
  if (r < 0 && OR_MAX64_VALUE + r <= hf) return r + OR_MAX64_VALUE;
  return r;
}

/* ceil(log2 |v|) as Encode computes it (glibc log2, then ceil). */
int or_encode_logc(double v) { return (int)ceil(log2(fabs(v))); }

/* x[0..n) (n <= slots) -> coefficient vector coeff[N] of FitToNativeVector-equivalent signed
 * values (COEFFICIENT domain, before the per-tower reduction) and the scale-down exponent
 * *log_approx (the residues are coeff * 2^log_approx mod q_t).  Returns -1 on bad sizes, -3 on a
 * non-finite scaled value. */
int or_encode_coeffs_ex(const double* x, size_t n, uint32_t N, uint32_t slots, double delta,
                        int64_t* coeff, int* log_approx) {
  if (n > slots || 2ull * slots > N) return -1;
  double* re = calloc(slots, sizeof(double));
  double* im = calloc(slots, sizeof(double));
  for (size_t i = 0; i < n; ++i) re[i] = x[i];
  or_fft_special_inv(re, im, slots);
  uint32_t gap = N / (2 * slots);
  memset(coeff, 0, sizeof(int64_t) * N);
  int logc = 0;
  for (uint32_t i = 0; i < slots; ++i) {
    re[i] *= delta;
    im[i] *= delta;
    if (!isfinite(re[i]) || !isfinite(im[i])) {
      free(re);
      free(im);
      return -3;
    }
    if (re[i] != 0 && or_encode_logc(re[i]) > logc) logc = or_encode_logc(re[i]);
    if (im[i] != 0 && or_encode_logc(im[i]) > logc) logc = or_encode_logc(im[i]);
  }
  const int a = logc > OR_MAX_BITS_IN_WORD ? logc - OR_MAX_BITS_IN_WORD : 0;
  const double approx = ldexp(1.0, a);
  for (uint32_t i = 0; i < slots; ++i) {
    coeff[i * gap] = or_fit_wrap(or_round_half_away(re[i] / approx));
    coeff[N / 2 + i * gap] = or_fit_wrap(or_round_half_away(im[i] / approx));
  }
  free(re);
  free(im);
  *log_approx = a;
  return 0;
}

/* The plain signed coefficients; -2 when the vector takes the scale-down path (its
 * coefficients are coeff * 2^logApprox, not int64 values). */
int or_encode_coeffs(const double* x, size_t n, uint32_t N, uint32_t slots, double delta,
                     int64_t* coeff) {
  int a = 0;
  int rc = or_encode_coeffs_ex(x, n, N, slots, delta, coeff, &a);
  return rc ? rc : (a ? -2 : 0);
}

/* full encode: coeffs -> per-tower residues (x 2^logApprox) -> NTT (EVALUATION). out[L][N]. */
int or_encode(const double* x, size_t n, uint32_t N, uint32_t slots, double delta, uint32_t L,
              const uint64_t* q, const uint64_t* psi, uint64_t* out) {
  int64_t* c = malloc(sizeof(int64_t) * N);
  int a = 0;
  int rc = or_encode_coeffs_ex(x, n, N, slots, delta, c, &a);
  if (rc) {
    free(c);
    return rc;
  }
  for (uint32_t t = 0; t < L; ++t) {
    const uint64_t pw = or_powmod(2, (uint64_t)a, q[t]);
    for (uint32_t j = 0; j < N; ++j) out[(size_t)t * N + j] = mulmod(or_mod_signed(c[j], q[t]), pw, q[t]);
    or_ntt_fwd(out + (size_t)t * N, N, q[t], psi[t]);
  }
  free(c);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* encrypt with injected randomness (ckks.cpp:81 cc->Encrypt(pk, pt))        */
/* v ternary, e0/e1 Gaussian, all COEFFICIENT-domain signed, same integers in */
/* every tower; c0 = NTT(v)*b + NTT(e0) + m, c1 = NTT(v)*a + NTT(e1)         */
/* [PALISADE-1.11 LPAlgorithmCKKS::Encrypt].  pk[2][L][N], m[L][N] EVAL.      */
/* ------------------------------------------------------------------------ */
void or_encrypt(const uint64_t* pk, const uint64_t* m, const int64_t* v, const int64_t* e0,
                const int64_t* e1, uint32_t N, uint32_t L, const uint64_t* q,
                const uint64_t* psi, uint64_t* ct /* [2][L][N] */) {
  uint64_t* V = malloc(sizeof(uint64_t) * N);
  uint64_t* E0 = malloc(sizeof(uint64_t) * N);
  uint64_t* E1 = malloc(sizeof(uint64_t) * N);
  for (uint32_t t = 0; t < L; ++t) {
    for (uint32_t j = 0; j < N; ++j) {
      V[j] = or_mod_signed(v[j], q[t]);
      E0[j] = or_mod_signed(e0[j], q[t]);
      E1[j] = or_mod_signed(e1[j], q[t]);
    }
    or_ntt_fwd(V, N, q[t], psi[t]);
    or_ntt_fwd(E0, N, q[t], psi[t]);
    or_ntt_fwd(E1, N, q[t], psi[t]);
    const uint64_t* b = pk + (size_t)t * N;
    const uint64_t* a = pk + ((size_t)L + t) * N;
    const uint64_t* mt = m + (size_t)t * N;
    uint64_t* c0 = ct + (size_t)t * N;
    uint64_t* c1 = ct + ((size_t)L + t) * N;
    for (uint32_t j = 0; j < N; ++j) {
      c0[j] = addmod(addmod(mulmod(V[j], b[j], q[t]), E0[j], q[t]), mt[j], q[t]);
      c1[j] = addmod(mulmod(V[j], a[j], q[t]), E1[j], q[t]);
    }
  }
  free(V);
  free(E0);
  free(E1);
}

/* keygen with injected randomness [PALISADE-1.11 LPAlgorithmCKKS::KeyGen]:
 * s ternary, e Gaussian (coefficient domain, shared across towers), a uniform
 * per tower (sampled directly in EVAL); b = NTT(e) - a*NTT(s).
 * outputs: sk[L][N] = NTT(s), pk[2][L][N] = (b, a). a_eval given [L][N]. */
void or_keygen(const int64_t* s, const int64_t* e, const uint64_t* a_eval, uint32_t N, uint32_t L,
               const uint64_t* q, const uint64_t* psi, uint64_t* sk, uint64_t* pk) {
  uint64_t* E = malloc(sizeof(uint64_t) * N);
  for (uint32_t t = 0; t < L; ++t) {
    uint64_t* S = sk + (size_t)t * N;
    for (uint32_t j = 0; j < N; ++j) {
      S[j] = or_mod_signed(s[j], q[t]);
      E[j] = or_mod_signed(e[j], q[t]);
    }
    or_ntt_fwd(S, N, q[t], psi[t]);
    or_ntt_fwd(E, N, q[t], psi[t]);
    const uint64_t* a = a_eval + (size_t)t * N;
    for (uint32_t j = 0; j < N; ++j) {
      pk[(size_t)t * N + j] = submod(E[j], mulmod(a[j], S[j], q[t]), q[t]);
      pk[((size_t)L + t) * N + j] = a[j];
    }
  }
  free(E);
}

/* ------------------------------------------------------------------------ */
/* weighted average  (ckks.cpp:264-320 computeWeightedAverage)               */
/* per learner i: float sc = w_i (:287); EvalMult(ct, sc) (:288) scales every */
/* residue by W_t = W mod q_t with W = (int64)((double)sc * Delta0 + 0.5)     */
/* [PALISADE-1.11 EvalMult(ct,double)]; EvalAdd (:295-296) adds mod q_t.      */
/* ------------------------------------------------------------------------ */

int64_t or_weight_to_int(float w, double delta0) {
  return (int64_t)((double)w * delta0 + 0.5);
}

/* cts[c] -> [K][2][L][N]; out [K][2][L][N].  Reference form (u128 %). */
void or_wavg(const uint64_t* const* cts, const float* w, size_t C, size_t K, uint32_t N,
             uint32_t L, const uint64_t* q, double delta0, uint64_t* out) {
  uint64_t* W = malloc(sizeof(uint64_t) * C * L);
  for (size_t c = 0; c < C; ++c) {
    int64_t Wi = or_weight_to_int(w[c], delta0);
    for (uint32_t t = 0; t < L; ++t) W[c * L + t] = or_mod_signed(Wi, q[t]);
  }
  size_t per_ct = 2ull * L * N;
  for (size_t k = 0; k < K; ++k)
    for (uint32_t p = 0; p < 2; ++p)
      for (uint32_t t = 0; t < L; ++t) {
        size_t base = k * per_ct + ((size_t)p * L + t) * N;
        for (uint32_t j = 0; j < N; ++j) {
          uint64_t acc = 0;
          for (size_t c = 0; c < C; ++c)
            acc = addmod(acc, mulmod(cts[c][base + j], W[c * L + t], q[t]), q[t]);
          out[base + j] = acc;
        }
      }
  free(W);
}

/* CPU-baseline form: Shoup constant multiplication (what PALISADE's
 * NativeVector::ModMul-by-constant does per tower), optional OpenMP over the
 * (ct, poly, tower) rows.  nthreads <= 0 -> single thread. */
void or_wavg_fast(const uint64_t* const* cts, const float* w, size_t C, size_t K, uint32_t N,
                  uint32_t L, const uint64_t* q, double delta0, uint64_t* out, int nthreads) {
  uint64_t* W = malloc(sizeof(uint64_t) * C * L);
  uint64_t* Wp = malloc(sizeof(uint64_t) * C * L);
  for (size_t c = 0; c < C; ++c) {
    int64_t Wi = or_weight_to_int(w[c], delta0);
    for (uint32_t t = 0; t < L; ++t) {
      W[c * L + t] = or_mod_signed(Wi, q[t]);
      Wp[c * L + t] = (uint64_t)(((u128)W[c * L + t] << 64) / q[t]);
    }
  }
  long rows = (long)(K * 2 * L);
#ifdef _OPENMP
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel for num_threads(nthreads) schedule(static)
#endif
  for (long r = 0; r < rows; ++r) {
    uint32_t t = (uint32_t)(r % L);
    uint64_t qt = q[t];
    size_t base = (size_t)r * N;
    uint64_t* o = out + base;
    for (uint32_t j = 0; j < N; ++j) o[j] = 0;
    for (size_t c = 0; c < C; ++c) {
      const uint64_t* x = cts[c] + base;
      uint64_t w0 = W[c * L + t], wp = Wp[c * L + t];
      for (uint32_t j = 0; j < N; ++j) {
        uint64_t hi = (uint64_t)(((u128)x[j] * wp) >> 64);
        uint64_t rr = x[j] * w0 - hi * qt;
        if (rr >= qt) rr -= qt;
        uint64_t s = o[j] + rr;
        o[j] = s >= qt ? s - qt : s;
      }
    }
  }
  free(W);
  free(Wp);
}

/* ------------------------------------------------------------------------ */
/* decrypt + decode  (ckks.cpp:170-213 -> cc->Decrypt(sk, ct, &pt) :189,    */
/* SetLength :198, GetRealPackedValue :199).                                 */
/* b = c0 + c1*s (EVAL) -> INTT -> exact CRT to the centered integer mod Q   */
/* -> (double)X * (1/scale) -> FFTSpecial -> real parts.  PALISADE's Decode   */
/* additionally symmetrises and adds Gaussian flooding noise [PALISADE-1.11]; */
/* the restatement returns the noise-free value (Re of the slot), which is    */
/* what the symmetrisation computes before the noise.                         */
/* ------------------------------------------------------------------------ */

/* multiword helpers for the exact CRT (little-endian u64 limbs; n of the MW words used) */
#define MW 17 /* 16 towers below 2^60 times L, plus the sign */
static void mw_mul_small(const uint64_t* a, uint64_t b, uint64_t* r, int n) {
  u128 carry = 0;
  for (int i = 0; i < n; ++i) {
    u128 p = (u128)a[i] * b + carry;
    r[i] = (uint64_t)p;
    carry = p >> 64;
  }
}
static void mw_add(uint64_t* a, const uint64_t* b, int n) {
  u128 carry = 0;
  for (int i = 0; i < n; ++i) {
    u128 s = (u128)a[i] + b[i] + carry;
    a[i] = (uint64_t)s;
    carry = s >> 64;
  }
}
static int mw_cmp(const uint64_t* a, const uint64_t* b, int n) {
  for (int i = n - 1; i >= 0; --i) {
    if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  }
  return 0;
}
static void mw_sub(uint64_t* a, const uint64_t* b, int n) {
  uint64_t borrow = 0;
  for (int i = 0; i < n; ++i) {
    u128 d = (u128)a[i] - b[i] - borrow;
    a[i] = (uint64_t)d;
    borrow = (uint64_t)((d >> 64) & 1);
  }
}

/* i128 -> double, the conversion the product kernels use: sign-magnitude, then
 * (double)mag_hi * 2^64 + (double)mag_lo (exact for |X| < 2^64). */
double or_i128_to_double(int64_t hi, uint64_t lo) {
  int neg = hi < 0;
  uint64_t mh = (uint64_t)hi, ml = lo;
  if (neg) { /* two's-complement negate of (hi, lo) */
    ml = ~ml + 1;
    mh = ~mh + (ml == 0 ? 1 : 0);
  }
  double d = (double)mh * 18446744073709551616.0 + (double)ml;
  return neg ? -d : d;
}

/* |X| (MW little-endian u64 words) with its sign -> double: Horner from the top word,
 * d = d * 2^64 + (double)w_i (round 6).  Leading zero words leave d unchanged, so for
 * |X| < 2^128 this is or_i128_to_double's (double)hi * 2^64 + (double)lo.  PALISADE's
 * BigInteger::ConvertToDouble rounding is not pinned (no reference fixture decodes |X| >= 2^64). */
double or_mw_to_double(const uint64_t* mag, int neg) {
  double d = (double)mag[MW - 1];
  for (int i = MW - 2; i >= 0; --i) d = d * 18446744073709551616.0 + (double)mag[i];
  return neg ? -d : d;
}

/* Q, (Q - 1) / 2, Q/q_t and (Q/q_t)^-1 mod q_t of a tower set, computed once per call */
typedef struct {
  uint32_t L;
  int n; /* words in use: L Q < 2^(64 n) */
  const uint64_t* q;
  uint64_t Q[MW], half[MW], qhat[16][MW], qhat_inv[16];
} crt_plan;

static void crt_plan_init(crt_plan* P, uint32_t L, const uint64_t* q) {
  uint64_t tmp[MW];
  memset(P, 0, sizeof(*P));
  P->L = L;
  P->q = q;
  P->n = MW;
  P->Q[0] = 1;
  for (uint32_t t = 0; t < L; ++t) {
    mw_mul_small(P->Q, q[t], tmp, MW);
    memcpy(P->Q, tmp, sizeof(tmp));
  }
  for (int i = 0; i < MW; ++i) P->half[i] = (P->Q[i] >> 1) | (i + 1 < MW ? P->Q[i + 1] << 63 : 0);
  int top = MW - 1;
  while (top > 0 && !P->Q[top]) --top;
  P->n = top + 2 < MW ? top + 2 : MW; /* room for L Q */
  for (uint32_t t = 0; t < L; ++t) {
    P->qhat[t][0] = 1;
    uint64_t qhat_mod = 1;
    for (uint32_t u = 0; u < L; ++u)
      if (u != t) {
        mw_mul_small(P->qhat[t], q[u], tmp, MW);
        memcpy(P->qhat[t], tmp, sizeof(tmp));
        qhat_mod = mulmod(qhat_mod, q[u] % q[t], q[t]);
      }
    P->qhat_inv[t] = inv_mod(qhat_mod, q[t]);
  }
}

/* exact centered CRT of residues r[t] (t < L): X in [-(Q-1)/2, (Q-1)/2] for Q = prod q_t
 * (PALISADE's CRTInterpolate + centring mod Q before Decode, ckks.cpp:189)
 * as magnitude words mag[MW] and a sign. */
static void crt_plan_centered(const crt_plan* P, const uint64_t* r, uint64_t* mag, int* neg_out) {
  uint64_t X[MW] = {0}, tmp[MW];
  const int n = P->n;
  for (uint32_t t = 0; t < P->L; ++t) {
    uint64_t y = mulmod(r[t], P->qhat_inv[t], P->q[t]);
    mw_mul_small(P->qhat[t], y, tmp, n);
    mw_add(X, tmp, n);
  }
  while (mw_cmp(X, P->Q, n) >= 0) mw_sub(X, P->Q, n);
  /* center: X > Q/2 -> X - Q (negative) */
  int neg = mw_cmp(X, P->half, n) > 0;
  if (neg) { /* |X| = Q - X */
    uint64_t A[MW];
    memcpy(A, P->Q, sizeof(A));
    mw_sub(A, X, n);
    memcpy(X, A, sizeof(A));
  }
  memcpy(mag, X, sizeof(X));
  *neg_out = neg;
}

/* the centred value as a two's-complement i128 (hi, lo); returns 0, or -3 if |X| >= 2^127 */
int or_crt_centered(const uint64_t* r, uint32_t L, const uint64_t* q, int64_t* hi,
                    uint64_t* lo) {
  crt_plan P;
  uint64_t X[MW];
  int neg;
  crt_plan_init(&P, L, q);
  crt_plan_centered(&P, r, X, &neg);
  for (int i = 2; i < MW; ++i)
    if (X[i]) return -3;
  if (X[1] >> 63) return -3;
  u128 mag = ((u128)X[1] << 64) | X[0];
  i128 v = neg ? -(i128)mag : (i128)mag;
  *hi = (int64_t)(v >> 64);
  *lo = (uint64_t)v;
  return 0;
}

/* the centred value as a double (or_mw_to_double), any |X| <= (Q - 1) / 2 */
double or_crt_centered_double(const uint64_t* r, uint32_t L, const uint64_t* q) {
  crt_plan P;
  uint64_t X[MW];
  int neg;
  crt_plan_init(&P, L, q);
  crt_plan_centered(&P, r, X, &neg);
  return or_mw_to_double(X, neg);
}

/* decrypt one ciphertext ct[2][L][N] with sk[L][N] (EVAL).  Writes the first
 * `n` real slot values to out.  Returns 0 / negative on error. */
/* b = c0 + c1*s -> INTT -> centered CRT -> / scale, as coefficient pairs
 * (re_i, im_i) = (c[i*gap], c[N/2 + i*gap]) / scale (PALISADE Decode's curValues
 * before the 2^p normalisation). */
int or_decrypt_coeffs(const uint64_t* ct, const uint64_t* sk, uint32_t N, uint32_t L,
                      const uint64_t* q, const uint64_t* psi, uint32_t slots, double scale,
                      double* re, double* im) {
  uint64_t* b = malloc(sizeof(uint64_t) * L * N);
  for (uint32_t t = 0; t < L; ++t) {
    const uint64_t* c0 = ct + (size_t)t * N;
    const uint64_t* c1 = ct + ((size_t)L + t) * N;
    const uint64_t* s = sk + (size_t)t * N;
    uint64_t* bt = b + (size_t)t * N;
    for (uint32_t j = 0; j < N; ++j) bt[j] = addmod(c0[j], mulmod(c1[j], s[j], q[t]), q[t]);
    or_ntt_inv(bt, N, q[t], psi[t]);
  }
  double inv_scale = 1.0 / scale;
  uint32_t gap = N / (2 * slots);
  uint64_t r[16], X[MW];
  crt_plan P;
  crt_plan_init(&P, L, q);
  for (uint32_t i = 0; i < slots; ++i) {
    for (int part = 0; part < 2; ++part) {
      uint32_t j = (part ? N / 2 : 0) + i * gap;
      int neg;
      for (uint32_t t = 0; t < L; ++t) r[t] = b[(size_t)t * N + j];
      crt_plan_centered(&P, r, X, &neg);
      double v = or_mw_to_double(X, neg) * inv_scale;
      if (part) im[i] = v; else re[i] = v;
    }
  }
  free(b);
  return 0;
}

int or_decrypt(const uint64_t* ct, const uint64_t* sk, uint32_t N, uint32_t L,
               const uint64_t* q, const uint64_t* psi, uint32_t slots, double scale,
               size_t n, double* out) {
  if (n > slots) return -1;
  double* re = malloc(sizeof(double) * slots);
  double* im = malloc(sizeof(double) * slots);
  int rc = or_decrypt_coeffs(ct, sk, N, L, q, psi, slots, scale, re, im);
  if (!rc) {
    or_fft_special(re, im, slots);
    for (size_t i = 0; i < n; ++i) out[i] = re[i];
  }
  free(re);
  free(im);
  return rc;
}

/* ckks.cpp:61-104 encrypt() and ckks.cpp:170-213 decrypt() over a whole vector, with the
 * reference's schedule: "#pragma omp parallel for" over ciphertexts (ckks.cpp:70, :186), here with
 * nthreads threads (the CPU baseline's all-core figure, bench.py).  Ciphertext k of encrypt holds
 * x[k*slots .. min(n, (k+1)*slots)) with the seeded sampler's stream g0 + k (encrypt_vector in
 * oracle.py); decrypt's ciphertext k contributes min(slots, n - k*slots) values (:192-196).
 * Returns 0, or the first failing ciphertext's code. */
void or_sample_encrypt(uint64_t seed, uint64_t g, uint32_t N, double sigma, int64_t* v, int64_t* e0,
                       int64_t* e1);
int or_encrypt_vector(const double* x, size_t n, const uint64_t* pk, uint32_t N, uint32_t L,
                      const uint64_t* q, const uint64_t* psi, uint32_t slots, double delta, double sigma,
                      uint64_t seed, uint64_t g0, uint64_t* out, int nthreads) {
  const size_t K = n ? (n + slots - 1) / slots : 1;
  int rc = 0;
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1)
  for (size_t k = 0; k < K; ++k) {
    uint64_t* m = malloc(sizeof(uint64_t) * (size_t)L * N);
    int64_t* v = malloc(sizeof(int64_t) * 3 * (size_t)N);
    const size_t lo = k * slots, len = n > lo ? (n - lo < slots ? n - lo : slots) : 0;
    int r = or_encode(x + lo, len, N, slots, delta, L, q, psi, m);
    if (!r) {
      or_sample_encrypt(seed, g0 + k, N, sigma, v, v + N, v + 2 * (size_t)N);
      or_encrypt(pk, m, v, v + N, v + 2 * (size_t)N, N, L, q, psi, out + k * 2 * (size_t)L * N);
    }
    if (r) {
#pragma omp critical
      if (!rc) rc = r;
    }
    free(m);
    free(v);
  }
  return rc;
}

int or_decrypt_vector(const uint64_t* cts, size_t K, const uint64_t* sk, uint32_t N, uint32_t L,
                      const uint64_t* q, const uint64_t* psi, uint32_t slots, double scale, size_t n,
                      double* out, int nthreads) {
  int rc = 0;
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1)
  for (size_t k = 0; k < K; ++k) {
    const size_t lo = k * slots;
    if (lo >= n) continue;
    const size_t len = n - lo < slots ? n - lo : slots;
    int r = or_decrypt(cts + k * 2 * (size_t)L * N, sk, N, L, q, psi, slots, scale, len, out + lo);
    if (r) {
#pragma omp critical
      if (!rc) rc = r;
    }
  }
  return rc;
}

/* PALISADE 1.11 CKKSPackedEncoding::Decode noise flooding [PALISADE-1.11, SURVEY
 * App. B.6], restated on the coefficient pairs above (output units; PALISADE's
 * 2^p-scaled values are these times 2^p, an exact power-of-two rescaling):
 *   conj_0 = (re_0, -im_0), conj_i = (-im_{S-i}, -re_{S-i})        (m(X^-1))
 *   u = v - conj over its S independent components (i = 0: im; 0 < i < S/2: re, im;
 *   i = S/2: re);  sigma = 0.5 * sqrt(sum (u - mean)^2 / (S - 1))  (S = 1: |im_0|)
 *   sigma_p = sigma 2^p;  fail if log2 sigma_p > p - 5;  sigma_p >= sqrt(N)/8;
 *   stddev_p = sqrt(M + 1) sigma_p;  logError = round(log2(stddev_p sqrt(2S))).
 * The normalisation constants are restated, not pinned (PALISADE absent). */
void or_decode_stats(const double* re, const double* im, uint32_t S, uint32_t N, uint32_t p_bits,
                     double m_factor, double* stddev_p, int* log_error, int* fail) {
  double sigma;
  uint32_t half = S / 2;
  if (S == 1) {
    sigma = fabs(im[0]);
  } else {
    double s1 = 0.0;
    for (uint32_t i = 0; i <= half; ++i) {
      if (i == 0) s1 += 2.0 * im[0];
      else if (i == half) s1 += re[i] + im[i];
      else s1 += (re[i] + im[S - i]) + (im[i] + re[S - i]);
    }
    double mean = s1 / (double)S, s2 = 0.0;
    for (uint32_t i = 0; i <= half; ++i) {
      double a, b;
      if (i == 0) { a = 2.0 * im[0]; s2 += (a - mean) * (a - mean); }
      else if (i == half) { a = re[i] + im[i]; s2 += (a - mean) * (a - mean); }
      else {
        a = re[i] + im[S - i];
        b = im[i] + re[S - i];
        s2 += (a - mean) * (a - mean) + (b - mean) * (b - mean);
      }
    }
    sigma = 0.5 * sqrt(s2 / (double)(S - 1));
  }
  double two_p = ldexp(1.0, (int)p_bits);
  double sp = sigma * two_p;
  *fail = !(log2(sp) <= (double)p_bits - 5.0);
  double fl = 0.125 * sqrt((double)N);
  if (sp < fl) sp = fl;
  *stddev_p = sqrt(m_factor + 1.0) * sp;
  *log_error = (int)rint(log2(*stddev_p * sqrt(2.0 * (double)S)));
}

/* (v + conj)/2 + nsd * z in place; z[2i], z[2i+1] = the (re, im) normals of slot i. */
void or_decode_symmetrize(double* re, double* im, uint32_t S, const double* z, double nsd) {
  uint32_t half = S / 2;
  for (uint32_t i = 0; i <= half; ++i) {
    if (i == 0) {
      re[0] = re[0] + nsd * z[0];
      im[0] = nsd * z[1];
      if (S == 1) break;
    } else if (i == half) {
      double a = re[i], b = im[i];
      re[i] = 0.5 * (a - b) + nsd * z[2 * i];
      im[i] = 0.5 * (b - a) + nsd * z[2 * i + 1];
    } else {
      double xr = re[i], xi = im[i], yr = re[S - i], yi = im[S - i];
      re[i] = 0.5 * (xr - yi) + nsd * z[2 * i];
      im[i] = 0.5 * (xi - yr) + nsd * z[2 * i + 1];
      re[S - i] = 0.5 * (yr - xi) + nsd * z[2 * (S - i)];
      im[S - i] = 0.5 * (yi - xr) + nsd * z[2 * (S - i) + 1];
    }
  }
}

/* ------------------------------------------------------------------------ */
/* Randomness spec of the product (NOT PALISADE's Blake2 PRNG, which is      */
/* seeded from std::random_device and cannot be reproduced).  Restated here  */
/* so GPU encrypt/keygen with a fixed seed can be checked bit-for-bit.       */
/*   ChaCha20 block (RFC 8439 rounds), state = consts | key[8] |              */
/*   counter64 (words 12,13) | nonce64 (words 14,15).                         */
/*   key[8] = splitmix64(seed) x4, each split lo/hi.                          */
/*   Stream (nonce, counter): u64 word w = block(w/8) words (2(w%8), 2(w%8)+1)*/
/*   (encrypt: coefficient j <- word (j mod N/8)*8 + j div N/8, see below)     */
/*   ternary: r % 3 - 1;  Gaussian: k = #{i : (r>>1) >= cdt[i]}, sign r&1.    */
/* ------------------------------------------------------------------------ */

#define ROTL32(v, n) (((v) << (n)) | ((v) >> (32 - (n))))
#define QR(a, b, c, d)            \
  a += b; d ^= a; d = ROTL32(d, 16); \
  c += d; b ^= c; b = ROTL32(b, 12); \
  a += b; d ^= a; d = ROTL32(d, 8);  \
  c += d; b ^= c; b = ROTL32(b, 7);

void or_chacha20_block(const uint32_t key[8], uint64_t counter, uint64_t nonce, uint32_t out[16]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                    key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                    (uint32_t)counter, (uint32_t)(counter >> 32), (uint32_t)nonce,
                    (uint32_t)(nonce >> 32)};
  uint32_t x[16];
  memcpy(x, s, sizeof(x));
  for (int i = 0; i < 10; ++i) {
    QR(x[0], x[4], x[8], x[12]);
    QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]);
    QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]);
    QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]);
    QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}

static uint64_t splitmix64(uint64_t* st) {
  uint64_t z = (*st += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
void or_seed_to_key(uint64_t seed, uint32_t key[8]) {
  uint64_t st = seed;
  for (int i = 0; i < 4; ++i) {
    uint64_t z = splitmix64(&st);
    key[2 * i] = (uint32_t)z;
    key[2 * i + 1] = (uint32_t)(z >> 32);
  }
}
/* u64 words [w0, w0+cnt) of stream (key, nonce) */
void or_stream_words(const uint32_t key[8], uint64_t nonce, uint64_t w0, size_t cnt,
                     uint64_t* out) {
  uint32_t blk[16];
  uint64_t cur = (uint64_t)-1;
  for (size_t i = 0; i < cnt; ++i) {
    uint64_t w = w0 + i;
    if (w / 8 != cur) {
      cur = w / 8;
      or_chacha20_block(key, cur, nonce, blk);
    }
    uint32_t k = (uint32_t)(w % 8);
    out[i] = (uint64_t)blk[2 * k] | ((uint64_t)blk[2 * k + 1] << 32);
  }
}

/* Cumulative distribution table for the discrete Gaussian D_{Z,sigma}
 * (P(x) ~ exp(-x^2 / (2 sigma^2)), sigma = 3.19 from cryptocontext.txt@2502),
 * folded to |x|: thresholds on 63-bit uniforms.  cdt[k] = floor(P(|x| <= k) *
 * 2^63) for k = 0..T-1 (T = ceil(13 sigma) + 1); value = #{k : u >= cdt[k]}. */
int or_gauss_cdt(double sigma, uint64_t* cdt, int max_entries) {
  int T = (int)ceil(13.0 * sigma) + 1;
  if (T > max_entries) return -1;
  long double S = 1.0L;
  for (int k = 1; k <= T; ++k) S += 2.0L * expl(-(long double)k * k / (2.0L * sigma * sigma));
  long double acc = 1.0L / S;
  for (int k = 0; k < T; ++k) {
    long double v = acc * 9223372036854775808.0L;
    cdt[k] = v >= 9223372036854775807.0L ? 0x7FFFFFFFFFFFFFFFull : (uint64_t)v;
    acc += 2.0L * expl(-(long double)(k + 1) * (k + 1) / (2.0L * sigma * sigma)) / S;
  }
  return T;
}
static inline int64_t gauss_from_word(uint64_t r, const uint64_t* cdt, int T) {
  uint64_t u = r >> 1;
  int64_t k = 0;
  for (int i = 0; i < T; ++i) k += (u >= cdt[i]);
  return (r & 1) ? -k : k;
}
static inline int64_t ternary_from_word(uint64_t r) { return (int64_t)(r % 3) - 1; }

/* Encrypt randomness for global ciphertext index g (sampler v2, round 3; the product's
 * kernels/dev_common.h states the same).  nonce = (1<<56)|g, ChaCha20 blocks of 16 32-bit
 * words; N16 = N/16, coefficient j = h + N16 i (h < N16, i < 16):
 *   v : block h/4 of [0, N/64), words 4(h%4)..+3 -> U = w0 + w1 2^32 + w2 2^64 + w3 2^96;
 *       trit_i = the i-th base-3 digit of U / 2^128 (U <- 3U mod 2^128, the carry out is
 *       the digit); v_j = trit_i - 1.
 *   e0: block N/64 + h, word i; e1: block N/64 + N16 + h, word i.  A word w: sign w & 1,
 *       U63 = (w >> 1) 2^32 + lo32, |e| = #{t : U63 >= cdt[t]}, where lo32 = word i of block
 *       N/64 + 2 N16 + h (e0) / N/64 + 3 N16 + h (e1) (the product reads it only when the
 *       top 31 bits tie with a table entry; here it is always read: same value). */
static inline int64_t gauss_from_split(uint32_t w, uint32_t lo, const uint64_t* cdt, int T) {
  const uint64_t u = ((uint64_t)(w >> 1) << 32) | lo;
  int64_t k = 0;
  for (int t = 0; t < T; ++t) k += (u >= cdt[t]);
  return (w & 1) ? -k : k;
}
void or_sample_encrypt(uint64_t seed, uint64_t g, uint32_t N, double sigma, int64_t* v,
                       int64_t* e0, int64_t* e1) {
  uint32_t key[8];
  or_seed_to_key(seed, key);
  uint64_t cdt[64];
  int T = or_gauss_cdt(sigma, cdt, 64);
  const uint64_t nonce = (1ull << 56) | g;
  const uint32_t N16 = N / 16, V0 = N / 64;
  for (uint32_t h = 0; h < N16; ++h) {
    uint32_t vb[16], b0[16], b1[16], t0[16], t1[16];
    or_chacha20_block(key, h / 4, nonce, vb);
    or_chacha20_block(key, V0 + h, nonce, b0);
    or_chacha20_block(key, V0 + N16 + h, nonce, b1);
    or_chacha20_block(key, V0 + 2ull * N16 + h, nonce, t0);
    or_chacha20_block(key, V0 + 3ull * N16 + h, nonce, t1);
    const uint32_t* w4 = vb + 4 * (h % 4);
    u128 U = (u128)w4[0] | ((u128)w4[1] << 32) | ((u128)w4[2] << 64) | ((u128)w4[3] << 96);
    for (uint32_t i = 0; i < 16; ++i) {
      const uint32_t j = h + N16 * i;
      /* 3U = 2U + U; the digit is the carry out of bit 128 */
      const u128 U2 = U << 1;
      uint32_t carry = (uint32_t)(U >> 127);
      const u128 U3 = U2 + U;
      carry += (U3 < U2);
      U = U3;
      v[j] = (int64_t)carry - 1;
      e0[j] = gauss_from_split(b0[i], t0[i], cdt, T);
      e1[j] = gauss_from_split(b1[i], t1[i], cdt, T);
    }
  }
}

/* uniform residue mod q from two words (bias < 2^-67) */
static uint64_t uniform_mod(uint64_t lo, uint64_t hi, uint64_t q) {
  return (uint64_t)((((u128)hi << 64) | lo) % q);
}

/* KeyGen randomness: nonce = (2<<56): s words [0,N), e words [N,2N);
 * a for tower t: nonce = (2<<56)|(1+t), words [0,2N) -> (lo,hi) pairs. */
void or_sample_keygen(uint64_t seed, uint32_t N, uint32_t L, const uint64_t* q, double sigma,
                      int64_t* s, int64_t* e, uint64_t* a_eval) {
  uint32_t key[8];
  or_seed_to_key(seed, key);
  uint64_t cdt[64];
  int T = or_gauss_cdt(sigma, cdt, 64);
  uint64_t* w = malloc(sizeof(uint64_t) * 2 * N);
  or_stream_words(key, 2ull << 56, 0, 2ull * N, w);
  for (uint32_t j = 0; j < N; ++j) {
    s[j] = ternary_from_word(w[j]);
    e[j] = gauss_from_word(w[N + j], cdt, T);
  }
  for (uint32_t t = 0; t < L; ++t) {
    or_stream_words(key, (2ull << 56) | (1 + t), 0, 2ull * N, w);
    for (uint32_t j = 0; j < N; ++j) a_eval[(size_t)t * N + j] = uniform_mod(w[2 * j], w[2 * j + 1], q[t]);
  }
  free(w);
}

/* Decode-flooding normals of ciphertext g (product spec): the slot at FFT-input
 * position P (slot i sits at P = bitrev(i), the order decrypt's CRT writes them) draws
 * ChaCha20 block (counter P >> 3, nonce (3 << 56) | g); its 32-bit words 2 (P mod 8) and
 * 2 (P mod 8) + 1 give one Box-Muller pair (u1 = (w + 1) 2^-32, u2 = w' 2^-32,
 * r = sqrt(-2 ln u1), (r cos 2 pi u2, r sin 2 pi u2)).  z[2i], z[2i+1] = (re, im)
 * normals of slot i. */
void or_flood_normals(uint64_t seed, uint64_t g, uint32_t S, double* z) {
  uint32_t key[8], blk[16];
  or_seed_to_key(seed, key);
  int logS = 0;
  while ((1u << logS) < S) ++logS;
  for (uint32_t P = 0; P < S; P += 8) {
    or_chacha20_block(key, P >> 3, (3ull << 56) | g, blk);
    for (uint32_t pr = 0; pr < 8 && P + pr < S; ++pr) {
      double u1 = ((double)blk[2 * pr] + 1.0) * 0x1.0p-32;
      double u2 = (double)blk[2 * pr + 1] * 0x1.0p-32;
      double r = sqrt(-2.0 * log(u1));
      uint32_t i = bitrev(P + pr, logS);
      z[2 * i] = r * cos(2.0 * M_PI * u2);
      z[2 * i + 1] = r * sin(2.0 * M_PI * u2);
    }
  }
}

/* Decode-flooding normals in the output domain (round 5, the product's stream for 2^6 slots and
 * more): slot i's normal is normal (i div S/16) of ChaCha20 block (i mod S/16) (nonce (3 << 56) | g);
 * the block's words 2m, 2m + 1 are one Box-Muller pair (as or_flood_normals), giving normals 2m
 * (r cos) and 2m + 1 (r sin).  zo[i] for i < S. */
void or_flood_out_normals(uint64_t seed, uint64_t g, uint32_t S, double* zo) {
  uint32_t key[8], blk[16];
  or_seed_to_key(seed, key);
  const uint32_t S16 = S / 16;
  for (uint32_t b = 0; b < S16; ++b) {
    or_chacha20_block(key, b, (3ull << 56) | g, blk);
    for (uint32_t m = 0; m < 8; ++m) {
      double u1 = ((double)blk[2 * m] + 1.0) * 0x1.0p-32;
      double u2 = (double)blk[2 * m + 1] * 0x1.0p-32;
      double r = sqrt(-2.0 * log(u1));
      zo[b + S16 * (2 * m)] = r * cos(2.0 * M_PI * u2);
      zo[b + S16 * (2 * m + 1)] = r * sin(2.0 * M_PI * u2);
    }
  }
}

/* decrypt + flooded decode of one ciphertext (seeded stream, ciphertext index g).
 * PALISADE adds N(0, sd) to every coefficient of the symmetrized decryption, then decodes: the
 * decoded slots' real parts carry Re(F z) sd for an i.i.d. standard complex Gaussian vector z of
 * the S FFT inputs.  FFTSpecial is F with F F^H = S I (rows: evaluations at the S powers zeta^(5^k)
 * of a primitive 4S-th root; distinct 5^k are congruent mod 4, so every off-diagonal geometric sum
 * vanishes), hence Re(F z) is i.i.d. N(0, S) over the slots: the same distribution as adding
 * N(0, sd sqrt(S)) to each decoded real part.  From 2^6 slots on that is how the noise is drawn
 * (or_flood_out_normals, round 5): the exact decode plus output-domain noise, so the product adds it
 * in the FFT's last pass.  Below 2^6 slots the input-domain form (round 2) stays. */
int or_decrypt_flood(const uint64_t* ct, const uint64_t* sk, uint32_t N, uint32_t L,
                     const uint64_t* q, const uint64_t* psi, uint32_t slots, double scale,
                     uint32_t p_bits, double m_factor, uint64_t seed, uint64_t g, size_t n,
                     double* out, int* log_error, int* fail) {
  if (n > slots) return -1;
  double* re = malloc(sizeof(double) * slots);
  double* im = malloc(sizeof(double) * slots);
  double* z = malloc(sizeof(double) * 2 * slots);
  int rc = or_decrypt_coeffs(ct, sk, N, L, q, psi, slots, scale, re, im);
  if (!rc) {
    double sd;
    or_decode_stats(re, im, slots, N, p_bits, m_factor, &sd, log_error, fail);
    const double nsd = sd / ldexp(1.0, (int)p_bits);
    if (slots >= 64) {
      or_flood_out_normals(seed, g, slots, z);
      or_fft_special(re, im, slots);
      const double nso = nsd * sqrt((double)slots);
      for (size_t i = 0; i < n; ++i) out[i] = re[i] + nso * z[i];
    } else {
      or_flood_normals(seed, g, slots, z);
      or_decode_symmetrize(re, im, slots, z, nsd);
      or_fft_special(re, im, slots);
      for (size_t i = 0; i < n; ++i) out[i] = re[i];
    }
  }
  free(z);
  free(re);
  free(im);
  return rc;
}

/* ------------------------------------------------------------------------ */
/* EvalMult (ct x ct) + HYBRID relinearization, ModReduce,     */
/* EvalMultKeyGen  [PALISADE-1.11: ParamsGenCKKS (HYBRID special primes),    */
/* KeySwitchHYBRID::KeySwitchGen / EvalFastKeySwitchCore (ApproxModUp,       */
/* ApproxModDown), DCRTPoly::DropLastElementAndScale].  The reference's      */
/* contexts are HYBRID / EXACTRESCALE / dnum 2 (cryptocontext.txt@2514); its */
/* one evaluation key (palisade_pybind/.../key-eval-mult.txt) pins the       */
/* special primes (tests/test_oracle_f4.py).  Textbook form: every product   */
/* reduced with u128 %, every conversion summed tower by tower.              */
/* ------------------------------------------------------------------------ */

/* bit length of prod(q[i0..i1)) via 32-bit limbs */
static uint32_t prod_bits(const uint64_t* q, uint32_t i0, uint32_t i1) {
  uint32_t limb[64] = {1};
  uint32_t n = 1;
  for (uint32_t i = i0; i < i1; ++i) {
    uint32_t parts[2] = {(uint32_t)q[i], (uint32_t)(q[i] >> 32)};
    uint32_t res[64] = {0};
    for (uint32_t a = 0; a < n; ++a)
      for (uint32_t b = 0; b < 2; ++b) {
        uint64_t carry = (uint64_t)limb[a] * parts[b];
        for (uint32_t c = a + b; carry; ++c) {
          carry += res[c];
          res[c] = (uint32_t)carry;
          carry >>= 32;
        }
      }
    n += 2;
    while (n > 1 && !res[n - 1]) --n;
    memcpy(limb, res, sizeof(limb));
  }
  uint32_t bits = 32 * (n - 1);
  for (uint32_t top = limb[n - 1]; top; top >>= 1) ++bits;
  return bits;
}

/* PALISADE 1.11 ParamsGenCKKS ring dimension for genCryptoContextCKKS(multDepth,
 * scaleFactorBits, batch) with ringDim 0 (ckks.cpp:28) [PALISADE-1.11]:
 *   qBound = firstModSize + (L - 1) scaleBits;  HYBRID: qBound += ceil(ceil(qBound/dnum)/60) 60
 *   N = smallest HE-standard (ternary, 128-bit classic) dimension with log2 bound >= qBound,
 *       and N >= 2 batch.
 * Pinned by code/params_results.csv:2-16: every (batch, scale bits) row has the N = 8192
 * archive size (tests/test_palisade_codec.py). Returns 0 when no dimension fits. */
uint32_t or_ring_dim(uint32_t L, uint32_t scale_bits, uint32_t first_mod_bits, uint32_t batch) {
  static const uint32_t dims[] = {1024, 2048, 4096, 8192, 16384, 32768, 65536, 131072};
  static const uint32_t maxlog[] = {27, 54, 109, 218, 438, 881, 1761, 3524};
  uint32_t dn = (L - 1 > 3) ? 3 : (L - 1 > 0 ? 2 : 1);
  if (dn > L) dn = L;
  uint32_t qb = (L > 1 ? first_mod_bits : scale_bits) + (L - 1) * scale_bits;
  uint32_t digit = (qb + dn - 1) / dn;
  qb += ((digit + 59) / 60) * 60;
  for (int i = 0; i < 8; ++i)
    if (qb <= maxlog[i] && dims[i] >= 2ull * batch) return dims[i];
  return 0;
}

/* ComputeNumLargeDigits(0, multDepth = L - 1): 3 above depth 3, 2 from depth 1, else 1;
 * alpha = ceil(L / dnum); kP = ceil(maxBits / 60) primes below FirstPrime(60, 2N) by
 * PreviousPrime, skipping Q's moduli; roots are the minimal primitive 2N-th roots. */
int or_special_primes(uint32_t N, uint32_t L, const uint64_t* q, uint32_t* dnum, uint32_t* alpha,
                      uint32_t* kP, uint64_t* p, uint64_t* ppsi) {
  uint32_t dn = (L - 1 > 3) ? 3 : (L - 1 > 0 ? 2 : 1);
  if (dn > L) dn = L;
  uint32_t al = (L + dn - 1) / dn, maxb = 0;
  for (uint32_t j = 0; j < dn; ++j) {
    uint32_t i1 = (j + 1) * al < L ? (j + 1) * al : L;
    uint32_t b = prod_bits(q, j * al, i1);
    if (b > maxb) maxb = b;
  }
  uint32_t k = (maxb + 59) / 60;
  uint64_t m = 2ull * N, c = or_first_prime(60, m);
  for (uint32_t i = 0; i < k; ++i) {
    int dup;
    do {
      c = or_prev_prime(c, m);
      dup = 0;
      for (uint32_t t = 0; t < L; ++t) dup |= (c == q[t]);
    } while (dup);
    p[i] = c;
    ppsi[i] = or_min_root(m, c);
  }
  *dnum = dn;
  *alpha = al;
  *kP = k;
  return 0;
}

/* tower t of the extended basis Q u P */
static inline uint64_t ext_mod(uint32_t t, uint32_t L, const uint64_t* q, const uint64_t* p) {
  return t < L ? q[t] : p[t - L];
}

/* EvalMultKeyGen with the product's seeded ChaCha20 stream: e_j words [0,N) of nonce
 * (4<<56)|(j<<16); a_{j,t} word pairs of nonce (4<<56)|(j<<16)|(1+t) (t over Q u P).
 * b_j[t] = e_j - a_j s + [t in digit j] (P mod q_t) s^2; evk [2][dnum][L+kP][N]. */
void or_evk_keygen(uint64_t seed, uint32_t N, uint32_t L, const uint64_t* q, const uint64_t* psi,
                   uint32_t kP, const uint64_t* p, const uint64_t* ppsi, uint32_t dnum, uint32_t alpha,
                   double sigma, const uint64_t* sk, uint64_t* evk) {
  uint32_t key[8];
  or_seed_to_key(seed, key);
  uint64_t cdt[64];
  int T = or_gauss_cdt(sigma, cdt, 64);
  const uint32_t T0 = L + kP;
  int64_t* s = malloc(sizeof(int64_t) * N);
  int64_t* e = malloc(sizeof(int64_t) * N);
  uint64_t* w = malloc(sizeof(uint64_t) * 2 * N);
  uint64_t* S = malloc(sizeof(uint64_t) * (size_t)T0 * N);
  uint64_t* E = malloc(sizeof(uint64_t) * N);
  /* s: centred coefficients of tower 0 of the secret key */
  memcpy(E, sk, sizeof(uint64_t) * N);
  or_ntt_inv(E, N, q[0], psi[0]);
  for (uint32_t i = 0; i < N; ++i) s[i] = E[i] > q[0] / 2 ? -(int64_t)(q[0] - E[i]) : (int64_t)E[i];
  for (uint32_t t = 0; t < T0; ++t) {
    uint64_t mt = ext_mod(t, L, q, p), rt = t < L ? psi[t] : ppsi[t - L];
    for (uint32_t i = 0; i < N; ++i) S[(size_t)t * N + i] = or_mod_signed(s[i], mt);
    or_ntt_fwd(S + (size_t)t * N, N, mt, rt);
  }
  for (uint32_t j = 0; j < dnum; ++j) {
    uint64_t nonce = (4ull << 56) | ((uint64_t)j << 16);
    or_stream_words(key, nonce, 0, N, w);
    for (uint32_t i = 0; i < N; ++i) e[i] = gauss_from_word(w[i], cdt, T);
    for (uint32_t t = 0; t < T0; ++t) {
      uint64_t mt = ext_mod(t, L, q, p), rt = t < L ? psi[t] : ppsi[t - L];
      for (uint32_t i = 0; i < N; ++i) E[i] = or_mod_signed(e[i], mt);
      or_ntt_fwd(E, N, mt, rt);
      uint64_t pm = 1;
      for (uint32_t u = 0; u < kP; ++u) pm = mulmod(pm, p[u] % mt, mt);
      int in_digit = t < L && t >= j * alpha && t < (j + 1) * alpha;
      uint64_t* a = w; /* reuse: word pairs of this tower */
      or_stream_words(key, nonce | (1 + t), 0, 2ull * N, a);
      uint64_t* B = evk + ((size_t)j * T0 + t) * N;
      uint64_t* A = evk + ((size_t)(dnum + j) * T0 + t) * N;
      const uint64_t* St = S + (size_t)t * N;
      for (uint32_t i = 0; i < N; ++i) {
        uint64_t av = uniform_mod(a[2 * i], a[2 * i + 1], mt);
        uint64_t b = submod(E[i], mulmod(av, St[i], mt), mt);
        if (in_digit) b = addmod(b, mulmod(pm, mulmod(St[i], St[i], mt), mt), mt);
        B[i] = b;
        A[i] = av;
      }
    }
  }
  free(s);
  free(e);
  free(w);
  free(S);
  free(E);
}

/* EvalMult of one ciphertext pair x, y [2][Ll][N] (EVALUATION) -> out [2][Ll][N]. */
void or_eval_mult(const uint64_t* x, const uint64_t* y, uint32_t N, uint32_t Ll, uint32_t L, const uint64_t* q,
                  const uint64_t* psi, uint32_t kP, const uint64_t* p, const uint64_t* ppsi, uint32_t dnum,
                  uint32_t alpha, const uint64_t* evk, uint64_t* out) {
  const uint32_t T = Ll + kP, T0 = L + kP, dn = (Ll + alpha - 1) / alpha;
  const size_t LN = (size_t)Ll * N;
  uint64_t* c2 = malloc(sizeof(uint64_t) * LN);
  uint64_t* ext = malloc(sizeof(uint64_t) * (size_t)T * N);
  uint64_t* acc = calloc((size_t)2 * T * N, sizeof(uint64_t));
  uint64_t* tmp = malloc(sizeof(uint64_t) * N);
  uint64_t em[32], er[32];
  for (uint32_t t = 0; t < T; ++t) {
    em[t] = t < Ll ? q[t] : p[t - Ll];
    er[t] = t < Ll ? psi[t] : ppsi[t - Ll];
  }
  /* tensor */
  for (uint32_t t = 0; t < Ll; ++t)
    for (uint32_t i = 0; i < N; ++i) {
      size_t e0 = (size_t)t * N + i, e1 = LN + e0;
      uint64_t qt = q[t];
      out[e0] = mulmod(x[e0], y[e0], qt);
      out[e1] = addmod(mulmod(x[e0], y[e1], qt), mulmod(x[e1], y[e0], qt), qt);
      c2[e0] = mulmod(x[e1], y[e1], qt);
    }
  for (uint32_t t = 0; t < Ll; ++t) or_ntt_inv(c2 + (size_t)t * N, N, q[t], psi[t]);
  /* ModUp per digit, inner product with the key */
  for (uint32_t j = 0; j < dn; ++j) {
    uint32_t s0 = j * alpha, cnt = (s0 + alpha <= Ll) ? alpha : Ll - s0;
    for (uint32_t t = 0; t < T; ++t) {
      uint64_t mt = em[t];
      uint64_t* o = ext + (size_t)t * N;
      if (t >= s0 && t < s0 + cnt) {
        memcpy(o, c2 + (size_t)t * N, sizeof(uint64_t) * N);
      } else {
        for (uint32_t i = 0; i < N; ++i) {
          uint64_t sum = 0;
          for (uint32_t u = 0; u < cnt; ++u) {
            uint64_t qi = q[s0 + u], hi_ = 1, ht = 1;
            for (uint32_t v = 0; v < cnt; ++v)
              if (v != u) {
                hi_ = mulmod(hi_, q[s0 + v] % qi, qi);
                ht = mulmod(ht, q[s0 + v] % mt, mt);
              }
            uint64_t yv = mulmod(c2[(size_t)(s0 + u) * N + i], inv_mod(hi_, qi), qi);
            sum = addmod(sum, mulmod(yv % mt, ht, mt), mt);
          }
          o[i] = sum;
        }
      }
      or_ntt_fwd(o, N, mt, er[t]);
      uint32_t tk = t < Ll ? t : L + (t - Ll);
      const uint64_t* B = evk + ((size_t)j * T0 + tk) * N;
      const uint64_t* A = evk + ((size_t)(dnum + j) * T0 + tk) * N;
      for (uint32_t i = 0; i < N; ++i) {
        size_t a0 = (size_t)t * N + i, a1 = (size_t)(T + t) * N + i;
        acc[a0] = addmod(acc[a0], mulmod(o[i], B[i], mt), mt);
        acc[a1] = addmod(acc[a1], mulmod(o[i], A[i], mt), mt);
      }
    }
  }
  /* ModDown: (acc_Q - conv_{P->Q}(acc_P)) P^-1, added to the tensor's c0, c1 */
  for (uint32_t poly = 0; poly < 2; ++poly) {
    uint64_t* a = acc + (size_t)poly * T * N;
    for (uint32_t m = 0; m < kP; ++m) or_ntt_inv(a + (size_t)(Ll + m) * N, N, p[m], ppsi[m]);
    for (uint32_t t = 0; t < Ll; ++t) {
      uint64_t qt = q[t], Pm = 1;
      for (uint32_t m = 0; m < kP; ++m) Pm = mulmod(Pm, p[m] % qt, qt);
      for (uint32_t i = 0; i < N; ++i) {
        uint64_t sum = 0;
        for (uint32_t m = 0; m < kP; ++m) {
          uint64_t pm = p[m], hp = 1, hq = 1;
          for (uint32_t v = 0; v < kP; ++v)
            if (v != m) {
              hp = mulmod(hp, p[v] % pm, pm);
              hq = mulmod(hq, p[v] % qt, qt);
            }
          uint64_t yv = mulmod(a[(size_t)(Ll + m) * N + i], inv_mod(hp, pm), pm);
          sum = addmod(sum, mulmod(yv % qt, hq, qt), qt);
        }
        tmp[i] = sum;
      }
      or_ntt_fwd(tmp, N, qt, psi[t]);
      uint64_t pinv = inv_mod(Pm, qt);
      uint64_t* o = out + (size_t)poly * LN + (size_t)t * N;
      for (uint32_t i = 0; i < N; ++i)
        o[i] = addmod(o[i], mulmod(submod(a[(size_t)t * N + i], tmp[i], qt), pinv, qt), qt);
    }
  }
  free(c2);
  free(ext);
  free(acc);
  free(tmp);
}

/* ModReduce of one ciphertext in [2][Ll][N] -> out [2][Ll-1][N]: (c_t - [c_l]) q_l^-1 with
 * [c_l] the last tower's coefficients taken centred (NativeVector::SwitchModulus). */
void or_rescale(const uint64_t* in, uint32_t N, uint32_t Ll, const uint64_t* q, const uint64_t* psi,
                uint64_t* out) {
  const uint32_t Lo = Ll - 1;
  const uint64_t ql = q[Lo];
  uint64_t* last = malloc(sizeof(uint64_t) * N);
  uint64_t* v = malloc(sizeof(uint64_t) * N);
  for (uint32_t poly = 0; poly < 2; ++poly) {
    memcpy(last, in + ((size_t)poly * Ll + Lo) * N, sizeof(uint64_t) * N);
    or_ntt_inv(last, N, ql, psi[Lo]);
    for (uint32_t t = 0; t < Lo; ++t) {
      uint64_t qt = q[t];
      for (uint32_t i = 0; i < N; ++i) {
        int64_t c = last[i] > ql / 2 ? -(int64_t)(ql - last[i]) : (int64_t)last[i];
        v[i] = or_mod_signed(c, qt);
      }
      or_ntt_fwd(v, N, qt, psi[t]);
      uint64_t inv = inv_mod(ql % qt, qt);
      const uint64_t* x = in + ((size_t)poly * Ll + t) * N;
      uint64_t* o = out + ((size_t)poly * Lo + t) * N;
      for (uint32_t i = 0; i < N; ++i) o[i] = mulmod(submod(x[i], v[i], qt), inv, qt);
    }
  }
  free(last);
  free(v);
}

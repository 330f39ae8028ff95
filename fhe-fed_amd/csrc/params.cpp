// params.cpp — host-side parameter generation and constant tables.
//
// Restates PALISADE 1.11 ParamsGen as reached from ckks.cpp:28
// (genCryptoContextCKKS(multDepth, scaleFactorBits, batchSize)): the EXACTRESCALE
// modulus chain, minimal primitive 2N-th roots and the HE-standard ring dimension.
// These are one-time setup computations on the host; every per-ciphertext
// operation runs in kernels.hip.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "shelfi_internal.h"

namespace shelfi {

static inline uint64_t mulmod(uint64_t a, uint64_t b, uint64_t q) {
  return (uint64_t)(((u128)a * b) % q);
}

uint64_t powmod(uint64_t a, uint64_t e, uint64_t q) {
  uint64_t r = 1 % q;
  a %= q;
  for (; e; e >>= 1) {
    if (e & 1) r = mulmod(r, a, q);
    a = mulmod(a, a, q);
  }
  return r;
}

uint64_t invmod(uint64_t a, uint64_t q) { return powmod(a, q - 2, q); }

uint64_t shoup(uint64_t w, uint64_t q) { return (uint64_t)(((u128)w << 64) / q); }

uint64_t mod_signed(int64_t v, uint64_t q) {
  if (v >= 0) return (uint64_t)v % q;
  uint64_t m = ((uint64_t)(-(v + 1)) + 1) % q;
  return m ? q - m : 0;
}

bool is_prime(uint64_t n) {
  static const uint64_t a[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
  if (n < 2) return false;
  for (uint64_t p : a)
    if (n % p == 0) return n == p;
  uint64_t d = n - 1;
  int s = 0;
  while (!(d & 1)) d >>= 1, ++s;
  for (uint64_t b : a) {
    uint64_t x = powmod(b, d, n);
    if (x == 1 || x == n - 1) continue;
    bool witness = true;
    for (int r = 1; r < s && witness; ++r) {
      x = mulmod(x, x, n);
      if (x == n - 1) witness = false;
    }
    if (witness) return false;
  }
  return true;
}

// PALISADE FirstPrime / PreviousPrime / NextPrime over q == 1 (mod m).
static uint64_t first_prime(uint32_t bits, uint64_t m) {
  uint64_t q = (1ull << bits) + 1;
  while (!is_prime(q)) q += m;
  return q;
}
static uint64_t prev_prime(uint64_t q, uint64_t m) {
  do q -= m;
  while (!is_prime(q));
  return q;
}
static uint64_t next_prime(uint64_t q, uint64_t m) {
  do q += m;
  while (!is_prime(q));
  return q;
}

// PALISADE RootOfUnity(m, q): smallest primitive m-th root (cryptocontext.txt@1935).
uint64_t min_root(uint64_t m, uint64_t q) {
  uint64_t r = 0;
  for (uint64_t g = 2;; ++g) {
    r = powmod(g, (q - 1) / m, q);
    if (powmod(r, m / 2, q) == q - 1) break;
  }
  uint64_t r2 = mulmod(r, r, q), x = r, best = r;
  for (uint64_t k = 1; k < m / 2; ++k) {
    x = mulmod(x, r2, q);
    if (x < best) best = x;
  }
  return best;
}

// PALISADE 1.11 ParamsGenCKKS's ring dimension, as reached from ckks.cpp:28
// (genCryptoContextCKKS(multDepth, scaleFactorBits, batchSize), ringDim 0, HYBRID key
// switching with dnum = ComputeNumLargeDigits(0, multDepth)) [PALISADE-1.11]:
//   qBound  = firstModSize + (numPrimes - 1) * scaleFactorBits          (an estimate in bits)
//   qBound += ceil(ceil(qBound / dnum) / 60) * 60                         (HYBRID: log2 P)
//   N       = FindRingDim(HEStd_ternary, HEStd_128_classic, qBound), and N >= 2 * batch.
// Bounding log2(Q * P), not log2 Q, is what code/params_results.csv:2-16 records: the
// archive size of one client's CNN_OriginalFedAvg ciphertexts is the same at scale bits 14,
// 20, 33, 40 and 52 for each batch, i.e. N = 8192 at every row (log Q alone would give 4096
// at batch 1024/2048 below 52 bits).
uint32_t hybrid_dnum(uint32_t L) {
  const uint32_t depth = L - 1;
  uint32_t dn = depth > 3 ? 3 : (depth > 0 ? 2 : 1);
  return dn > L ? L : dn;
}

double ring_dim_qbound(uint32_t L, uint32_t scale_bits, uint32_t first_mod_bits) {
  double qb = (L > 1 ? first_mod_bits : scale_bits) + (double)(L - 1) * scale_bits;
  qb += std::ceil(std::ceil(qb / hybrid_dnum(L)) / 60.0) * 60.0;
  return qb;
}

uint32_t default_ring_dim(uint32_t L, uint32_t scale_bits, uint32_t first_mod_bits,
                          uint32_t batch) {
  static const uint32_t dims[] = {1024, 2048, 4096, 8192, 16384, 32768, 65536, 131072};
  static const uint32_t maxlog[] = {27, 54, 109, 218, 438, 881, 1761, 3524};
  const double qb = ring_dim_qbound(L, scale_bits, first_mod_bits);
  for (int i = 0; i < 8; ++i)
    if (qb <= maxlog[i] && dims[i] >= 2ull * batch) return dims[i];
  return 0;
}

void generate_chain(uint32_t N, uint32_t L, uint32_t scale_bits, uint32_t first_mod_bits,
                    uint64_t* q, uint64_t* psi) {
  const uint64_t m = 2ull * N;
  q[L - 1] = first_prime(scale_bits, m);
  uint64_t qp = q[L - 1], qn = q[L - 1];
  unsigned cnt = 0;
  for (int i = (int)L - 2; i >= 1; --i, ++cnt) {
    if (cnt % 2 == 0)
      q[i] = qp = prev_prime(qp, m);
    else
      q[i] = qn = next_prime(qn, m);
  }
  if (L > 1)
    q[0] = (first_mod_bits == scale_bits) ? prev_prime(qp, m)
                                          : prev_prime(first_prime(first_mod_bits, m), m);
  for (uint32_t t = 0; t < L; ++t) psi[t] = min_root(m, q[t]);
}

// PALISADE 1.11 HYBRID key-switching parameters of a Q chain (ParamsGenCKKS):
// dnum = ComputeNumLargeDigits(0, multDepth) (3 above multDepth 3, 2 from 1, else 1), digits
// of alpha = ceil(L / dnum) towers, kP = ceil(maxBits / 60) special primes where maxBits is
// the bit length of the largest digit product, taken below FirstPrime(60, 2N) with
// PreviousPrime, skipping the moduli of Q.  Pinned by key-eval-mult.txt
// (palisade_pybind/SHELFI_FHE/resources/cryptoparams/: N = 2^14, Q = 60/52/53-bit towers,
// its key polynomials carry exactly the two special primes this returns).
void special_primes(uint32_t N, uint32_t L, const uint64_t* q, uint32_t* dnum, uint32_t* alpha,
                    uint32_t* kP, uint64_t* p, uint64_t* ppsi) {
  const uint32_t dn = hybrid_dnum(L);
  const uint32_t al = (L + dn - 1) / dn;
  uint32_t max_bits = 0;
  for (uint32_t j = 0; j < dn; ++j) {
    std::vector<uint64_t> prod(1, 1);  // little-endian 64-bit limbs
    for (uint32_t i = j * al; i < std::min(L, (j + 1) * al); ++i) {
      u128 carry = 0;
      for (auto& w : prod) {
        const u128 v = (u128)w * q[i] + carry;
        w = (uint64_t)v;
        carry = v >> 64;
      }
      if (carry) prod.push_back((uint64_t)carry);
    }
    uint32_t bits = 64 * (uint32_t)(prod.size() - 1);
    for (uint64_t top = prod.back(); top; top >>= 1) ++bits;
    max_bits = std::max(max_bits, bits);
  }
  const uint32_t k = (max_bits + 59) / 60;
  const uint64_t m = 2ull * N;
  uint64_t c = first_prime(60, m);
  for (uint32_t i = 0; i < k; ++i) {
    bool in_q;
    do {
      c = prev_prime(c, m);
      in_q = false;
      for (uint32_t t = 0; t < L; ++t) in_q = in_q || c == q[t];
    } while (in_q);
    p[i] = c;
    if (ppsi) ppsi[i] = min_root(m, c);
  }
  *dnum = dn;
  *alpha = al;
  *kP = k;
}

// CKKS special-FFT twiddles, flat index lenh + j, M = 4 * slots, ksi[k] =
// (cos 2 pi k / M, sin 2 pi k / M), rotGroup[j] = 5^j mod M (PALISADE
// DiscreteFourierTransform / HEAAN fftSpecial[Inv]).
void fft_twiddles(uint32_t slots, double* inv_re, double* inv_im, double* fwd_re,
                  double* fwd_im) {
  const uint64_t M = 4ull * slots;
  std::vector<uint64_t> rot(slots ? slots : 1);
  uint64_t f = 1;
  for (uint32_t j = 0; j < slots; ++j) rot[j] = f, f = (f * 5) % M;
  inv_re[0] = inv_im[0] = fwd_re[0] = fwd_im[0] = 0.0;
  for (uint32_t lenh = 1; lenh < slots; lenh <<= 1) {
    const uint64_t lenq = 8ull * lenh, g = M / lenq;
    for (uint32_t j = 0; j < lenh; ++j) {
      const uint64_t ii = ((lenq - rot[j] % lenq) * g) % M, fi = ((rot[j] % lenq) * g) % M;
      const double ai = 2.0 * M_PI * (double)ii / (double)M;
      const double af = 2.0 * M_PI * (double)fi / (double)M;
      inv_re[lenh + j] = std::cos(ai);
      inv_im[lenh + j] = std::sin(ai);
      fwd_re[lenh + j] = std::cos(af);
      fwd_im[lenh + j] = std::sin(af);
    }
  }
}

// Discrete Gaussian (sigma from cryptocontext.txt@2502) folded CDT on 63-bit
// uniforms: value = #{k : u >= cdt[k]}, sign from a separate bit.
int gauss_cdt(double sigma, uint64_t* cdt, int max_entries) {
  const int T = (int)std::ceil(13.0 * sigma) + 1;
  if (T > max_entries) return -1;
  long double S = 1.0L;
  for (int k = 1; k <= T; ++k) S += 2.0L * expl(-(long double)k * k / (2.0L * sigma * sigma));
  long double acc = 1.0L / S;
  for (int k = 0; k < T; ++k) {
    const long double v = acc * 9223372036854775808.0L;
    cdt[k] = v >= 9223372036854775807.0L ? 0x7FFFFFFFFFFFFFFFull : (uint64_t)v;
    acc += 2.0L * expl(-(long double)(k + 1) * (k + 1) / (2.0L * sigma * sigma)) / S;
  }
  return T;
}

uint64_t fnv1a(const void* data, size_t n, uint64_t h) {
  const uint8_t* p = (const uint8_t*)data;
  for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}

}  // namespace shelfi

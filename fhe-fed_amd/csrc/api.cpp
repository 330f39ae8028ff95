// api.cpp — the C ABI (include/shelfi.h) over the HIP kernels.
//
// Mirrors the reference's CKKS scheme wrapper, palisade_pybind/SHELFI_FHE/src/ckks.cpp:
//   shelfi_ctx_create        <- CKKS::CKKS                      (ckks.cpp:5-9)
//   shelfi_load              <- CKKS::loadCryptoParams          (ckks.cpp:11-23)
//   shelfi_keygen            <- CKKS::genCryptoContextAndKeyGen (ckks.cpp:25-59)
//   shelfi_encrypt           <- CKKS::encrypt                   (ckks.cpp:61-104)
//   shelfi_decrypt           <- CKKS::decrypt                   (ckks.cpp:170-213)
//   shelfi_weighted_average  <- CKKS::computeWeightedAverage    (ckks.cpp:264-320)
// Host code here only validates, moves bytes and precomputes constant tables; every
// per-ciphertext operation is a kernel in kernels.hip.
#include <sys/random.h>

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <fstream>
#include <mutex>
#include <new>

#include "api_util.h"
#include "host_stage.h"
#include "palisade_codec.h"
#include "palisade_io.h"
#include "shelfi_internal.h"

using namespace shelfi;

namespace shelfi {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

// ------------------------------------------------------------ blob format ----
// 64-byte little-endian header followed by K x 2 x L x N uint64 residues in the
// device layout [ct][poly][tower][coeff] (EVALUATION, PALISADE bit-reversed order).
struct BlobHeader {
  char magic[4];           // "SHCT"
  uint16_t version;        // 1
  uint16_t header_bytes;   // 64
  uint32_t logN;
  uint32_t L;
  uint64_t K;              // ciphertexts in the blob
  uint32_t depth;          // PALISADE depth (1 fresh, 2 after EvalMult by constant)
  uint32_t level;          // always 0 (no rescale on this path)
  double scale;            // scaling factor (Delta for fresh, Delta^2 after EvalMult)
  uint64_t params_id;      // hash of (N, L, q)
  uint64_t key_id;         // hash of the public key (PALISADE keyTag analogue)
  uint32_t batch;          // slots per ciphertext
  uint32_t encoding;       // 4 = CKKSPacked (PALISADE PlaintextEncodings)
};
static_assert(sizeof(BlobHeader) == 64, "blob header must be 64 bytes");

static uint64_t compute_params_id(const Params& p) {
  uint64_t h = fnv1a(&p.N, sizeof(p.N));
  h = fnv1a(&p.L, sizeof(p.L), h);
  return fnv1a(p.q, sizeof(uint64_t) * p.L, h);
}

static BlobHeader parse_blob(const uint8_t* blob, size_t len, const shelfi_ctx* ctx) {
  if (!blob || len < sizeof(BlobHeader)) throw Error{SHELFI_ERR_FORMAT, "ciphertext blob too short"};
  BlobHeader h;
  std::memcpy(&h, blob, sizeof(h));
  // version 1: uint64 residues [K][2][L][N]; version 2: the packed wire payload (the arena's slice
  // format with C = 1, U_t bits per residue: DESIGN.md §3, §5.3)
  if (std::memcmp(h.magic, "SHCT", 4) != 0 || (h.version != 1 && h.version != 2) || h.header_bytes != 64)
    throw Error{SHELFI_ERR_FORMAT, "not a SHELFI ciphertext blob (bad magic/version)"};
  if (h.L == 0 || h.L > kMaxTowers || h.logN < 10 || h.logN > 17)
    throw Error{SHELFI_ERR_FORMAT, "corrupt ciphertext blob header"};
  if (ctx) {
    if (h.logN != ctx->p.logN || h.L != ctx->p.L || h.params_id != ctx->params_id)
      throw Error{SHELFI_ERR_FORMAT, "ciphertext was produced under different crypto parameters"};
  }
  const uint64_t payload = len - sizeof(BlobHeader);
  if (h.version == 2 && !ctx) {
    // without a context the packed widths are unknown: a ciphertext is 2 (N / 512) rows of 64 U
    // bytes for some 32 L <= U <= 60 L
    const uint64_t unit = 2ull * (1ull << (h.logN - 9)) * 64;
    bool ok = h.K ? payload % h.K == 0 : payload == 0;
    if (ok && h.K) {
      const uint64_t per = payload / h.K;
      ok = per % unit == 0 && per / unit >= 32ull * h.L && per / unit <= 60ull * h.L;
    }
    if (!ok) throw Error{SHELFI_ERR_FORMAT, "ciphertext blob length does not match header"};
    return h;
  }
  // K comes from an untrusted header: bound it by the payload before multiplying, so a
  // forged K whose K * ct_bytes wraps mod 2^64 cannot pass the length check.
  const uint64_t ct_bytes = h.version == 1 ? 2ull * h.L * (8ull << h.logN) : arena_ct_words(ctx->p, 1) * 8;
  if (h.K > payload / ct_bytes || len != sizeof(BlobHeader) + h.K * ct_bytes)
    throw Error{SHELFI_ERR_FORMAT, "ciphertext blob length does not match header"};
  return h;
}

// Calls on one context are serialized (as the reference's GIL serializes its object).
static std::mutex& ctx_mutex(const shelfi_ctx* ctx) { return ctx->mu; }


void seed_to_key(uint64_t seed, uint32_t key[8]) {
  uint64_t st = seed;
  for (int i = 0; i < 4; ++i) {
    uint64_t z = (st += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    key[2 * i] = (uint32_t)z;
    key[2 * i + 1] = (uint32_t)(z >> 32);
  }
}

void os_random(void* buf, size_t n) {
  uint8_t* p = (uint8_t*)buf;
  while (n) {
    ssize_t r = getrandom(p, n, 0);
    if (r < 0) throw Error{SHELFI_ERR_DEVICE, "getrandom() failed"};
    p += r;
    n -= (size_t)r;
  }
}

// encryption/keygen stream key + first ciphertext index for this call
static void draw_key(shelfi_ctx* ctx, uint64_t count, uint32_t key[8], uint64_t* g0) {
  if (ctx->seed) {
    seed_to_key(ctx->seed, key);
    *g0 = ctx->enc_counter;
    ctx->enc_counter += count;
  } else {
    os_random(key, 32);
    *g0 = 0;
  }
}

// ------------------------------------------------------- tables / params ----
static void validate_params(uint32_t N, uint32_t L, uint32_t scale_bits, uint32_t first_mod_bits,
                            uint32_t batch) {
  if (L < 1 || L > (uint32_t)kMaxTowers) throw Error{SHELFI_ERR_ARG, "num_towers must be in [1,16]"};
  if (N < 1024 || N > (1u << 17) || (N & (N - 1)))
    throw Error{SHELFI_ERR_ARG, "ring dimension must be a power of two in [2^10, 2^17]"};
  if (!batch || (batch & (batch - 1)) || 2ull * batch > N)
    throw Error{SHELFI_ERR_ARG, "batchSize must be a power of two with 2*batchSize <= ring dimension"};
  if (scale_bits < 10 || scale_bits > 58)
    throw Error{SHELFI_ERR_ARG, "scaleFactorBits must be in [10, 58]"};
  if (first_mod_bits < scale_bits || first_mod_bits > 60)
    throw Error{SHELFI_ERR_ARG, "firstModBits must be in [scaleFactorBits, 60]"};
}

// Little-endian 30-bit limbs (the decode CRT's tables): the product of q[0..L) (except q[skip]), its
// two's-complement negation, mod 2^(30 n).
static std::vector<uint64_t> mw30_mul(std::vector<uint64_t> a, uint64_t m) {
  u128 carry = 0;
  for (auto& x : a) {
    const u128 v = (u128)x * m + carry;
    x = (uint64_t)v & ((1u << 30) - 1);
    carry = v >> 30;
  }
  return a;
}
static std::vector<uint64_t> mw30_qhat(const uint64_t* q, uint32_t L, uint32_t skip, uint32_t n) {
  std::vector<uint64_t> a(n, 0);
  a[0] = 1;
  for (uint32_t u = 0; u < L; ++u)
    if (u != skip) a = mw30_mul(std::move(a), q[u]);
  return a;
}
static std::vector<uint64_t> mw30_prod(const uint64_t* q, uint32_t L, uint32_t n) {
  return mw30_qhat(q, L, L, n);
}
static std::vector<uint64_t> mw30_neg(std::vector<uint64_t> a, uint32_t n) {
  uint64_t carry = 1;
  for (uint32_t j = 0; j < n; ++j) {
    const uint64_t v = ((~a[j]) & ((1u << 30) - 1)) + carry;
    a[j] = v & ((1u << 30) - 1);
    carry = v >> 30;
  }
  return a;
}

void free_ntt_tables(DeviceTables& dt) {
  dfree_t(dt.crt_mw);
  dt.crt_nc = 0;
  dfree_t(dt.tc);
  dfree_t(dt.psi_rev);
  dfree_t(dt.psi_rev_sh);
  dfree_t(dt.ipsi_rev);
  dfree_t(dt.ipsi_rev_sh);
  dfree_t(dt.tw_fwd_blk);
  dfree_t(dt.tw_inv_blk);
}

static void free_tables(shelfi_ctx* ctx) {
  eval_release(ctx, false);  // level / extended-basis tables belong to these parameters
  ctx->arena_refused.clear();  // arenas are laid out for these parameters
  free_ntt_tables(ctx->dt);
  dfree_t(ctx->dt.fft_inv);
  dfree_t(ctx->dt.fft_fwd);
  dfree_t(ctx->dt.cdt);
  dfree_t(ctx->dt.enc_tab);
  dfree_t(ctx->dt.enc_vtab);
}

static void free_keys(shelfi_ctx* ctx) {
  eval_release(ctx, true);  // the relinearization key belongs to the secret key
  ctx->arena_refused.clear();  // a reload starts a new parameter/key generation of arenas
  dfree_t(ctx->dk.pk);
  dfree_t(ctx->dk.pk_sh);
  dfree_t(ctx->dk.sk);
  dfree_t(ctx->dk.sk_sh);
  ctx->keys_loaded = false;
  ctx->key_id = 0;
  ctx->pk_host.clear();
  ctx->sk_host.clear();
}


static uint32_t bitrev_host(uint32_t x, uint32_t bits) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < bits; ++i) r = (r << 1) | ((x >> i) & 1);
  return r;
}

// NTT / CRT tables of the towers p.q[0..L) (the context's chain, one of its levels, or an
// extended basis Q_l u P of the key switching in eval.cpp).
void build_ntt_tables(const Params& p, DeviceTables& dt) {
  free_ntt_tables(dt);
  const uint32_t N = p.N, L = p.L;
  std::vector<TowerConst> tc(L);
  std::vector<uint64_t> pr((size_t)L * N), prs((size_t)L * N), ipr((size_t)L * N), iprs((size_t)L * N);
  for (uint32_t t = 0; t < L; ++t) {
    const uint64_t q = p.q[t];
    TowerConst& c = tc[t];
    std::memset(&c, 0, sizeof(c));
    c.q = q;
    c.one_shoup = (uint64_t)(((u128)1 << 64) / q);
    c.r30 = (1ull << 30) % q;
    c.r30_shoup = shoup(c.r30, q);
    c.r60 = (1ull << 60) % q;
    c.r60_shoup = shoup(c.r60, q);
    c.r64 = (uint64_t)(((u128)1 << 64) % q);
    c.r64_shoup = shoup(c.r64, q);
    c.ninv = invmod(N % q, q);
    c.ninv_shoup = shoup(c.ninv, q);
    uint64_t qhat_mod = 1;
    for (uint32_t u = 0; u < L; ++u)
      if (u != t) qhat_mod = (uint64_t)(((u128)qhat_mod * (p.q[u] % q)) % q);
    c.qhat_inv = invmod(qhat_mod, q);
    c.qhat_inv_shoup = shoup(c.qhat_inv, q);
    c.ninv_qhat = (uint64_t)(((u128)c.ninv * c.qhat_inv) % q);
    c.ninv_qhat_shoup = shoup(c.ninv_qhat, q);
    {
      const std::vector<uint64_t> qh = mw30_qhat(p.q, L, t, 7), nq = mw30_neg(mw30_prod(p.q, L, 7), 7);
      for (int j = 0; j < 7; ++j) {
        c.crt30[j] = (uint32_t)qh[j];
        c.nq30[j] = (uint32_t)nq[j];
      }
    }
    c.inv_q = 1.0 / (double)q;
    c.nq = (uint64_t)0 - q;
    c.n4q = (uint64_t)0 - (q << 2);
    c.n8q = (uint64_t)0 - (q << 3);
    {
      const uint32_t E = 63 - (uint32_t)__builtin_clzll(q);  // 2^E <= q < 2^(E+1)
      c.red_ok = E >= 40;
      c.red_sh = E >= 32 ? E - 32 : 0;
      c.red_r = c.red_ok ? (uint32_t)(((u128)1 << (32 + E)) / q) : 0;
      c.crt_sh = E >= 31 ? E - 31 : 0;
      c.bq62 = ((1ull << 62) / q) * q;
      c.inv_q32 = (float)((double)(1ull << c.crt_sh) / (double)q);
    }
    // twiddles: psi^bitrev(i), psi^-bitrev(i)
    const uint64_t ipsi = invmod(p.psi[t], q);
    uint64_t a = 1, b = 1;
    for (uint32_t i = 0; i < N; ++i) {
      const uint32_t r = bitrev_host(i, p.logN);
      pr[(size_t)t * N + r] = a;
      ipr[(size_t)t * N + r] = b;
      a = (uint64_t)(((u128)a * p.psi[t]) % q);
      b = (uint64_t)(((u128)b * ipsi) % q);
    }
    for (uint32_t i = 0; i < N; ++i) {
      prs[(size_t)t * N + i] = shoup(pr[(size_t)t * N + i], q);
      iprs[(size_t)t * N + i] = shoup(ipr[(size_t)t * N + i], q);
    }
    c.ninv_qhat_w1 = (uint64_t)(((u128)c.ninv_qhat * ipr[(size_t)t * N + 1]) % q);
    c.ninv_qhat_w1_shoup = shoup(c.ninv_qhat_w1, q);
  }
  {
    // decode's CRT (DeviceTables::crt_nc / crt_mw): |sum_t y_t Q/q_t - k Q| < L Q, plus a sign bit
    uint32_t qbits = 0;
    for (uint32_t t = 0; t < L; ++t) qbits += 64 - (uint32_t)__builtin_clzll(p.q[t]);
    const uint32_t need = qbits + (32 - (uint32_t)__builtin_clz(L)) + 1;
    const uint32_t nc = std::max<uint32_t>(5, (need + 29) / 30);
    dt.crt_nc = (L <= 7 && nc <= 7) ? nc : 0;
    const uint32_t NL = (need + 1 + 29) / 30, NW = (qbits + 63) / 64 + 1;
    if (NL > (uint32_t)kCrtMwMaxLimbs) throw Error{SHELFI_ERR_ARG, "tower chain too wide for the exact CRT"};
    std::vector<uint32_t> mw(4 + (size_t)(L + 2) * NL, 0);
    mw[0] = NL;
    mw[1] = NW;
    const std::vector<uint64_t> Qm = mw30_prod(p.q, L, NL), nQ = mw30_neg(Qm, NL);
    for (uint32_t t = 0; t < L; ++t) {
      const std::vector<uint64_t> qh = mw30_qhat(p.q, L, t, NL);
      for (uint32_t j = 0; j < NL; ++j) mw[4 + (size_t)t * NL + j] = (uint32_t)qh[j];
    }
    for (uint32_t j = 0; j < NL; ++j) {
      mw[4 + (size_t)L * NL + j] = (uint32_t)nQ[j];
      // (Q - 1) / 2 = Q >> 1 (Q odd)
      mw[4 + (size_t)(L + 1) * NL + j] = (uint32_t)((Qm[j] >> 1) | (j + 1 < NL ? (Qm[j + 1] & 1) << 29 : 0));
    }
    dt.crt_mw = upload(mw.data(), mw.size());
  }
  dt.tc = upload(tc.data(), L);
  dt.red_ok = true;
  for (uint32_t t = 0; t < L; ++t) dt.red_ok = dt.red_ok && tc[t].red_ok;
  dt.psi_rev = upload(pr.data(), pr.size());
  dt.psi_rev_sh = upload(prs.data(), prs.size());
  dt.ipsi_rev = upload(ipr.data(), ipr.size());
  dt.ipsi_rev_sh = upload(iprs.data(), iprs.size());
  {
    // per-block twiddle slices: entry 2^l + i of block b = psi table index
    // 2^(sstart + l) + b 2^l + i (local stage l of a 2^BL-element block)
    auto slices = [&](uint32_t BL, const std::vector<uint64_t>& w, const std::vector<uint64_t>& ws) {
      const uint32_t sstart = p.logN - BL;
      std::vector<ulonglong2> out((size_t)L * N);
      for (uint32_t t = 0; t < L; ++t)
        for (uint32_t b = 0; b < (1u << sstart); ++b) {
          const size_t base = (size_t)t * N + ((size_t)b << BL);
          out[base] = make_ulonglong2(0, 0);
          for (uint32_t l = 0; l < BL; ++l)
            for (uint32_t i = 0; i < (1u << l); ++i) {
              const size_t src = (size_t)t * N + (1ull << (sstart + l)) + ((size_t)b << l) + i;
              out[base + (1u << l) + i] = make_ulonglong2(w[src], ws[src]);
            }
        }
      return out;
    };
    const uint32_t BL = ntt_block_log(p.logN);
    dt.tw_fwd_blk = upload(slices(BL, pr, prs).data(), (size_t)L * N);
    dt.tw_inv_blk = upload(slices(BL, ipr, iprs).data(), (size_t)L * N);
  }
}

// (Re)build every device table for ctx->p.
static void build_tables(shelfi_ctx* ctx) {
  free_tables(ctx);
  Params& p = ctx->p;
  build_ntt_tables(p, ctx->dt);
  const uint32_t S = p.batch;
  std::vector<double> ir(S), ii(S), fr(S), fi(S);
  fft_twiddles(S, ir.data(), ii.data(), fr.data(), fi.data());
  std::vector<double2> tinv(S), tfwd(S);
  for (uint32_t i = 0; i < S; ++i) {
    tinv[i] = make_double2(ir[i], ii[i]);
    tfwd[i] = make_double2(fr[i], fi[i]);
  }
  ctx->dt.fft_inv = upload(tinv.data(), S);
  ctx->dt.fft_fwd = upload(tfwd.data(), S);
  uint64_t cdt[64];
  // <= 63 entries: the samplers' 6-step binary search over the 64-padded table counts
  // at most 63 (sigma <= 4.77; the default 3.19 gives 43)
  ctx->dt.cdt_len = gauss_cdt(p.sigma, cdt, 63);
  if (ctx->dt.cdt_len < 0) throw Error{SHELFI_ERR_ARG, "Gaussian table too large"};
  ctx->dt.cdt = upload(cdt, (size_t)ctx->dt.cdt_len);
  // enc_cols_fused's small-polynomial tables: the columns pass's first twiddles are
  // psi_rev[1] = psi^(N/2) (stage 0) and psi_rev[2], psi_rev[3] = psi^(N/4), psi^(3N/4) (stage 1)
  {
    std::vector<uint64_t> et((size_t)p.L * kEncTab);
    for (uint32_t t = 0; t < p.L; ++t) {
      const uint64_t q = p.q[t];
      const uint64_t W0 = powmod(p.psi[t], p.N / 2, q), W1 = powmod(p.psi[t], p.N / 4, q),
                     W2 = powmod(p.psi[t], 3ull * p.N / 4, q);
      const auto mul = [q](uint64_t a, uint64_t b) { return (uint64_t)(((u128)a * b) % q); };
      const auto sm = [q](int v) { return v < 0 ? q - (uint64_t)(-v) : (uint64_t)v; };  // |v| < q
      const auto add = [q](uint64_t a, uint64_t b) { return (uint64_t)(((u128)a + b) % q); };
      const auto sub = [q](uint64_t a, uint64_t b) { return a >= b ? a - b : a + q - b; };
      uint64_t* T = et.data() + (size_t)t * kEncTab;
      for (int idx = 0; idx < 81; ++idx) {
        const uint64_t a = sm(idx % 3 - 1), b = sm(idx / 3 % 3 - 1), c = sm(idx / 9 % 3 - 1), d = sm(idx / 27 - 1);
        const uint64_t u = add(a, mul(W0, c)), v = add(b, mul(W0, d));  // stage 0 (pairs a-c, b-d)
        const uint64_t u2 = sub(a, mul(W0, c)), v2 = sub(b, mul(W0, d));
        T[0 * 81 + idx] = add(u, mul(W1, v));  // stage 1 (pairs a'-b' with W1, c'-d' with W2)
        T[1 * 81 + idx] = sub(u, mul(W1, v));
        T[2 * 81 + idx] = add(u2, mul(W2, v2));
        T[3 * 81 + idx] = sub(u2, mul(W2, v2));
      }
      for (int e = -64; e < 64; ++e) {
        const uint64_t m = mul(W0, sm(e < 0 ? -e : e));
        T[kEncVTab + 64 + e] = e < 0 ? (m ? q - m : 0) : m;
      }
    }
    ctx->dt.enc_tab = upload(et.data(), et.size());
  }
  // NTT(v)'s 4 column stages as table sums (DeviceTables::enc_vtab): the stages' 16 x 16 matrix M_t
  // (row r' of the output from input row r, the columns pass's twiddles psi_rev[m + i] at stage
  // s = log2 m) applied to the ternary rows of each group g = {g, g + 4, g + 8, g + 12}
  if (p.logN >= 15 && p.logN - ntt_block_log(p.logN) == 4) {
    constexpr int R = 16;
    std::vector<uint64_t> vt((size_t)p.L * R * 4 * 81);
    for (uint32_t t = 0; t < p.L; ++t) {
      const uint64_t q = p.q[t];
      const auto mul = [q](uint64_t a, uint64_t b) { return (uint64_t)(((u128)a * b) % q); };
      const auto add = [q](uint64_t a, uint64_t b) { return (uint64_t)(((u128)a + b) % q); };
      const auto sub = [q](uint64_t a, uint64_t b) { return a >= b ? a - b : a + q - b; };
      // psi_rev[m + i] = psi^bitrev_logN(m + i)
      const auto tw = [&](uint32_t idx) { return powmod(p.psi[t], bitrev_host(idx, p.logN), q); };
      uint64_t M[R][R];  // M[r'][r]
      for (int r = 0; r < R; ++r) {
        uint64_t x[R] = {0};
        x[r] = 1;
        for (int s = 0; s < 4; ++s) {
          const int m = 1 << s, tr = R >> (s + 1);
          for (int i = 0; i < m; ++i) {
            const uint64_t W = tw((uint32_t)(m + i));
            for (int jj = 0; jj < tr; ++jj) {
              const int r0 = 2 * i * tr + jj, r1 = r0 + tr;
              const uint64_t a = x[r0], b = mul(W, x[r1]);
              x[r0] = add(a, b);
              x[r1] = sub(a, b);
            }
          }
        }
        for (int rp = 0; rp < R; ++rp) M[rp][r] = x[rp];
      }
      for (int rp = 0; rp < R; ++rp)
        for (int g = 0; g < 4; ++g)
          for (int idx = 0; idx < 81; ++idx) {
            uint64_t acc = 0;
            for (int kk = 0, d = idx; kk < 4; ++kk, d /= 3) {
              const int trit = d % 3 - 1;
              const uint64_t e = M[rp][g + 4 * kk];
              acc = trit > 0 ? add(acc, e) : trit < 0 ? sub(acc, e) : acc;
            }
            vt[(((size_t)t * R + rp) * 4 + g) * 81 + idx] = acc;
          }
    }
    ctx->dt.enc_vtab = upload(vt.data(), vt.size());
  }
  ctx->params_id = compute_params_id(p);
}

static void set_params(shelfi_ctx* ctx, uint32_t N, uint32_t L, uint32_t scale_bits,
                       uint32_t first_mod_bits, uint32_t batch, const uint64_t* q,
                       const uint64_t* psi) {
  Params p;
  p.N = N;
  p.logN = (uint32_t)__builtin_ctz(N);
  p.L = L;
  p.batch = batch;
  p.gap = N / (2 * batch);
  p.scale_bits = scale_bits;
  p.first_mod_bits = first_mod_bits;
  for (uint32_t t = 0; t < L; ++t) {
    if (q[t] >= (1ull << 60) || q[t] % (2ull * N) != 1)
      throw Error{SHELFI_ERR_ARG, "modulus out of range (need q < 2^60, q = 1 mod 2N)"};
    if (powmod(psi[t], N, q[t]) != q[t] - 1)
      throw Error{SHELFI_ERR_ARG, "root of unity is not a primitive 2N-th root"};
    p.q[t] = q[t];
    p.psi[t] = psi[t];
  }
  // EXACTRESCALE level-0 scaling factor = (double)q_{L-1} (CT1.txt@265059).
  p.delta = (double)q[L - 1];
  ctx->p = p;
  build_tables(ctx);
}

// keys: host copies -> device (+ Shoup companions)
static void install_keys(shelfi_ctx* ctx, const uint64_t* pk, const uint64_t* sk, bool palisade) {
  const Params& p = ctx->p;
  const size_t LN = (size_t)p.L * p.N;
  for (size_t i = 0; i < 2 * LN; ++i)
    if (pk[i] >= p.q[(i / p.N) % p.L]) throw Error{SHELFI_ERR_FORMAT, "public key residue >= q"};
  for (size_t i = 0; i < LN; ++i)
    if (sk[i] >= p.q[i / p.N]) throw Error{SHELFI_ERR_FORMAT, "secret key residue >= q"};
  free_keys(ctx);
  std::vector<uint64_t> pks(2 * LN), sks(LN);
  for (size_t i = 0; i < 2 * LN; ++i) pks[i] = shoup(pk[i], p.q[(i / p.N) % p.L]);
  for (size_t i = 0; i < LN; ++i) sks[i] = shoup(sk[i], p.q[i / p.N]);
  ctx->dk.pk = upload(pk, 2 * LN);
  ctx->dk.pk_sh = upload(pks.data(), 2 * LN);
  ctx->dk.sk = upload(sk, LN);
  ctx->dk.sk_sh = upload(sks.data(), LN);
  ctx->pk_host.assign(pk, pk + 2 * LN);
  ctx->sk_host.assign(sk, sk + LN);
  ctx->key_id = fnv1a(pk, sizeof(uint64_t) * 2 * LN, ctx->params_id);
  ctx->keys_loaded = true;
  ctx->palisade_keys = palisade;
  if (!palisade) {  // PALISADE wire format needs the PALISADE context + key tag
    ctx->pal_ctx_obj.clear();
    ctx->pal_keytag.clear();
    ctx->wire = 0;
  }
}

void require_keys(const shelfi_ctx* ctx) {
  if (!ctx->keys_loaded)
    throw Error{SHELFI_ERR_STATE,
                "no keys: call loadCryptoParams() or genCryptoContextAndKeyGen() first"};
}

// -------------------------------------------------- own key-file format ----
// cryptocontext.txt: "SHCC" u32 version, u32 N, L, batch, scale_bits, first_mod_bits,
//                    f64 sigma, u64 q[L], u64 psi[L]
// key-public.txt:    "SHPK" u32 version, u64 params_id, u64 [2][L][N]
// key-private.txt:   "SHSK" u32 version, u64 params_id, u64 [L][N]
static void write_file(const std::string& path, const std::string& data) {
  std::ofstream f(path, std::ios::binary | std::ios::trunc);
  if (!f) throw Error{SHELFI_ERR_IO, "cannot open " + path + " for writing"};
  f.write(data.data(), (std::streamsize)data.size());
  if (!f) throw Error{SHELFI_ERR_IO, "error writing " + path};
}
static std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw Error{SHELFI_ERR_IO, "could not read " + path};
  return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}
template <class T>
static void put(std::string& s, const T& v) {
  s.append(reinterpret_cast<const char*>(&v), sizeof(T));
}
template <class T>
static T get(const std::string& s, size_t& off) {
  if (off + sizeof(T) > s.size()) throw Error{SHELFI_ERR_FORMAT, "truncated key file"};
  T v;
  std::memcpy(&v, s.data() + off, sizeof(T));
  off += sizeof(T);
  return v;
}

// PALISADE context parameters of ctx->p, as genCryptoContextCKKS(multDepth, scaleFactorBits,
// batchSize) records them (ckks.cpp:28): the scaling-factor bits in the plaintext-modulus
// field, the batch in the encoding parameters, the default RLWE fields of the reference's
// committed cryptocontext.txt.
static PalisadeCtxParams palisade_params_of(const Params& p) {
  PalisadeCtxParams cp;
  cp.N = p.N;
  cp.L = p.L;
  cp.q.assign(p.q, p.q + p.L);
  cp.psi.assign(p.psi, p.psi + p.L);
  cp.plaintext_modulus = p.scale_bits;
  cp.batch = p.batch;
  cp.sigma = (float)p.sigma;
  // the block ends (..., ks = HYBRID 2, rs = EXACTRESCALE 1, dnum): dnum follows multDepth
  // (2 for the reference's multDepth 1 and for key-eval-mult.txt's multDepth 2; special_primes)
  uint32_t dn, al, kp;
  uint64_t sp[kMaxTowers];
  special_primes(p.N, p.L, p.q, &dn, &al, &kp, sp, nullptr);
  cp.fields.back() = dn;
  return cp;
}

// PALISADE's GenerateUniqueKeyID: four 32-bit draws, 8 lowercase hex digits each
static std::string make_keytag(const shelfi_ctx* ctx) {
  uint32_t r[4];
  if (ctx->seed) {
    uint32_t k[8];
    seed_to_key(ctx->seed ^ 0x6b65797461670000ull, k);  // "keytag"
    std::memcpy(r, k, sizeof(r));
  } else {
    os_random(r, sizeof(r));
  }
  char buf[33];
  for (int i = 0; i < 4; ++i) std::snprintf(buf + 8 * i, 9, "%08x", r[i]);
  return std::string(buf, 32);
}

// W = (int64)((double)(float)w * Delta + 0.5) (ckks.cpp:287-288, PALISADE EvalMult by a
// constant). The cast is undefined for NaN, +-inf and |w * Delta| >= 2^63, so such weights
// are rejected instead of producing a garbage aggregate.
static int64_t weight_int(float w, double delta) {
  const double v = (double)w * delta + 0.5;
  if (!std::isfinite(v) || v >= 9223372036854775808.0 || v < -9223372036854775808.0)
    throw Error{SHELFI_ERR_RANGE, "scaling factor is not finite or |w * scale| >= 2^63"};
  return (int64_t)v;
}

static void check_weights(const float* w, size_t n, double delta) {
  for (size_t c = 0; c < n; ++c) (void)weight_int(w[c], delta);
}

// W per learner, split into 30-bit limbs
static void fill_weights(WavgArgs& a, const Params& p, const float* w, size_t n) {
  for (size_t c = 0; c < n; ++c) {
    const int64_t W = weight_int(w[c], p.delta);
    for (uint32_t t = 0; t < p.L; ++t) {
      const uint64_t wt = mod_signed(W, p.q[t]);
      a.wl[c][t][0] = (uint32_t)(wt & ((1u << 30) - 1));
      a.wl[c][t][1] = (uint32_t)(wt >> 30);
    }
  }
}

// Weight limbs [C][L][2] of wavg_packed in a device buffer: a ring of slots, the
// last one reused while the weights repeat (every step of a round), a slot rewritten
// only after the kernels that read it have completed.
static int arena_weight_slot(shelfi_ctx* ctx, const float* w, size_t C, hipStream_t s) {
  const Params& p = ctx->p;
  std::vector<uint32_t> wl(C * p.L * 2);
  for (size_t c = 0; c < C; ++c) {
    const int64_t W = weight_int(w[c], p.delta);  // ckks.cpp:287-288
    for (uint32_t t = 0; t < p.L; ++t) {
      const uint64_t wt = mod_signed(W, p.q[t]);
      wl[(c * p.L + t) * 2] = (uint32_t)(wt & ((1u << 30) - 1));
      wl[(c * p.L + t) * 2 + 1] = (uint32_t)(wt >> 30);
    }
  }
  const int last = ctx->wl_last_slot;
  if (last >= 0 && ctx->wl_host[last] == wl) return last;
  const int i = ctx->wl_next;
  ctx->wl_next = (i + 1) % shelfi_ctx::kWeightRing;
  if (ctx->wl_done[i]) SHELFI_HIP(hipEventSynchronize(ctx->wl_done[i]));
  else SHELFI_HIP(hipEventCreateWithFlags(&ctx->wl_done[i], hipEventDisableTiming));
  const size_t bytes = wl.size() * sizeof(uint32_t);
  if (ctx->wl_cap[i] < bytes) {
    if (ctx->wl_dev[i]) (void)hipFree(ctx->wl_dev[i]);
    ctx->wl_dev[i] = nullptr;
    ctx->wl_cap[i] = 0;
    SHELFI_HIP(hipMalloc(&ctx->wl_dev[i], bytes));
    ctx->wl_cap[i] = bytes;
  }
  ctx->wl_host[i] = std::move(wl);  // stays alive until the slot is reused
  SHELFI_HIP(hipMemcpyAsync(ctx->wl_dev[i], ctx->wl_host[i].data(), bytes, hipMemcpyHostToDevice, s));
  ctx->wl_last_slot = i;
  return i;
}

// Process-wide switches: each reload publishes a new immutable snapshot through an
// atomic pointer; snapshots are never freed (a few dozen bytes per reload), so a launch path on
// another thread reads a consistent struct, never one being written.
static std::atomic<const Switches*> g_switches{nullptr};

static bool env_flag(const char* name, char off_or_on, bool dflt) {
  const char* e = getenv(name);
  return e && *e == off_or_on ? !dflt : dflt;
}
static int env_choice(const char* name, std::initializer_list<int> allowed, int dflt) {
  const char* e = getenv(name);
  if (!e) return dflt;
  const int v = atoi(e);
  for (int a : allowed)
    if (a == v) return v;
  return dflt;
}

void reload_switches() {
  Switches s;
  s.xcd_order = env_flag("SHELFI_XCD_ORDER", '0', true);
  s.ntt_wl = env_flag("SHELFI_NTT_WL", '0', true);
  s.fft_ct = env_flag("SHELFI_FFT_CT", '0', true);
  s.fft_whole = env_flag("SHELFI_FFT_WHOLE", '0', true);
  s.enc_fused = env_flag("SHELFI_ENC_FUSED_COLS", '0', true);
  s.enc_pp = env_flag("SHELFI_ENC_PP", '0', true);
  s.dec_pp = env_flag("SHELFI_DEC_PP", '0', true);
  s.enc_nored = env_flag("SHELFI_ENC_NORED", '0', true);
  s.enc_tab = env_flag("SHELFI_ENC_TAB", '0', true);
  s.enc_vt = env_flag("SHELFI_ENC_VT", '0', true);
  s.enc_ts = env_choice("SHELFI_ENC_TS", {0, 1}, -1);
  s.dec_all_towers = env_flag("SHELFI_DEC_ALL_TOWERS", '1', false);
  s.enc_x5 = env_flag("SHELFI_ENC_X5", '0', true);
  s.stage_trace = env_choice("SHELFI_STAGE_TRACE", {0, 1}, 0) == 1;
  if (const char* e = getenv("SHELFI_PACK_KERNEL")) s.pack_kernel = !strcmp(e, "v4") ? 4 : !strcmp(e, "r3") ? 3 : 0;
  s.pack_unroll = env_choice("SHELFI_PACK_UNROLL", {1, 2, 4, 8}, 0);
  s.pack_waves = env_choice("SHELFI_PACK_WAVES", {2, 8}, 0);
  s.wavg_rows = env_choice("SHELFI_WAVG_ROWS", {1, 2}, 0);
  if (const char* e = getenv("SHELFI_WAVG_STRANDS"))
    if (atoi(e) > 1 && atoi(e) <= 4096) s.wavg_strands = (uint32_t)atoi(e);
  s.arena_stager = env_choice("SHELFI_ARENA_STAGER", {0, 1}, -1);
  if (const char* e = getenv("SHELFI_DEV_CHUNK_MIB"))
    if (atoll(e) > 0) s.dev_chunk_mib = (uint64_t)atoll(e);
  if (const char* e = getenv("SHELFI_WAVG_CHUNK_MIB"))
    if (atoll(e) > 0) s.wavg_chunk_mib = (uint64_t)atoll(e);
  if (const char* e = getenv("SHELFI_STAGE_SLOT_MIB"))
    if (atoll(e) > 0 && atoll(e) <= 256) s.stage_slot_mib = (uint64_t)atoll(e);
  s.h2d_direct = env_flag("SHELFI_H2D_DIRECT", '1', false);
  s.h2d_two = env_flag("SHELFI_H2D_TWO", '0', true);
  g_switches.store(new Switches(s), std::memory_order_release);
}
const Switches& switches() { return *g_switches.load(std::memory_order_acquire); }
static const bool g_switches_read = (reload_switches(), true);

}  // namespace shelfi

// ============================================================== C ABI ======
extern "C" {

void shelfi_reload_switches(void) { reload_switches(); }

int shelfi_abi_version(void) { return SHELFI_ABI_VERSION; }
const char* shelfi_last_error(void) { return g_last_error.c_str(); }
void shelfi_free(void* p) { std::free(p); }

int shelfi_params_generate(uint32_t ring_dim, uint32_t num_towers, uint32_t scale_bits,
                           uint32_t first_mod_bits, uint32_t batch, uint32_t* ring_dim_out,
                           uint64_t* moduli_out, uint64_t* roots_out) {
  return guarded([&] {
    uint32_t N = ring_dim ? ring_dim
                          : default_ring_dim(num_towers, scale_bits, first_mod_bits, batch);
    if (!N) throw Error{SHELFI_ERR_ARG, "no ring dimension satisfies the security/batch constraints"};
    validate_params(N, num_towers, scale_bits, first_mod_bits, batch);
    uint64_t q[kMaxTowers], psi[kMaxTowers];
    generate_chain(N, num_towers, scale_bits, first_mod_bits, q, psi);
    if (ring_dim_out) *ring_dim_out = N;
    for (uint32_t t = 0; t < num_towers; ++t) {
      if (moduli_out) moduli_out[t] = q[t];
      if (roots_out) roots_out[t] = psi[t];
    }
  });
}

int shelfi_read_palisade(const char* cryptodir, uint32_t* ring_dim, uint32_t* num_towers,
                         uint64_t* moduli, uint64_t* roots, uint64_t* pk, uint64_t* sk) {
  if (!cryptodir) return SHELFI_ERR_ARG;
  return guarded([&] {
    const std::string dir(cryptodir);
    PalisadeContext pc = palisade_read_context(read_file(dir + "cryptocontext.txt"));
    const uint32_t L = (uint32_t)pc.q.size();
    if (ring_dim) *ring_dim = pc.N;
    if (num_towers) *num_towers = L;
    for (uint32_t t = 0; t < L; ++t) {
      if (moduli) moduli[t] = pc.q[t];
      if (roots) roots[t] = pc.psi[t];
    }
    if (pk || sk) {
      std::vector<uint64_t> p, s;
      palisade_read_keys(read_file(dir + "key-public.txt"), read_file(dir + "key-private.txt"),
                         pc.N, pc.q, p, s);
      if (pk) std::memcpy(pk, p.data(), p.size() * 8);
      if (sk) std::memcpy(sk, s.data(), s.size() * 8);
    }
  });
}

int shelfi_ctx_create(uint32_t ring_dim, uint32_t num_towers, uint32_t scale_bits,
                      uint32_t first_mod_bits, uint32_t batch, int device, shelfi_ctx** out) {
  if (!out) return SHELFI_ERR_ARG;
  *out = nullptr;
  shelfi_ctx* ctx = new (std::nothrow) shelfi_ctx();
  if (!ctx) return SHELFI_ERR_DEVICE;
  reload_switches();  // the process-wide probe switches are re-read when a context is created
  int rc = guarded([&] {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
      throw Error{SHELFI_ERR_DEVICE, "no HIP device available (libshelfi requires an MI355X / gfx950)"};
    if (device < 0 || device >= count) throw Error{SHELFI_ERR_ARG, "device ordinal out of range"};
    hipDeviceProp_t prop;
    SHELFI_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
      throw Error{SHELFI_ERR_DEVICE, std::string("device is ") + prop.gcnArchName +
                                         "; libshelfi is built for gfx950 only"};
    ctx->device = device;
    DeviceGuard g(device);
    uint32_t N = ring_dim ? ring_dim
                          : default_ring_dim(num_towers, scale_bits, first_mod_bits, batch);
    if (!N) throw Error{SHELFI_ERR_ARG, "no ring dimension satisfies the security/batch constraints"};
    validate_params(N, num_towers, scale_bits, first_mod_bits, batch);
    uint64_t q[kMaxTowers], psi[kMaxTowers];
    generate_chain(N, num_towers, scale_bits, first_mod_bits, q, psi);
    SHELFI_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    SHELFI_HIP(hipStreamCreateWithFlags(&ctx->stream2, hipStreamNonBlocking));
    SHELFI_HIP(hipStreamCreateWithFlags(&ctx->stream3, hipStreamNonBlocking));
    SHELFI_HIP(hipMalloc(&ctx->dev_flag, 32));
    SHELFI_HIP(hipHostMalloc((void**)&ctx->host_flag, 32, hipHostMallocDefault));
    // GenFlag words: pinned, mapped and coherent host memory the kernels store to (system scope)
    SHELFI_HIP(hipHostMalloc((void**)&ctx->map_flag_host, 64, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(ctx->map_flag_host, 0, 64);
    SHELFI_HIP(hipHostGetDevicePointer((void**)&ctx->map_flag_dev, ctx->map_flag_host, 0));
    set_params(ctx, N, num_towers, scale_bits, first_mod_bits, batch, q, psi);
  });
  if (rc != SHELFI_OK) {
    shelfi_ctx_destroy(ctx);
    return rc;
  }
  *out = ctx;
  return SHELFI_OK;
}

void shelfi_ctx_destroy(shelfi_ctx* ctx) {
  if (!ctx) return;
  {
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
    if (ctx->stream3) (void)hipStreamSynchronize(ctx->stream3);
    comm_release(ctx);
    free_keys(ctx);
    free_tables(ctx);
    delete ctx->stage;
    ctx->stage = nullptr;
    delete ctx->drain;
    ctx->drain = nullptr;
    delete ctx->up2;
    ctx->up2 = nullptr;
    if (ctx->stream4) (void)hipStreamDestroy(ctx->stream4);
    ctx->stream4 = nullptr;
    for (int i = 0; i < shelfi_ctx::kWeightRing; ++i) {
      if (ctx->wl_done[i]) (void)hipEventSynchronize(ctx->wl_done[i]);
      if (ctx->wl_done[i]) (void)hipEventDestroy(ctx->wl_done[i]);
      if (ctx->wl_dev[i]) (void)hipFree(ctx->wl_dev[i]);
    }
    dfree_t(ctx->unit_wl);
    dfree(ctx->scratch);
    dfree(ctx->io);
    if (ctx->gather_host) (void)hipHostFree(ctx->gather_host);
    ctx->gather_host = nullptr;
    dfree_t(ctx->dev_flag);
    if (ctx->host_flag) (void)hipHostFree(ctx->host_flag);
    ctx->host_flag = nullptr;
    if (ctx->map_flag_host) (void)hipHostFree(ctx->map_flag_host);
    ctx->map_flag_host = ctx->map_flag_dev = nullptr;
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->stream2) (void)hipStreamDestroy(ctx->stream2);
    if (ctx->stream3) (void)hipStreamDestroy(ctx->stream3);
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  delete ctx;
}

int shelfi_ctx_info(const shelfi_ctx* ctx, shelfi_info* o) {
  if (!ctx || !o) return SHELFI_ERR_ARG;
  std::memset(o, 0, sizeof(*o));
  o->ring_dim = ctx->p.N;
  o->num_towers = ctx->p.L;
  o->batch = ctx->p.batch;
  o->scale_bits = ctx->p.scale_bits;
  o->first_mod_bits = ctx->p.first_mod_bits;
  o->device = ctx->device;
  for (uint32_t t = 0; t < ctx->p.L; ++t) {
    o->moduli[t] = ctx->p.q[t];
    o->roots[t] = ctx->p.psi[t];
  }
  o->delta = ctx->p.delta;
  o->key_id = ctx->key_id;
  o->keys_loaded = ctx->keys_loaded ? 1 : 0;
  o->palisade_keys = ctx->palisade_keys ? 1 : 0;
  return SHELFI_OK;
}

int shelfi_set_seed(shelfi_ctx* ctx, uint64_t seed) {
  if (!ctx) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  ctx->seed = seed;
  ctx->enc_counter = 0;
  return SHELFI_OK;
}

int shelfi_set_keys(shelfi_ctx* ctx, const uint64_t* pk, const uint64_t* sk) {
  if (!ctx || !pk || !sk) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    DeviceGuard g(ctx->device);
    install_keys(ctx, pk, sk, false);
  });
}

int shelfi_get_keys(const shelfi_ctx* ctx, uint64_t* pk, uint64_t* sk) {
  if (!ctx) return SHELFI_ERR_ARG;
  if (!ctx->keys_loaded) {
    set_error("no keys loaded");
    return SHELFI_ERR_STATE;
  }
  if (pk) std::memcpy(pk, ctx->pk_host.data(), ctx->pk_host.size() * sizeof(uint64_t));
  if (sk) std::memcpy(sk, ctx->sk_host.data(), ctx->sk_host.size() * sizeof(uint64_t));
  return SHELFI_OK;
}

int shelfi_keygen(shelfi_ctx* ctx, const char* cryptodir) {
  if (!ctx) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    DeviceGuard g(ctx->device);
    const Params& p = ctx->p;
    const size_t LN = (size_t)p.L * p.N;
    uint32_t key[8];
    if (ctx->seed)
      seed_to_key(ctx->seed, key);
    else
      os_random(key, 32);
    void* sk_d = nullptr;
    void* pk_d = nullptr;
    SHELFI_HIP(hipMalloc(&sk_d, LN * 8));
    SHELFI_HIP(hipMalloc(&pk_d, 2 * LN * 8));
    void* scratch = ensure(ctx->scratch, ctx->scratch_bytes, keygen_scratch_bytes(p));
    std::vector<uint64_t> sk(LN), pk(2 * LN);
    try {
      launch_keygen(p, ctx->dt, key, (uint64_t*)sk_d, (uint64_t*)pk_d, scratch, ctx->stream);
      SHELFI_HIP(hipMemcpyAsync(sk.data(), sk_d, LN * 8, hipMemcpyDeviceToHost, ctx->stream));
      SHELFI_HIP(hipMemcpyAsync(pk.data(), pk_d, 2 * LN * 8, hipMemcpyDeviceToHost, ctx->stream));
      SHELFI_HIP(hipStreamSynchronize(ctx->stream));
    } catch (...) {
      (void)hipFree(sk_d);
      (void)hipFree(pk_d);
      throw;
    }
    (void)hipFree(sk_d);
    (void)hipFree(pk_d);
    std::memset(key, 0, sizeof(key));
    install_keys(ctx, pk.data(), sk.data(), true);
    // ckks.cpp:36-56: context first, then public, then private key, in PALISADE 1.11's
    // cereal PortableBinary format (palisade_codec.h), so PALISADE clients can load them
    const PalisadeCtxParams cp = palisade_params_of(ctx->p);
    std::string tag = make_keytag(ctx);
    if (cryptodir && *cryptodir) {
      const std::string dir(cryptodir);
      write_file(dir + "cryptocontext.txt", palisade_context_file(cp));
      write_file(dir + "key-public.txt", palisade_key_file(cp, tag, pk.data(), true));
      write_file(dir + "key-private.txt", palisade_key_file(cp, tag, sk.data(), false));
    }
    ctx->pal_ctx_obj = palisade_context_object(cp, 3);
    ctx->pal_keytag = std::move(tag);
  });
}

int shelfi_load(shelfi_ctx* ctx, const char* cryptodir) {
  if (!ctx || !cryptodir) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    DeviceGuard g(ctx->device);
    const std::string dir(cryptodir);
    const std::string cc = read_file(dir + "cryptocontext.txt");
    if (cc.size() >= 4 && cc.compare(0, 4, "SHCC") == 0) {
      size_t off = 4;
      if (get<uint32_t>(cc, off) != 1) throw Error{SHELFI_ERR_FORMAT, "unsupported context version"};
      const uint32_t N = get<uint32_t>(cc, off), L = get<uint32_t>(cc, off);
      const uint32_t batch = get<uint32_t>(cc, off), sb = get<uint32_t>(cc, off);
      const uint32_t fb = get<uint32_t>(cc, off);
      const double sigma = get<double>(cc, off);
      if (L < 1 || L > (uint32_t)kMaxTowers) throw Error{SHELFI_ERR_FORMAT, "bad tower count"};
      uint64_t q[kMaxTowers], psi[kMaxTowers];
      for (uint32_t t = 0; t < L; ++t) q[t] = get<uint64_t>(cc, off);
      for (uint32_t t = 0; t < L; ++t) psi[t] = get<uint64_t>(cc, off);
      validate_params(N, L, sb, fb, batch);
      free_keys(ctx);
      set_params(ctx, N, L, sb, fb, batch, q, psi);
      ctx->p.sigma = sigma;
      const size_t LN = (size_t)L * N;
      const std::string ps = read_file(dir + "key-public.txt");
      const std::string ss = read_file(dir + "key-private.txt");
      size_t po = 4, so = 4;
      if (ps.compare(0, 4, "SHPK") != 0 || ss.compare(0, 4, "SHSK") != 0)
        throw Error{SHELFI_ERR_FORMAT, "key files do not match the context format"};
      (void)get<uint32_t>(ps, po);
      (void)get<uint32_t>(ss, so);
      if (get<uint64_t>(ps, po) != ctx->params_id || get<uint64_t>(ss, so) != ctx->params_id)
        throw Error{SHELFI_ERR_FORMAT, "key files were generated for a different context"};
      if (ps.size() != po + 2 * LN * 8 || ss.size() != so + LN * 8)
        throw Error{SHELFI_ERR_FORMAT, "key file size mismatch"};
      install_keys(ctx, reinterpret_cast<const uint64_t*>(ps.data() + po),
                   reinterpret_cast<const uint64_t*>(ss.data() + so), false);
    } else {
      // PALISADE 1.11 cereal-binary files (the reference's committed key material)
      PalisadeContext pc = palisade_read_context(cc);
      const uint32_t N = pc.N, L = (uint32_t)pc.q.size();
      const uint32_t batch = std::min<uint32_t>(ctx->p.batch, N / 2);
      // the scaling-factor bits the context was generated with (its plaintext-modulus
      // field), when the file has the layout palisade_codec.h restates
      uint32_t sb = ctx->p.scale_bits;
      try {
        const PalisadeCtxParams cp = palisade_parse_context_file(cc);
        if (cp.plaintext_modulus >= 10 && cp.plaintext_modulus <= 58) sb = (uint32_t)cp.plaintext_modulus;
      } catch (const Error&) {
      }
      const uint32_t fb = std::max(ctx->p.first_mod_bits, sb);
      validate_params(N, L, sb, fb, batch);
      free_keys(ctx);
      set_params(ctx, N, L, sb, fb, batch, pc.q.data(), pc.psi.data());
      std::vector<uint64_t> pk, sk;
      const std::string pub = read_file(dir + "key-public.txt");
      palisade_read_keys(pub, read_file(dir + "key-private.txt"), N, pc.q, pk, sk);
      std::string ctx_obj, keytag;
      palisade_key_context(pub, ctx_obj, keytag);  // for PALISADE-format output (§8 f1)
      install_keys(ctx, pk.data(), sk.data(), true);
      ctx->pal_ctx_obj = std::move(ctx_obj);
      ctx->pal_keytag = std::move(keytag);
      load_evalkey_if_present(ctx, dir);  // §8 f4: a key-eval-mult.txt of these keys
    }
  });
}

static BlobHeader make_header(const shelfi_ctx* ctx, uint64_t K, uint32_t depth, double scale);

// Where the residues of a bytes-API ciphertext batch live in host memory: a library
// blob (one contiguous payload) or a PALISADE archive (2*L tower runs per ciphertext,
// palisade_codec.h).  Both map onto the device layout [K][2][L][N].
// Packed wire payload sizes (version-2 blobs): bytes of one (ct, poly) group of the first Lu towers.
static uint64_t packed_poly_bytes(const Params& p, uint32_t Lu) {
  const ArenaPack ap = arena_pack(p);
  uint64_t u = 0;
  for (uint32_t t = 0; t < Lu; ++t) u += ap.w[t];
  return (uint64_t)(p.N / kArenaChunk) * 64 * u;
}
// The widths of the first Lu towers (the buffers a prefix upload unpacks)
static ArenaPack arena_pack_prefix(const Params& p, uint32_t Lu) {
  Params q = p;
  q.L = Lu;
  return arena_pack(q);
}

struct CtLayout {
  uint8_t* base = nullptr;
  bool pal = false;
  bool packed = false;  // a version-2 (packed) library blob
  int fmt() const { return pal ? 1 : packed ? 2 : 0; }  // shelfi_set_wire_format's numbering
  uint64_t K = 0;
  uint32_t depth = 0;
  uint64_t level = 0;
  double scale = 0.0;
  std::vector<size_t> off;  // PALISADE tower offsets [K][2][L]
  // ciphertexts [k0, k0 + kn) as host pieces in [K][2][L][N] order; with Lu < L only each
  // polynomial's first Lu towers (the decode's prefix, decode_towers): [kn][2][Lu][N]
  void pieces(uint64_t k0, uint64_t kn, const Params& p, std::vector<HostPiece>& out, uint32_t Lu = 0) const {
    out.clear();
    if (!Lu) Lu = p.L;
    const size_t poly_bytes = (size_t)p.L * p.N * 8, ct_bytes = 2 * poly_bytes;
    if (packed) {  // (ct, poly) groups of packed rows; a tower prefix is a prefix of each group
      const uint64_t pg = packed_poly_bytes(p, p.L);
      if (Lu == p.L) {
        out.push_back(HostPiece{base + sizeof(BlobHeader) + k0 * 2 * pg, kn * 2 * pg});
        return;
      }
      const uint64_t pl = packed_poly_bytes(p, Lu);
      for (uint64_t i = 2 * k0; i < 2 * (k0 + kn); ++i)
        out.push_back(HostPiece{base + sizeof(BlobHeader) + i * pg, (size_t)pl});
      return;
    }
    if (!pal) {
      if (Lu == p.L) {
        out.push_back(HostPiece{base + sizeof(BlobHeader) + k0 * ct_bytes, kn * ct_bytes});
        return;
      }
      for (uint64_t i = 2 * k0; i < 2 * (k0 + kn); ++i)
        out.push_back(HostPiece{base + sizeof(BlobHeader) + i * poly_bytes, (size_t)Lu * p.N * 8});
      return;
    }
    for (uint64_t i = 2 * k0; i < 2 * (k0 + kn); ++i)
      for (uint32_t t = 0; t < Lu; ++t) out.push_back(HostPiece{base + off[i * p.L + t], (size_t)p.N * 8});
  }
};

// A caller's ciphertext batch, validated against the context (params and key).
static CtLayout open_cts(const shelfi_ctx* ctx, const uint8_t* b, size_t len) {
  CtLayout v;
  v.base = const_cast<uint8_t*>(b);
  if (b && palisade_looks_like_archive(b, len)) {
    PalisadeArchive A = palisade_parse_archive(b, len);
    v.pal = true;
    v.K = A.K;
    if (A.K) {
      const Params& p = ctx->p;
      bool same = A.N == p.N && A.L == p.L;
      for (uint32_t t = 0; same && t < p.L; ++t) same = A.q[t] == p.q[t];
      if (!same)
        throw Error{SHELFI_ERR_FORMAT, "PALISADE ciphertexts were produced under different crypto parameters"};
      if (ctx->pal_keytag.empty() || A.keytag != ctx->pal_keytag)
        throw Error{SHELFI_ERR_FORMAT, "PALISADE ciphertexts were encrypted under a different key (keyTag)"};
      if (A.encoding != 4) throw Error{SHELFI_ERR_FORMAT, "PALISADE ciphertexts are not CKKS-packed"};
    }
    v.depth = (uint32_t)A.depth;
    v.level = A.level;
    v.scale = A.scale;
    v.off = std::move(A.tower_off);
    return v;
  }
  BlobHeader h = parse_blob(b, len, ctx);
  v.packed = h.version == 2;
  v.K = h.K;
  v.depth = h.depth;
  v.level = h.level;
  v.scale = h.scale;
  if (v.K && h.key_id != ctx->key_id)
    throw Error{SHELFI_ERR_FORMAT, "ciphertext was encrypted under a different key"};
  return v;
}

// Size of (and, with buf, the header / framing of) an output batch in the ctx's
// format; returns its layout.
static CtLayout make_output(const shelfi_ctx* ctx, int fmt, uint64_t K, uint32_t depth,
                            uint64_t level, double scale, uint8_t* buf, size_t* total) {
  const bool pal = fmt == 1;
  CtLayout v;
  v.base = buf;
  v.pal = pal;
  v.packed = fmt == 2;
  v.K = K;
  v.depth = depth;
  v.level = level;
  v.scale = scale;
  const Params& p = ctx->p;
  if (pal) {
    if (ctx->pal_ctx_obj.empty())
      throw Error{SHELFI_ERR_STATE, "PALISADE wire format needs keys loaded from PALISADE files"};
    // key_params: what the reference writes (its keys always come from key-public.txt)
    v.off = palisade_layout(ctx->pal_ctx_obj, ctx->pal_keytag, p.N, p.L, p.q, K, depth, level, scale,
                            4, true, true, buf, total);
    return v;
  }
  *total = sizeof(BlobHeader) + K * (v.packed ? 2 * packed_poly_bytes(p, p.L) : 2ull * p.L * p.N * 8);
  if (buf) {
    BlobHeader h = make_header(ctx, K, depth, scale);
    if (v.packed) h.version = 2;
    std::memcpy(buf, &h, sizeof(h));
  }
  return v;
}

// ------------------------------------------------------------- bytes API ----
static BlobHeader make_header(const shelfi_ctx* ctx, uint64_t K, uint32_t depth, double scale) {
  const Params& p = ctx->p;
  BlobHeader h;
  std::memset(&h, 0, sizeof(h));
  std::memcpy(h.magic, "SHCT", 4);
  h.version = 1;
  h.header_bytes = 64;
  h.logN = p.logN;
  h.L = p.L;
  h.K = K;
  h.depth = depth;
  h.level = 0;
  h.scale = scale;
  h.params_id = ctx->params_id;
  h.key_id = ctx->key_id;
  h.batch = p.batch;
  h.encoding = 4;
  return h;
}

// Three-stage pipeline over chunks: H2D on stream A, kernels on stream B (scratch is
// reused chunk after chunk on B), D2H on stream C, two staging buffer sets.
struct Pipe {
  hipStream_t a, b, c;
  hipEvent_t in_ready[2], computed[2], out_free[2];
  explicit Pipe(shelfi_ctx* ctx) : a(ctx->stream), b(ctx->stream2), c(ctx->stream3) {
    for (int i = 0; i < 2; ++i) {
      in_ready[i] = computed[i] = out_free[i] = nullptr;
    }
    for (int i = 0; i < 2; ++i) {
      SHELFI_HIP(hipEventCreateWithFlags(&in_ready[i], hipEventDisableTiming));
      SHELFI_HIP(hipEventCreateWithFlags(&computed[i], hipEventDisableTiming));
      SHELFI_HIP(hipEventCreateWithFlags(&out_free[i], hipEventDisableTiming));
    }
  }
  ~Pipe() {
    (void)hipStreamSynchronize(c);  // no-ops on success; on an error, nothing stays in flight
    (void)hipStreamSynchronize(b);
    (void)hipStreamSynchronize(a);
    for (int i = 0; i < 2; ++i) {
      if (in_ready[i]) (void)hipEventDestroy(in_ready[i]);
      if (computed[i]) (void)hipEventDestroy(computed[i]);
      if (out_free[i]) (void)hipEventDestroy(out_free[i]);
    }
  }
  void sync() {
    SHELFI_HIP(hipStreamSynchronize(c));
    SHELFI_HIP(hipStreamSynchronize(b));
    SHELFI_HIP(hipStreamSynchronize(a));
  }
};

// The ctx's pinned staging rings (8 slots each way, SHELFI_STAGE_SLOT_MIB each), created on first use
// and re-created between calls when the slot size switch changes (the ring is idle then).  16 MiB: a
// bytes-API learner chunk (4 cts, 8 MiB + its archive headers) is one DMA; pinned copies of 8 / 16 / 32
// MiB ran 53.5 / 55.4 / 56.3 GB/s (profiles/r05u/pinned_h2d.json) and the archive aggregation 45.1 -> 48.4
// GB/s with 16 MiB slots, the other bytes-API rates within noise (profiles/r05u/bench_slot*).
static Stager& stager(shelfi_ctx* ctx) {
  const size_t slot = (size_t)switches().stage_slot_mib << 20;
  if (ctx->stage && ctx->stage->slot_bytes() != slot) {
    delete ctx->stage;
    ctx->stage = nullptr;
  }
  if (!ctx->stage) ctx->stage = new Stager(slot, 8, 8, default_copy_threads());
  return *ctx->stage;
}

// Drops the staged outputs of a pipeline that threw (declared after its Pipe, so the
// slots are abandoned before the streams are drained).
struct StageRun {
  Stager& s;
  bool done = false;
  explicit StageRun(Stager& st) : s(st) { s.begin(); }
  void finish() {
    s.finish();
    done = true;
  }
  ~StageRun() {
    if (!done) s.abort();
  }
};

// A call's generation of the GenFlag words (shelfi_internal.h).  Every caller synchronises before the next
// call starts, so no kernel writes the words while the host clears them at a wrap of the counter.
static GenFlag next_gen_flag(shelfi_ctx* ctx) {
  if (++ctx->map_gen == 0) {
    std::memset(ctx->map_flag_host, 0, 64);
    ctx->map_gen = 1;
  }
  return GenFlag{ctx->map_flag_dev, ctx->map_gen};
}
// after the call's synchronisation: did it raise word w?
static bool gen_flag_raised(const shelfi_ctx* ctx, const GenFlag& f, int w) {
  return __atomic_load_n(ctx->map_flag_host + w, __ATOMIC_ACQUIRE) == f.gen;
}

// The encode range flag of an encrypt call (kernels.hip enc_range_flag): non-finite values are refused;
// a finite |x Delta| above 2^61 means the call is redone on the large-value path.
static bool encode_needs_approx(const shelfi_ctx* ctx, const GenFlag& f) {
  if (gen_flag_raised(ctx, f, 1)) throw Error{SHELFI_ERR_RANGE, "encrypt: non-finite input value"};
  return gen_flag_raised(ctx, f, 0);
}

// encode + encrypt n doubles (host) -> K ciphertext payloads written to out_payload (approx: every
// chunk on the large-value path, launch_encrypt_approx; same key and counters, so the same samples).
static void encrypt_bytes_pipeline(shelfi_ctx* ctx, const double* x, size_t n, uint64_t K,
                                   const CtLayout& dst, const uint32_t key[8], uint64_t g0, bool approx) {
  const Params& p = ctx->p;
  const size_t ct_bytes = 2ull * p.L * p.N * 8;
  uint64_t kc = std::max<uint64_t>(1, (64ull << 20) / ct_bytes);
  kc = std::min<uint64_t>(kc, K);
  const size_t xin = kc * p.batch * 8, cto = kc * ct_bytes;
  // packed wire output: the chunk is packed on the device (U_t bits per residue) before its D2H
  const size_t pko = dst.packed ? kc * 2 * packed_poly_bytes(p, p.L) : 0;
  uint8_t* io = (uint8_t*)ensure(ctx->io, ctx->io_bytes, 2 * (xin + cto + pko));
  uint8_t* xb[2] = {io, io + xin};
  uint8_t* cb[2] = {io + 2 * xin, io + 2 * xin + cto};
  uint8_t* pb[2] = {io + 2 * (xin + cto), io + 2 * (xin + cto) + pko};
  const ArenaPack ap = arena_pack(p);
  void* scratch = ensure(ctx->scratch, ctx->scratch_bytes, encrypt_scratch_bytes(p, kc));
  Pipe pp(ctx);
  StageRun sr(stager(ctx));
  std::vector<HostPiece> pcs;
  const GenFlag fl = next_gen_flag(ctx);
  const uint64_t nchunks = (K + kc - 1) / kc;
  for (uint64_t ci = 0; ci < nchunks; ++ci) {
    const int b = (int)(ci & 1);
    const uint64_t k0 = ci * kc, kn = std::min<uint64_t>(kc, K - k0);
    const uint64_t xs = k0 * p.batch, xn = std::min<uint64_t>(n - xs, kn * p.batch);
    if (ci >= 2) SHELFI_HIP(hipStreamWaitEvent(pp.a, pp.computed[b], 0));  // x buffer consumed
    sr.s.h2d(xb[b], x + xs, xn * 8, pp.a);
    SHELFI_HIP(hipEventRecord(pp.in_ready[b], pp.a));
    SHELFI_HIP(hipStreamWaitEvent(pp.b, pp.in_ready[b], 0));
    if (ci >= 2) SHELFI_HIP(hipStreamWaitEvent(pp.b, pp.out_free[b], 0));  // ct buffer drained
    if (approx)
      launch_encrypt_approx(p, ctx->dt, ctx->dk, (const double*)xb[b], xn, kn, (uint64_t*)cb[b], scratch, key,
                            g0 + k0, pp.b);
    else
      launch_encrypt(p, ctx->dt, ctx->dk, (const double*)xb[b], xn, kn, (uint64_t*)cb[b], scratch, key,
                     g0 + k0, fl, pp.b);
    if (dst.packed)  // canonical residues: the residue check cannot fire
      launch_blob_pack((const uint64_t*)cb[b], kn, p.L, p.logN, ap, ctx->dt.tc, (uint32_t*)pb[b],
                       ctx->dev_flag + 5, pp.b);
    SHELFI_HIP(hipEventRecord(pp.computed[b], pp.b));
    SHELFI_HIP(hipStreamWaitEvent(pp.c, pp.computed[b], 0));
    dst.pieces(k0, kn, p, pcs);
    sr.s.d2hv(pcs.data(), pcs.size(), dst.packed ? pb[b] : cb[b], pp.c);
    SHELFI_HIP(hipEventRecord(pp.out_free[b], pp.c));
    sr.s.poll();
  }
  sr.finish();
  pp.sync();
  if (!approx && encode_needs_approx(ctx, fl))
    encrypt_bytes_pipeline(ctx, x, n, K, dst, key, g0, true);
}

int shelfi_encrypt_into(shelfi_ctx* ctx, const double* x, size_t n, uint8_t* out, size_t out_cap,
                        size_t* out_len) {
  if (!ctx || !out_len || (n && !x)) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    require_keys(ctx);
    DeviceGuard g(ctx->device);
    const Params& p = ctx->p;
    const uint64_t K = (n + p.batch - 1) / p.batch;  // ckks.cpp:65
    size_t total = 0;
    make_output(ctx, ctx->wire, K, 1, 0, p.delta, nullptr, &total);
    *out_len = total;
    if (!out) return;
    if (out_cap < total) throw Error{SHELFI_ERR_ARG, "output buffer too small"};
    advise_huge(out, total);
    // residues first (the parallel drains first-touch the fresh pages), framing after
    CtLayout dst = make_output(ctx, ctx->wire, K, 1, 0, p.delta, nullptr, &total);
    dst.base = out;
    if (K) {
      uint32_t key[8];
      uint64_t g0;
      draw_key(ctx, K, key, &g0);
      try {
        encrypt_bytes_pipeline(ctx, x, n, K, dst, key, g0, false);
      } catch (...) {
        std::memset(key, 0, sizeof(key));
        throw;
      }
      std::memset(key, 0, sizeof(key));
    }
    make_output(ctx, ctx->wire, K, 1, 0, p.delta, out, &total);
  });
}

int shelfi_encrypt(shelfi_ctx* ctx, const double* x, size_t n, uint8_t** out, size_t* out_len) {
  if (!ctx || !out || !out_len || (n && !x)) return SHELFI_ERR_ARG;
  *out = nullptr;
  size_t total = 0;
  int rc = shelfi_encrypt_into(ctx, x, n, nullptr, 0, &total);
  if (rc) return rc;
  uint8_t* blob = (uint8_t*)std::malloc(total ? total : 1);
  if (!blob) {
    set_error("host out of memory");
    return SHELFI_ERR_DEVICE;
  }
  rc = shelfi_encrypt_into(ctx, x, n, blob, total, &total);
  if (rc) {
    std::free(blob);
    return rc;
  }
  *out = blob;
  *out_len = total;
  return SHELFI_OK;
}

// Validates the learners' blobs (same params, key, K, depth, scale) and returns the
// header of the result (depth + 1, scale * Delta: EvalMult by a constant, no rescale).
// Validates the learners' batches (same format, params, key, K, depth, scale).
static std::vector<CtLayout> wavg_inputs(const shelfi_ctx* ctx, const uint8_t* const* blobs,
                                         const size_t* lens, size_t C) {
  if (C == 0) throw Error{SHELFI_ERR_ARG, "computeWeightedAverage: no learners"};
  std::vector<CtLayout> in;
  in.reserve(C);
  for (size_t c = 0; c < C; ++c) {
    in.push_back(open_cts(ctx, blobs[c], lens[c]));
    const CtLayout& h = in.back();
    const CtLayout& h0 = in.front();
    if (h.pal != h0.pal)
      throw Error{SHELFI_ERR_FORMAT, "learners mix PALISADE archives and library blobs"};
    if (h.packed != h0.packed)
      throw Error{SHELFI_ERR_FORMAT, "learners mix packed and uint64 library blobs"};
    if (h.K != h0.K)
      throw Error{SHELFI_ERR_FORMAT, "learners hold different numbers of ciphertexts"};
    if (h.depth != h0.depth || h.scale != h0.scale || h.level != h0.level)
      throw Error{SHELFI_ERR_FORMAT, "learners' ciphertexts have different depth/scale"};
  }
  return in;
}

// Pipelined bytes -> bytes aggregation: the K ciphertexts are processed in chunks;
// chunk i's H2D copies (all learners, stream A) overlap chunk i-1's wavg + D2H
// (stream B), with two device buffer sets.  Writes the payload of the result.
// Uploads (round 5): each learner's chunk is one contiguous byte range of its blob -- a PALISADE
// archive's range (tower headers included) lands raw and its tower runs are gathered into [K][2][L][N]
// on the device.  By default the range goes through the pinned staging ring (pool threads memcpy it
// into 16 MiB pinned slots that are DMA'd); SHELFI_H2D_DIRECT=1 copies it straight from the caller's
// pageable memory instead, which is faster only on blobs the runtime has already pinned: on fresh blobs
// (every aggregation round's uploads) the runtime pins their pages on each first copy.  16 x 64 cts of
// archives, input GB/s fresh malloc'd / fresh encrypt outputs / warm: ring 48.2 / 48.9 / 48.5
// (profiles/r05u/slot_size.json, 16 MiB), direct 18.7 / 34.4 / 53.7 (taper_palisade.json).  The sum's D2H lands
// in a pinned buffer that the AsyncDrain worker scatters into the output, so the uploading thread never
// stops to drain.  (Zero-copy uploads registered in place with hipHostRegister measured slower than
// the ring and were removed in round 5: tools/h2d_register_ab.py.)
static void wavg_bytes_pipeline(shelfi_ctx* ctx, const std::vector<CtLayout>& in,
                                const float* weights, size_t C, uint64_t K, const CtLayout& dst,
                                const size_t* lens) {
  const Params& p = ctx->p;
  const size_t ct_bytes = 2ull * p.L * p.N * 8;
  const bool direct = switches().h2d_direct;
  // learners per wavg launch: all of them, up to kWavgMaxLearners (more: accumulated groups).  Cutting a
  // single-chunk call (cfg2's 16 x 4 cts) into 2 / 4 / 8 groups to overlap uploads with the device work
  // measured the same as one group once a step's learners share the ring's slots (profiles/r05ct)
  const size_t group = std::min<size_t>(C, kWavgMaxLearners);
  // chunk of input per learner-group buffer: direct uploads want ~32 MiB per copy (8 MiB copies ran
  // 51.6 GB/s, 2 MiB 41.3, 32 MiB 55.6, on pinned-warm blobs), so 32 MiB per learner; through the ring
  // ~128 MiB per group (round 4: 32 / 64 / 128 / 256 MiB ran 60.4 / 52.4 / 48.2 / 48.7 ms for 16 learners x
  // 64 cts, profiles/r04w/api_chunk.txt); SHELFI_WAVG_CHUNK_MIB overrides (A/B probe switch)
  const uint64_t chunk_mib = switches().wavg_chunk_mib ? switches().wavg_chunk_mib : direct ? 32 * group : 128;
  uint64_t kc = std::max<uint64_t>(1, (chunk_mib << 20) / (ct_bytes * group));
  // at least ~4 chunks through the ring, so a small call's gather + wavg + D2H overlap its later uploads: cfg2's
  // 16 x 4 cts in 4 chunks ran 41.0 / 44.4 / 42.8 GB/s (fresh copies / fresh encrypt outputs / warm) vs 39.0 /
  // 41.8 / 40.5 in one (profiles/r05cy)
  if (!direct && !switches().wavg_chunk_mib) kc = std::min<uint64_t>(kc, std::max<uint64_t>(1, (K + 3) / 4));
  // packed wire (version-2 blobs): uploads land packed and are unpacked on the device; a packed
  // output is packed before its D2H
  const uint64_t pct = 2 * packed_poly_bytes(p, p.L);
  const bool pin = in.front().packed, pout = dst.packed;
  const bool raw = in.front().pal;  // archives: raw ranges, gathered on the device
  kc = std::min<uint64_t>(kc, K);
  const size_t in_chunk = group * kc * ct_bytes, out_chunk = kc * ct_bytes;
  const size_t pin_chunk = pin ? group * kc * pct : 0, pout_chunk = pout ? kc * pct : 0;
  const uint64_t nchunks = (K + kc - 1) / kc;
  std::vector<HostPiece> pcs;
  // raw ranges: a step's (chunk, learner group) learners' byte ranges (tower headers included) land back to
  // back in its raw buffer, so the ring packs them into full slots (one DMA per slot, not per learner: each
  // DMA costs ~17 us of gap on the copy engine, profiles/r05cp); the whole call's gather table -- every
  // step's run offsets into its raw buffer -- is written once into pinned memory and uploaded by one copy
  // ahead of the data (no per-step table copies or host waits)
  size_t raw_cap = 0, runs_total = 0;  // raw_cap: the largest step's bytes
  std::vector<size_t> step_run0;       // step -> its first table entry
  if (raw) {
    for (uint64_t ci = 0; ci < nchunks; ++ci) {
      const uint64_t k0 = ci * kc, kn = std::min<uint64_t>(kc, K - k0);
      for (size_t c0 = 0; c0 < C; c0 += group) {
        size_t bytes = 0;
        for (size_t c = c0; c < std::min(C, c0 + group); ++c) {
          in[c].pieces(k0, kn, p, pcs);
          bytes += (size_t)(pcs.back().p + pcs.back().n - pcs.front().p);
          runs_total += pcs.size();
        }
        raw_cap = std::max(raw_cap, bytes);
      }
    }
    raw_cap = (raw_cap + 64 + 255) & ~(size_t)255;  // + the gather's read-ahead of one dword
    if (ctx->gather_cap < runs_total) {
      if (ctx->gather_host) SHELFI_HIP(hipHostFree(ctx->gather_host));
      ctx->gather_host = nullptr;
      ctx->gather_cap = 0;
      SHELFI_HIP(hipHostMalloc((void**)&ctx->gather_host, runs_total * 8, hipHostMallocDefault));
      ctx->gather_cap = runs_total;
    }
    size_t r = 0;
    for (uint64_t ci = 0; ci < nchunks; ++ci) {
      const uint64_t k0 = ci * kc, kn = std::min<uint64_t>(kc, K - k0);
      for (size_t c0 = 0; c0 < C; c0 += group) {
        step_run0.push_back(r);
        size_t off = 0;
        for (size_t c = c0; c < std::min(C, c0 + group); ++c) {
          in[c].pieces(k0, kn, p, pcs);
          const uint8_t* lo = pcs.front().p;
          for (const HostPiece& h : pcs) ctx->gather_host[r++] = (uint64_t)(off + (size_t)(h.p - lo));
          off += (size_t)(pcs.back().p + pcs.back().n - lo);
        }
      }
    }
    step_run0.push_back(r);
  }
  const size_t raw_chunk = raw ? raw_cap : 0, tab_bytes = (runs_total * 8 + 255) & ~(size_t)255;
  uint8_t* io = (uint8_t*)ensure(ctx->io, ctx->io_bytes,
                                 2 * (in_chunk + out_chunk + pin_chunk + pout_chunk + raw_chunk) + tab_bytes);
  uint8_t* inb[2] = {io, io + in_chunk};
  uint8_t* outb[2] = {io + 2 * in_chunk, io + 2 * in_chunk + out_chunk};
  uint8_t* const pbase = io + 2 * (in_chunk + out_chunk);
  uint8_t* pinb[2] = {pbase, pbase + pin_chunk};
  uint8_t* poutb[2] = {pbase + 2 * pin_chunk, pbase + 2 * pin_chunk + pout_chunk};
  uint8_t* const rbase = pbase + 2 * (pin_chunk + pout_chunk);
  uint8_t* rawb[2] = {rbase, rbase + raw_chunk};
  uint64_t* const tabd = (uint64_t*)(rbase + 2 * raw_chunk);
  const ArenaPack ap = arena_pack(p);
  // A: H2D of the learners' slices; B: wavg; C: staged D2H of the sum
  Pipe pp(ctx);
  StageRun sr(stager(ctx));
  if (!ctx->drain) ctx->drain = new AsyncDrain(default_copy_threads());
  const bool two = direct && switches().h2d_two && C > 1;
  if (two && !ctx->up2) {
    if (!ctx->stream4) SHELFI_HIP(hipStreamCreateWithFlags(&ctx->stream4, hipStreamNonBlocking));
    ctx->up2 = new AsyncUpload();
  }
  hipEvent_t up2_done[2] = {nullptr, nullptr};
  struct EvGuard {
    hipEvent_t* e;
    ~EvGuard() {
      for (int i = 0; i < 2; ++i)
        if (e[i]) (void)hipEventDestroy(e[i]);
    }
  } eg{up2_done};
  if (two)
    for (int i = 0; i < 2; ++i) SHELFI_HIP(hipEventCreateWithFlags(&up2_done[i], hipEventDisableTiming));
  struct UpGuard {  // on an error: the second thread's posted copies are issued and done before we unwind
    shelfi_ctx* c;
    bool armed;
    ~UpGuard() {
      if (!armed) return;
      try {
        c->up2->wait();
      } catch (...) {
      }
      (void)hipStreamSynchronize(c->stream4);
    }
  } ug{ctx, two};
  struct DrainGuard {  // on an error: the worker finishes what was posted before the streams go away
    AsyncDrain* d;
    bool armed;
    ~DrainGuard() {
      if (armed && d) try {
          d->finish();
        } catch (...) {
        }
    }
  } dg{ctx->drain, true};
  {  // the output's residue pages, first-touched on the drain worker during the uploads
    dst.pieces(0, K, p, pcs);
    const uint8_t* lo = pcs.front().p;
    ctx->drain->prefault(const_cast<uint8_t*>(lo), (size_t)(pcs.back().p + pcs.back().n - lo));
  }
  uint32_t* bad = ctx->dev_flag + 3;  // an upload residue >= q (the kernels assume canonical inputs)
  SHELFI_HIP(hipMemsetAsync(bad, 0, 4, pp.b));
  if (raw) SHELFI_HIP(hipMemcpyAsync(tabd, ctx->gather_host, runs_total * 8, hipMemcpyHostToDevice, pp.a));
  using clk = std::chrono::steady_clock;
  const bool trace = sr.s.trace();
  const auto t_start = clk::now();
  double t_up = 0.0;  // SHELFI_STAGE_TRACE: host seconds in the uploads
  // input buffers alternate by step (a learner group of a chunk), the sum's buffers by chunk
  uint64_t st = 0;
  std::vector<HostPiece> grp;  // a step's host pieces, in landing order
  for (uint64_t ci = 0; ci < nchunks; ++ci) {
    const int b = (int)(ci & 1);
    const uint64_t k0 = ci * kc, kn = std::min<uint64_t>(kc, K - k0);
    for (size_t c0 = 0; c0 < C; c0 += group) {
      const size_t gc = std::min(group, C - c0);
      const int bi = (int)(st & 1);
      if (st >= 2) {  // buffer free
        SHELFI_HIP(hipStreamWaitEvent(pp.a, pp.computed[bi], 0));
        if (two) SHELFI_HIP(hipStreamWaitEvent(ctx->stream4, pp.computed[bi], 0));
      }
      // where the uploads land: the learners' uint64 slots, or their packed staging (then unpacked), or
      // (archives) their raw ranges back to back, gathered below -- contiguous in every case, so through
      // the ring the whole group is one gather of pieces
      uint8_t* const land0 = raw ? rawb[bi] : pin ? pinb[bi] : inb[bi];
      size_t off = 0;
      grp.clear();
      for (size_t c = 0; c < gc; ++c) {
        in[c0 + c].pieces(k0, kn, p, pcs);
        const uint8_t* lo = pcs.front().p;
        const size_t span = (size_t)(pcs.back().p + pcs.back().n - lo);
        if (direct) {  // one pageable copy of the learner's whole range
          uint8_t* land = land0 + (raw ? off : c * kn * (pin ? pct : ct_bytes));
          const auto t0 = clk::now();
          if (two && (c & 1))  // every other learner from the second thread: two copies in flight
            ctx->up2->post(land, lo, span, ctx->stream4);
          else
            SHELFI_HIP(hipMemcpyAsync(land, lo, span, hipMemcpyHostToDevice, pp.a));
          if (trace) t_up += std::chrono::duration<double>(clk::now() - t0).count();
        } else if (raw) {
          grp.push_back(HostPiece{const_cast<uint8_t*>(lo), span});
        } else {
          grp.insert(grp.end(), pcs.begin(), pcs.end());
        }
        off += span;
      }
      if (!direct) {
        const auto t0 = clk::now();
        sr.s.h2dv(land0, grp.data(), grp.size(), pp.a);
        if (trace) t_up += std::chrono::duration<double>(clk::now() - t0).count();
      }
      if (two) {  // the second thread's copies of this chunk join stream A
        ctx->up2->wait();
        SHELFI_HIP(hipEventRecord(up2_done[bi], ctx->stream4));
        SHELFI_HIP(hipStreamWaitEvent(pp.a, up2_done[bi], 0));
      }
      SHELFI_HIP(hipEventRecord(pp.in_ready[bi], pp.a));
      SHELFI_HIP(hipStreamWaitEvent(pp.b, pp.in_ready[bi], 0));
      if (raw)
        launch_gather_runs(rawb[bi], tabd + step_run0[st], step_run0[st + 1] - step_run0[st], (uint32_t)(p.N * 8),
                           inb[bi], pp.b);
      if (pin)  // unpacked on the compute stream, so the upload stream moves on to the next chunk
        for (size_t c = 0; c < gc; ++c)
          launch_blob_unpack((const uint32_t*)(pinb[bi] + c * kn * pct), kn, p.L, p.logN, ap,
                             (uint64_t*)(inb[bi] + c * kn * ct_bytes), pp.b);
      if (ci >= 2 && c0 == 0) SHELFI_HIP(hipStreamWaitEvent(pp.b, pp.out_free[b], 0));
      WavgArgs a;
      std::memset(&a, 0, sizeof(a));
      for (size_t c = 0; c < gc; ++c) a.ptrs[c] = (const uint64_t*)(inb[bi] + c * kn * ct_bytes);
      fill_weights(a, p, weights + c0, gc);
      a.out = (uint64_t*)outb[b];
      a.rows = kn * 2 * p.L;
      a.C = (uint32_t)gc;
      a.L = p.L;
      a.logN = p.logN;
      a.accumulate = c0 ? 1 : 0;
      a.bad = bad;
      launch_wavg(a, ctx->dt.tc, pp.b);
      SHELFI_HIP(hipEventRecord(pp.computed[bi], pp.b));
      ++st;
      if (c0 + gc >= C) {
        if (pout) {  // the sum is canonical: the residue check cannot fire
          launch_blob_pack((const uint64_t*)outb[b], kn, p.L, p.logN, ap, ctx->dt.tc, (uint32_t*)poutb[b],
                           ctx->dev_flag + 5, pp.b);
          SHELFI_HIP(hipEventRecord(pp.computed[bi], pp.b));
        }
        // the last chunk's D2H follows its wavg on the compute stream (nothing is left to overlap, and the
        // cross-stream event cost ~0.1 ms before it: profiles/r05cp)
        const hipStream_t ds = ci + 1 == nchunks ? pp.b : pp.c;
        if (ds == pp.c) SHELFI_HIP(hipStreamWaitEvent(pp.c, pp.computed[bi], 0));
        dst.pieces(k0, kn, p, pcs);
        const uint8_t* sum = pout ? poutb[b] : outb[b];
        // one DMA into the drain's pinned buffer; its worker scatters it to the pieces
        size_t nbytes = 0;
        for (const HostPiece& h : pcs) nbytes += h.n;
        uint8_t* hb = ctx->drain->buffer(b, nbytes);  // waits until chunk ci - 2 is drained
        SHELFI_HIP(hipMemcpyAsync(hb, sum, nbytes, hipMemcpyDeviceToHost, ds));
        SHELFI_HIP(hipEventRecord(pp.out_free[b], ds));
        ctx->drain->post(b, pp.out_free[b], pcs);
      }
    }
  }
  SHELFI_HIP(hipMemcpyAsync(ctx->host_flag + 3, bad, 4, hipMemcpyDeviceToHost, pp.b));  // pinned: no sync copy
  const auto t_issued = clk::now();
  ctx->drain->finish();
  sr.finish();
  pp.sync();
  if (trace)
    std::fprintf(stderr, "[wavg-bytes] %s%s chunks %llu x %llu cts, %llu learners per group: issue %.2f ms "
                 "(uploads %.2f), tail %.2f ms\n", direct ? "direct" : "ring", raw ? "+gather" : "",
                 (unsigned long long)nchunks, (unsigned long long)kc, (unsigned long long)group,
                 std::chrono::duration<double>(t_issued - t_start).count() * 1e3, t_up * 1e3,
                 std::chrono::duration<double>(clk::now() - t_issued).count() * 1e3);
  if (ctx->host_flag[3])  // read back on pp.b before the sync above
    throw Error{SHELFI_ERR_FORMAT, "ciphertext residue >= its tower modulus (malformed learner data)"};
}

int shelfi_weighted_average_into(shelfi_ctx* ctx, const uint8_t* const* blobs, const size_t* lens,
                                 const float* weights, size_t C, uint8_t* out, size_t out_cap,
                                 size_t* out_len) {
  if (!ctx || !out_len || (C && (!blobs || !lens || !weights))) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    if (C == 0) {
      // ckks.cpp:270-309: with no learners the loop never runs and the empty
      // vector<Ciphertext> is serialized; here an empty batch in the ctx's wire format
      // (depth 2 / scale Delta^2: what a weighted average of fresh ciphertexts carries)
      const int fmt = ctx->wire;
      const double scale = ctx->p.delta * ctx->p.delta;
      size_t total = 0;
      make_output(ctx, fmt, 0, 2, 0, scale, nullptr, &total);
      *out_len = total;
      if (!out) return;
      if (out_cap < total) throw Error{SHELFI_ERR_ARG, "output buffer too small"};
      make_output(ctx, fmt, 0, 2, 0, scale, out, &total);
      return;
    }
    using clk = std::chrono::steady_clock;
    const auto t_in = clk::now();
    check_weights(weights, C, ctx->p.delta);
    DeviceGuard g(ctx->device);
    const std::vector<CtLayout> in = wavg_inputs(ctx, blobs, lens, C);
    const auto t_parsed = clk::now();
    const CtLayout& h0 = in.front();
    // EvalMult by a constant (ckks.cpp:288): depth + 1, scale * Delta, same level
    const uint32_t depth = h0.depth + 1;
    const double scale = h0.scale * ctx->p.delta;
    size_t total = 0;
    make_output(ctx, h0.fmt(), h0.K, depth, h0.level, scale, nullptr, &total);
    *out_len = total;
    if (!out) return;  // size query
    if (out_cap < total) throw Error{SHELFI_ERR_ARG, "output buffer too small"};
    advise_huge(out, total);
    // residues first (the parallel drains first-touch the fresh pages), framing after
    CtLayout dst = make_output(ctx, h0.fmt(), h0.K, depth, h0.level, scale, nullptr, &total);
    dst.base = out;
    const auto t_pipe = clk::now();
    if (h0.K) wavg_bytes_pipeline(ctx, in, weights, C, h0.K, dst, lens);
    const auto t_done = clk::now();
    make_output(ctx, h0.fmt(), h0.K, depth, h0.level, scale, out, &total);
    if (switches().stage_trace) {
      const auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count() * 1e3; };
      std::fprintf(stderr, "[wavg-call] parse %.3f ms, setup %.3f, pipeline %.3f, framing %.3f, total %.3f\n",
                   ms(t_in, t_parsed), ms(t_parsed, t_pipe), ms(t_pipe, t_done), ms(t_done, clk::now()),
                   ms(t_in, clk::now()));
    }
  });
}

int shelfi_weighted_average(shelfi_ctx* ctx, const uint8_t* const* blobs, const size_t* lens,
                            const float* weights, size_t C, uint8_t** out, size_t* out_len) {
  if (!ctx || !out || !out_len || (C && (!blobs || !lens || !weights))) return SHELFI_ERR_ARG;
  *out = nullptr;
  *out_len = 0;
  size_t total = 0;
  int rc = shelfi_weighted_average_into(ctx, blobs, lens, weights, C, nullptr, 0, &total);
  if (rc) return rc;
  uint8_t* buf = (uint8_t*)std::malloc(total ? total : 1);
  if (!buf) {
    set_error("host out of memory");
    return SHELFI_ERR_DEVICE;
  }
  rc = shelfi_weighted_average_into(ctx, blobs, lens, weights, C, buf, total, &total);
  if (rc) {
    std::free(buf);
    return rc;
  }
  *out = buf;
  *out_len = total;
  return SHELFI_OK;
}

// Noise-flooding setup for one decrypt of K ciphertexts (enabled by
// shelfi_set_decode_noise); its randomness comes from the ctx stream like encrypt's.
static DecodeNoise decode_noise_begin(shelfi_ctx* ctx, uint64_t K, const GenFlag& fl) {
  DecodeNoise dn;
  if (!ctx->decode_noise) return dn;
  dn.fail = fl;
  dn.enabled = 1;
  dn.m_factor = ctx->decode_m_factor;
  dn.p_bits = ctx->p.scale_bits;
  draw_key(ctx, K, dn.key, &dn.g0);
  dn.flags = ctx->dev_flag;
  // flag [2] (logError) is reset by the first chunk's flooding (launch_decrypt: inside
  // decode_stats_kernel, or a fill before the small-ring decode_flood_kernel)
  return dn;
}

// After a flooded decrypt was enqueued: its logError (device flag [2]) is read back only when asked for
// (shelfi_decode_log_error), not after every call; the precision failure is a GenFlag word (round 6).
static void decode_noise_readback(shelfi_ctx* ctx, const DecodeNoise& dn, hipStream_t) {
  if (dn.enabled) ctx->log_error_pending = true;
}

// After the decrypt's stream work has completed: record logError, raise PALISADE's
// precision failure (Decode throws math_error when log2 sigma > p - 5).
static void decode_noise_end(shelfi_ctx* ctx, DecodeNoise& dn) {
  if (!dn.enabled) return;
  std::memset(dn.key, 0, sizeof(dn.key));
  if (gen_flag_raised(ctx, dn.fail, 3))
    throw Error{SHELFI_ERR_PRECISION,
                "The decryption failed because the approximation error is too high. Check the "
                "parameters."};
}

int shelfi_set_decode_noise(shelfi_ctx* ctx, int enabled, double m_factor) {
  if (!ctx || !(m_factor >= 0.0) || !std::isfinite(m_factor)) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  ctx->decode_noise = enabled ? 1 : 0;
  ctx->decode_m_factor = m_factor;
  return SHELFI_OK;
}

int shelfi_set_decode_exact(shelfi_ctx* ctx, int exact) {
  if (!ctx) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  ctx->decode_exact = exact ? 1 : 0;
  return SHELFI_OK;
}

int shelfi_decode_log_error(shelfi_ctx* ctx, int* log_error) {
  if (!ctx || !log_error) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    if (ctx->log_error_pending) {  // the last flooded decrypt's, read now (every call has synchronised)
      DeviceGuard g(ctx->device);
      SHELFI_HIP(hipMemcpy(ctx->host_flag + 2, ctx->dev_flag + 2, 4, hipMemcpyDeviceToHost));
      ctx->last_log_error = (int)ctx->host_flag[2];
      ctx->log_error_pending = false;
    }
    *log_error = ctx->last_log_error;
  });
}

// Towers the decode's fast path reads: the shortest prefix of q_0 .. q_{towers-1} whose product
// exceeds 2^130.  crt_value decodes X exactly over that prefix Q' while |X| < 2^127: the centred
// residue of X mod Q' is X itself, and |X| / Q' < 2^-3 keeps k's estimate clear of its rounding
// boundary, so the towers past the prefix change no output bit.  A coefficient
// outside that range sets the CRT range flag and the call is redone over every tower through
// crt_exact_kernel (round 6), as PALISADE's BigInteger decode, up to (Q - 1) / 2.  2^15 / L4
// (60 + 3 x 52 bits): 3 of 4 towers.  SHELFI_DEC_ALL_TOWERS=1 decodes with every tower (A/B probe
// switch; on chains too wide for crt_value's columns that is crt_exact_kernel).
static uint32_t decode_towers(const Params& p, uint32_t towers) {
  if (switches().dec_all_towers) return towers;
  uint32_t bits = 0;
  for (uint32_t t = 0; t < towers; ++t) {
    bits += 63 - (uint32_t)__builtin_clzll(p.q[t]);  // q_t >= 2^floor(log2 q_t)
    if (bits > 130) return t + 1;
  }
  return towers;
}

int shelfi_decrypt(shelfi_ctx* ctx, const uint8_t* blob, size_t len, size_t n, double* out) {
  if (!ctx || (n && !out)) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    require_keys(ctx);
    DeviceGuard g(ctx->device);
    const Params& p = ctx->p;
    const CtLayout h = open_cts(ctx, blob, len);
    if (n > h.K * (uint64_t)p.batch)
      throw Error{SHELFI_ERR_ARG, "decrypt: data_dimensions exceeds the slots in the ciphertexts"};
    if (!n) return;
    // ckks.cpp:192-196: ciphertext i contributes min(batch, n - i*batch) values
    const uint64_t K = (n + p.batch - 1) / p.batch;
    advise_huge(out, n * 8);
    const GenFlag fl = next_gen_flag(ctx);
    DecodeNoise dn = decode_noise_begin(ctx, K, fl);
    const uint64_t g0 = dn.g0;
    // one pipelined pass over the call: the decode's tower prefix (decode_towers: only those towers
    // are uploaded) with the fast CRT, or (exact) every tower through crt_exact_kernel
    const auto run = [&](bool exact) {
      Params pd = p;
      pd.L = exact ? p.L : decode_towers(p, p.L);
      const DeviceTables& dtd = pd.L == p.L ? ctx->dt : level_tables(ctx, pd.L);
      const size_t ct_bytes = 2ull * pd.L * p.N * 8;  // only the decode's towers travel
      uint64_t kc = std::max<uint64_t>(1, (64ull << 20) / ct_bytes);
      kc = std::min<uint64_t>(kc, K);
      const size_t cin = kc * ct_bytes, dout = kc * p.batch * 8;
      // a packed blob's tower prefix lands packed and is unpacked on the device
      const uint64_t ppre = 2 * packed_poly_bytes(p, pd.L);  // packed bytes of one ciphertext's prefix
      const size_t pin = h.packed ? kc * ppre : 0;
      uint8_t* io = (uint8_t*)ensure(ctx->io, ctx->io_bytes, 2 * (cin + dout + pin));
      uint8_t* cb[2] = {io, io + cin};
      uint8_t* ob[2] = {io + 2 * cin, io + 2 * cin + dout};
      uint8_t* pb[2] = {io + 2 * (cin + dout), io + 2 * (cin + dout) + pin};
      const ArenaPack apd = arena_pack_prefix(p, pd.L);
      void* scratch = ensure(ctx->scratch, ctx->scratch_bytes, decrypt_scratch_bytes(pd, kc));
      Pipe pp(ctx);
      StageRun sr(stager(ctx));
      dn.g0 = g0;
      dn.reset = 1;
      std::vector<HostPiece> pcs;
      const uint64_t nchunks = (K + kc - 1) / kc;
      for (uint64_t ci = 0; ci < nchunks; ++ci) {
        const int b = (int)(ci & 1);
        const uint64_t k0 = ci * kc, kn = std::min<uint64_t>(kc, K - k0);
        const uint64_t o0 = k0 * p.batch, on = std::min<uint64_t>(n - o0, kn * p.batch);
        if (ci >= 2) SHELFI_HIP(hipStreamWaitEvent(pp.a, pp.computed[b], 0));
        h.pieces(k0, kn, p, pcs, pd.L);
        sr.s.h2dv(h.packed ? pb[b] : cb[b], pcs.data(), pcs.size(), pp.a);
        SHELFI_HIP(hipEventRecord(pp.in_ready[b], pp.a));
        SHELFI_HIP(hipStreamWaitEvent(pp.b, pp.in_ready[b], 0));
        if (h.packed) launch_blob_unpack((const uint32_t*)pb[b], kn, pd.L, p.logN, apd, (uint64_t*)cb[b], pp.b);
        if (ci >= 2) SHELFI_HIP(hipStreamWaitEvent(pp.b, pp.out_free[b], 0));
        dn.g0 += (ci ? kc : 0);
        launch_decrypt(pd, dtd, ctx->dk, (const uint64_t*)cb[b], kn, h.scale, on, (double*)ob[b],
                       scratch, pp.b, &dn, false, 0, fl, exact);
        dn.reset = 0;
        SHELFI_HIP(hipEventRecord(pp.computed[b], pp.b));
        SHELFI_HIP(hipStreamWaitEvent(pp.c, pp.computed[b], 0));
        sr.s.d2h(out + o0, ob[b], on * 8, pp.c);
        SHELFI_HIP(hipEventRecord(pp.out_free[b], pp.c));
        sr.s.poll();
      }
      decode_noise_readback(ctx, dn, pp.b);
      sr.finish();
      pp.sync();
    };
    if (ctx->decode_exact)
      run(true);
    else {
      run(false);
      if (gen_flag_raised(ctx, fl, 2)) run(true);  // a value outside the fast CRT's range: the call again, exactly
    }
    decode_noise_end(ctx, dn);
  });
}

int shelfi_blob_info(const uint8_t* blob, size_t len, uint64_t* num_cts, uint32_t* depth,
                     double* scale, uint64_t* key_id) {
  return guarded([&] {
    BlobHeader h = parse_blob(blob, len, nullptr);
    if (num_cts) *num_cts = h.K;
    if (depth) *depth = h.depth;
    if (scale) *scale = h.scale;
    if (key_id) *key_id = h.key_id;
  });
}

size_t shelfi_blob_header_bytes(void) { return sizeof(BlobHeader); }

// Host restatement of blob_unpack_kernel (the packed wire payload): row r of the
// [K][2][L][N] batch, lane l, field j -> residue 128 (j >> 1) + 2 l + (j & 1).
int shelfi_blob_unpack(const shelfi_ctx* ctx, const uint8_t* blob, size_t len, uint64_t* out) {
  if (!ctx || !blob || !out) return SHELFI_ERR_ARG;
  return guarded([&] {
    const BlobHeader h = parse_blob(blob, len, ctx);
    const Params& p = ctx->p;
    const uint8_t* pay = blob + sizeof(BlobHeader);
    if (h.version == 1) {
      std::memcpy(out, pay, h.K * 2ull * p.L * p.N * 8);
      return;
    }
    const ArenaPack ap = arena_pack(p);
    const uint32_t rpt = p.N / kArenaChunk;
    size_t off = 0;  // dwords
    const uint32_t* w = reinterpret_cast<const uint32_t*>(pay);
    uint64_t* o = out;
    for (uint64_t g = 0; g < h.K * 2; ++g)
      for (uint32_t t = 0; t < p.L; ++t) {
        const uint32_t U = ap.w[t], B = U & ~3u, F = U & 1u, D = B / 4;
        const uint32_t N4 = D / 4, H2 = (D % 4) >= 2 ? 1 : 0, H1 = D & 1;
        const uint32_t O2 = N4 * 256, O1 = O2 + H2 * 128;
        for (uint32_t c = 0; c < rpt; ++c, off += 16 * U, o += kArenaChunk) {
          const uint32_t* sl = w + off;
          for (uint32_t lane = 0; lane < 64; ++lane) {
            uint32_t d[15] = {0};
            for (uint32_t q = 0; q < N4; ++q)
              for (uint32_t i = 0; i < 4; ++i) d[4 * q + i] = sl[q * 256 + 4 * lane + i];
            if (H2) {
              d[4 * N4] = sl[O2 + 2 * lane];
              d[4 * N4 + 1] = sl[O2 + 2 * lane + 1];
            }
            if (H1) d[D - 1] = sl[O1 + lane];
            const uint32_t fl = F ? reinterpret_cast<const uint8_t*>(sl)[64 * B + lane] : 0;
            for (uint32_t j = 0; j < 8; ++j) {
              const uint32_t bo = j * B, i = bo >> 5, sh = bo & 31;
              uint64_t v = (uint64_t)d[i] >> sh;
              if (sh + B > 32) v |= (uint64_t)d[i + 1] << (32 - sh);
              if (sh + B > 64) v |= (uint64_t)d[i + 2] << (64 - sh);
              v &= (1ull << B) - 1;
              if (F) v |= (uint64_t)((fl >> j) & 1u) << B;
              o[128 * (j >> 1) + 2 * lane + (j & 1)] = v;
            }
          }
        }
      }
  });
}

int shelfi_blob_pack(const shelfi_ctx* ctx, const uint64_t* residues, uint64_t K, uint32_t depth,
                     double scale, uint8_t** out, size_t* out_len) {
  if (!ctx || !out || !out_len || (K && !residues)) return SHELFI_ERR_ARG;
  return guarded([&] {
    const Params& p = ctx->p;
    const size_t payload = K * 2ull * p.L * p.N * 8;
    const BlobHeader h = make_header(ctx, K, depth, scale);
    uint8_t* blob = (uint8_t*)std::malloc(sizeof(h) + payload);
    if (!blob) throw std::bad_alloc();
    std::memcpy(blob, &h, sizeof(h));
    if (payload) std::memcpy(blob + sizeof(h), residues, payload);
    *out = blob;
    *out_len = sizeof(h) + payload;
  });
}

// ------------------------------------------------------------ device API ----
int shelfi_dev_wavg(shelfi_ctx* ctx, const uint64_t* const* in_dev, const float* w, size_t C,
                    size_t K, uint64_t* out_dev, void* stream) {
  if (!ctx || !out_dev || (C && (!in_dev || !w))) return SHELFI_ERR_ARG;
  return guarded([&] {
    if (!C) throw Error{SHELFI_ERR_ARG, "no learners"};
    check_weights(w, C, ctx->p.delta);
    DeviceGuard g(ctx->device);
    const Params& p = ctx->p;
    hipStream_t s = (hipStream_t)stream;  // 0 = legacy default stream
    for (size_t c0 = 0; c0 < C; c0 += kWavgMaxLearners) {
      const size_t gc = std::min<size_t>(kWavgMaxLearners, C - c0);
      WavgArgs a;
      std::memset(&a, 0, sizeof(a));
      for (size_t c = 0; c < gc; ++c) a.ptrs[c] = in_dev[c0 + c];
      fill_weights(a, p, w + c0, gc);
      a.out = out_dev;
      a.rows = (uint64_t)K * 2 * p.L;
      a.C = (uint32_t)gc;
      a.L = p.L;
      a.logN = p.logN;
      a.accumulate = c0 ? 1 : 0;
      launch_wavg(a, ctx->dt.tc, s);
    }
  });
}

int shelfi_dev_check_residues(shelfi_ctx* ctx, const uint64_t* ct_dev, size_t K, void* stream) {
  if (!ctx || (K && !ct_dev)) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    if (!K) return;
    DeviceGuard g(ctx->device);
    const Params& p = ctx->p;
    hipStream_t s = (hipStream_t)stream;
    uint32_t* bad = ctx->dev_flag + 6;
    SHELFI_HIP(hipMemsetAsync(bad, 0, 4, s));
    launch_check_residues(ct_dev, (uint64_t)K * 2 * p.L, p.L, p.logN, ctx->dt.tc, bad, s);
    SHELFI_HIP(hipMemcpyAsync(ctx->host_flag + 6, bad, 4, hipMemcpyDeviceToHost, s));
    SHELFI_HIP(hipStreamSynchronize(s));
    if (ctx->host_flag[6])
      throw Error{SHELFI_ERR_FORMAT, "ciphertext residue >= its tower modulus (malformed batch)"};
  });
}

size_t shelfi_arena_words(const shelfi_ctx* ctx, size_t C, size_t K) {
  if (!ctx) return 0;
  return (size_t)arena_ct_words(ctx->p, C) * K;
}

}  // extern "C"

namespace shelfi {
// The refusal bookkeeping of one put into slot `learner` of the arena [arena, arena + words) of C
// learners (ctx lock held): the slot's earlier entry is superseded, and so is every entry that
// overlaps this arena but names another base, span or learner count (that arena was freed and
// this memory reused); a refused put records the slot.
static void arena_mark(shelfi_ctx* ctx, const uint64_t* arena, size_t words, size_t C, size_t learner,
                       bool refused) {
  auto& R = ctx->arena_refused;
  for (size_t i = 0; i < R.size();) {
    const auto& r = R[i];
    const bool same_arena = r.arena == arena && r.words == words && r.C == C;
    const bool overlaps = arena < r.arena + r.words && r.arena < arena + words;
    if ((same_arena && r.learner == learner) || (overlaps && !same_arena)) R.erase(R.begin() + (long)i);
    else ++i;
  }
  if (refused) R.push_back({arena, words, C, learner});
}

// Placement of a learner's batch into its packed slices (arena_pack_kernel: the canonical-residue
// check of every residue rides along, ~0.3 ms of HBM per 1.4 GiB against ~30 ms of PCIe for the
// upload), then the slot's refusal mark is set or cleared.  `rows_of(k0, kn, dst)` makes
// ciphertexts [k0, k0 + kn) available as contiguous [kn][2][L][N] device residues and returns
// them (a device batch: the caller's pointer; host data: staged through `dst`, the context's
// scratch, `chunk` ciphertexts at a time).  Synchronises `s`.  Called under the ctx lock.
template <class RowsOf>
static void arena_place(shelfi_ctx* ctx, size_t K, size_t learner, size_t C, uint64_t* arena_dev, hipStream_t s,
                        size_t chunk, bool staged, RowsOf rows_of) {
  const Params& p = ctx->p;
  const ArenaPack ap = arena_pack(p);
  uint32_t* bad = ctx->dev_flag + 4;
  SHELFI_HIP(hipMemsetAsync(bad, 0, 4, s));
  const uint64_t ct_rows = 2ull * p.L * (p.N / kArenaChunk);
  uint64_t* dst = nullptr;
  if (staged)
    dst = (uint64_t*)ensure(ctx->scratch, ctx->scratch_bytes, std::min(chunk, K) * 2ull * p.L * p.N * 8);
  for (size_t k0 = 0; k0 < K; k0 += chunk) {
    const size_t kn = std::min(chunk, K - k0);
    const uint64_t* src = rows_of(k0, kn, dst);
    launch_arena_pack(src, k0 * ct_rows, kn * ct_rows, (uint32_t)C, (uint32_t)learner, p.L, p.logN, ap,
                      ctx->dt.tc, arena_dev, bad, s);
  }
  uint32_t flag = 0;
  SHELFI_HIP(hipMemcpyAsync(&flag, bad, 4, hipMemcpyDeviceToHost, s));
  SHELFI_HIP(hipStreamSynchronize(s));
  arena_mark(ctx, arena_dev, (size_t)arena_ct_words(p, C) * K, C, learner, flag != 0);
  if (flag)
    throw Error{SHELFI_ERR_FORMAT,
                "learner " + std::to_string(learner) +
                    ": ciphertext residue >= its tower modulus (malformed upload; the arena slot is "
                    "marked refused until a valid upload replaces it)"};
}
// How host uploads reach the device: a contiguous run (a library blob's payload, a host batch) as one
// hipMemcpyAsync from the caller's pageable memory (54 GB/s for a 1.5 GB upload), the 2 L tower runs
// of 256 KiB per ciphertext of a PALISADE archive through the bytes API's pinned staging ring (49 vs
// 18.5 GB/s as separate copies; probes/r03_arena_put.txt).  SHELFI_ARENA_STAGER=0|1 forces one (A/B
// probe switch).
static bool arena_use_stager(size_t pieces, size_t bytes) {
  if (switches().arena_stager >= 0) return switches().arena_stager == 1;
  return pieces > 1 && bytes / pieces < (4u << 20);
}
// Host uploads are staged through the scratch in pieces of about 64 MiB.
static size_t arena_stage_cts(const Params& p) {
  return std::max<size_t>(1, (64ull << 20) / (2ull * p.L * p.N * 8));
}

// Packed widths of the resident arena: U_t = bitlength(q_t) when that is 1 mod 4 (a
// 4-multiple field + a flag plane for the top bit), else 4 ceil(bitlength(q_t) / 4); at least 32.
ArenaPack arena_pack(const Params& p) {
  ArenaPack ap;
  std::memset(&ap, 0, sizeof(ap));
  for (uint32_t t = 0; t < p.L; ++t) {
    const uint32_t bits = 64 - (uint32_t)__builtin_clzll(p.q[t]);
    const uint32_t U = bits <= 32 ? 32u : (bits % 4 == 1 ? bits : (bits + 3) & ~3u);
    if (U > 60) throw Error{SHELFI_ERR_ARG, "arena: modulus above 2^60"};
    ap.w[t] = U;
    ap.pre[t] = ap.sum;
    ap.sum += U;
  }
  return ap;
}
// uint64 words per ciphertext of a C-learner arena: 2 N sum_t U_t / 64 per learner
uint64_t arena_ct_words(const Params& p, uint64_t C) {
  return C * 2ull * (p.N / kArenaChunk) * 8ull * arena_pack(p).sum;
}

// An aggregation over arena words [a, a + words) must not read a refused slot (ctx lock held).
void arena_require_valid_locked(const shelfi_ctx* ctx, const uint64_t* a, size_t words) {
  for (const auto& r : ctx->arena_refused)
    if (a < r.arena + r.words && r.arena < a + words)
      throw Error{SHELFI_ERR_STATE, "the arena holds a refused upload for learner " +
                                        std::to_string(r.learner) + "; put a valid batch first"};
}

// The arena aggregation itself (ctx lock held, weights checked): one wavg_packed pass over any
// number of learners (groups of 16 folded into a running sum), weight limbs from the device ring.
void wavg_arena_enqueue(shelfi_ctx* ctx, const uint64_t* arena_dev, const float* w, size_t C, size_t K,
                        uint64_t* out_dev, hipStream_t s) {
  const Params& p = ctx->p;
  const int slot = arena_weight_slot(ctx, w, C, s);
  launch_wavg_packed(arena_dev, ctx->wl_dev[slot], (uint32_t)C, (uint64_t)K * 2 * p.L, p.L, p.logN, arena_pack(p),
                     ctx->dt.tc, out_dev, s);
  SHELFI_HIP(hipEventRecord(ctx->wl_done[slot], s));
}

// The same aggregation with its result written in the packed C = 1 layout (the packed share
// exchange's send buffer): out_packed receives K ciphertexts, arena_ct_words(p, 1) words each.
void wavg_arena_enqueue_packed(shelfi_ctx* ctx, const uint64_t* arena_dev, const float* w, size_t C, size_t K,
                               uint64_t* out_packed, hipStream_t s) {
  const Params& p = ctx->p;
  const int slot = arena_weight_slot(ctx, w, C, s);
  launch_wavg_packed_ex(reinterpret_cast<const uint32_t*>(arena_dev), ctx->wl_dev[slot], (uint32_t)C, (uint32_t)C,
                        0, (uint64_t)K * 2 * p.L, p.L, p.logN, arena_pack(p), ctx->dt.tc, nullptr,
                        reinterpret_cast<uint32_t*>(out_packed), s);
  SHELFI_HIP(hipEventRecord(ctx->wl_done[slot], s));
}

// sum_g x_g mod q_t over G packed C = 1 batches of K ciphertexts stacked `stride` uint64 words apart
// (the packed share exchange's receive buffer) -> uint64 [K][2][L][N] canonical: wavg_packed with
// unit weight limbs (w0 = 1, w1 = 0), so the fold is the mod-q reduction.
void sum_packed_enqueue(shelfi_ctx* ctx, const uint64_t* stacked, size_t G, size_t K, size_t stride,
                        uint64_t* out, hipStream_t s) {
  const Params& p = ctx->p;
  if (!G || G > (size_t)kMaxCommRanks) throw Error{SHELFI_ERR_ARG, "sum_packed: 1..16 batches"};
  if (stride < (size_t)arena_ct_words(p, 1) * K) throw Error{SHELFI_ERR_ARG, "sum_packed: stride below the batch"};
  if (!ctx->unit_wl) {
    std::vector<uint32_t> one((size_t)kMaxCommRanks * kMaxTowers * 2, 0);
    for (size_t i = 0; i < one.size(); i += 2) one[i] = 1;
    SHELFI_HIP(hipMalloc(&ctx->unit_wl, one.size() * sizeof(uint32_t)));
    SHELFI_HIP(hipMemcpy(ctx->unit_wl, one.data(), one.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  }
  if (!K) return;
  launch_wavg_packed_ex(reinterpret_cast<const uint32_t*>(stacked), ctx->unit_wl, (uint32_t)G, 1, 2ull * stride,
                        (uint64_t)K * 2 * p.L, p.L, p.logN, arena_pack(p), ctx->dt.tc, out, nullptr, s);
}

void check_wavg_weights(const float* w, size_t C, double delta) { check_weights(w, C, delta); }
}  // namespace shelfi

extern "C" {

int shelfi_dev_arena_put(shelfi_ctx* ctx, const void* src, int src_on_host, size_t K, size_t learner,
                         size_t C, uint64_t* arena_dev, void* stream) {
  if (!ctx || !arena_dev || (K && !src) || learner >= C) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    DeviceGuard g(ctx->device);
    if (!K) return;
    const Params& p = ctx->p;
    hipStream_t s = (hipStream_t)stream;
    const size_t ct_words = 2ull * p.L * p.N;
    if (!src_on_host) {
      arena_place(ctx, K, learner, C, arena_dev, s, K, false, [&](size_t k0, size_t, uint64_t*) {
        return (const uint64_t*)src + k0 * ct_words;
      });
      return;
    }
    // host batches go through the pinned staging ring (the bytes API's copy pool)
    StageRun sr(stager(ctx));
    arena_place(ctx, K, learner, C, arena_dev, s, arena_stage_cts(p), true, [&](size_t k0, size_t kn, uint64_t* dst) {
      if (!arena_use_stager(1, kn * ct_words * 8)) {
        SHELFI_HIP(hipMemcpyAsync(dst, (const uint64_t*)src + k0 * ct_words, kn * ct_words * 8,
                                  hipMemcpyHostToDevice, s));
      } else {
        const HostPiece pc{(uint8_t*)((const uint64_t*)src + k0 * ct_words), kn * ct_words * 8};
        sr.s.h2dv(dst, &pc, 1, s);
      }
      return (const uint64_t*)dst;
    });
    sr.finish();
  });
}

int shelfi_dev_arena_put_blob(shelfi_ctx* ctx, const uint8_t* blob, size_t len, size_t K, size_t learner,
                              size_t C, uint64_t* arena_dev, void* stream) {
  if (!ctx || !arena_dev || !blob || learner >= C) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    // header first, against the context (parameters, key tag / key id), before any copy; a
    // refused header marks the slot refused too, so the slot's previous round cannot be
    // aggregated as if this upload had landed (the residue check below does the same)
    CtLayout v;
    try {
      v = open_cts(ctx, blob, len);
      if (v.K != K)
        throw Error{SHELFI_ERR_FORMAT, "upload holds " + std::to_string(v.K) + " ciphertexts, the arena " +
                                           std::to_string(K)};
    } catch (...) {
      arena_mark(ctx, arena_dev, (size_t)arena_ct_words(ctx->p, C) * K, C, learner, true);
      throw;
    }
    if (!K) return;
    DeviceGuard g(ctx->device);
    const Params& p = ctx->p;
    hipStream_t s = (hipStream_t)stream;
    std::vector<HostPiece> pcs;
    StageRun sr(stager(ctx));
    // a packed blob lands packed (in the bytes-API buffer, idle under the ctx lock) and is unpacked
    const uint64_t pct = 2 * packed_poly_bytes(p, p.L);
    uint8_t* pk = v.packed ? (uint8_t*)ensure(ctx->io, ctx->io_bytes, std::min(K, arena_stage_cts(p)) * pct) : nullptr;
    const ArenaPack ap = arena_pack(p);
    arena_place(ctx, K, learner, C, arena_dev, s, arena_stage_cts(p), true, [&](size_t k0, size_t kn, uint64_t* dst) {
      // a blob: one payload run; an archive: 2 L tower runs per ciphertext
      v.pieces(k0, kn, p, pcs);
      uint8_t* land = v.packed ? pk : (uint8_t*)dst;
      size_t bytes = 0;
      for (const HostPiece& pc : pcs) bytes += pc.n;
      if (arena_use_stager(pcs.size(), bytes)) {
        sr.s.h2dv(land, pcs.data(), pcs.size(), s);  // pinned staging ring, gathered in order
      } else {
        uint8_t* d = land;
        for (const HostPiece& pc : pcs) {
          SHELFI_HIP(hipMemcpyAsync(d, pc.p, pc.n, hipMemcpyHostToDevice, s));
          d += pc.n;
        }
      }
      if (v.packed) launch_blob_unpack((const uint32_t*)pk, kn, p.L, p.logN, ap, dst, s);
      return (const uint64_t*)dst;
    });
    sr.finish();
  });
}

int shelfi_dev_arena_release(shelfi_ctx* ctx, const uint64_t* arena_dev, size_t words) {
  if (!ctx || (words && !arena_dev)) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    auto& R = ctx->arena_refused;
    for (size_t i = 0; i < R.size();)
      if (arena_dev < R[i].arena + R[i].words && R[i].arena < arena_dev + words) R.erase(R.begin() + (long)i);
      else ++i;
  });
}

int shelfi_dev_wavg_arena(shelfi_ctx* ctx, const uint64_t* arena_dev, const float* w, size_t C,
                          size_t K, uint64_t* out_dev, void* stream) {
  if (!ctx || !out_dev || (C && (!arena_dev || !w))) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    if (!C) throw Error{SHELFI_ERR_ARG, "no learners"};
    check_weights(w, C, ctx->p.delta);
    arena_require_valid_locked(ctx, arena_dev, (size_t)arena_ct_words(ctx->p, C) * K);
    DeviceGuard g(ctx->device);
    wavg_arena_enqueue(ctx, arena_dev, w, C, K, out_dev, (hipStream_t)stream);
  });
}

int shelfi_dev_wavg_arena_packed(shelfi_ctx* ctx, const uint64_t* arena_dev, const float* w, size_t C, size_t K,
                                 uint64_t* out_packed, void* stream) {
  if (!ctx || (K && !out_packed) || (C && (!arena_dev || !w))) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    if (!C) throw Error{SHELFI_ERR_ARG, "no learners"};
    check_weights(w, C, ctx->p.delta);
    arena_require_valid_locked(ctx, arena_dev, (size_t)arena_ct_words(ctx->p, C) * K);
    DeviceGuard g(ctx->device);
    wavg_arena_enqueue_packed(ctx, arena_dev, w, C, K, out_packed, (hipStream_t)stream);
  });
}

int shelfi_dev_sum_packed(shelfi_ctx* ctx, const uint64_t* stacked, size_t G, size_t K, size_t stride_words,
                          uint64_t* out_dev, void* stream) {
  if (!ctx || (K && (!stacked || !out_dev))) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    DeviceGuard g(ctx->device);
    sum_packed_enqueue(ctx, stacked, G, K, stride_words, out_dev, (hipStream_t)stream);
  });
}

int shelfi_dev_wavg_arena_pick_output(shelfi_ctx* ctx, const uint64_t* arena_dev, const float* w,
                                      size_t C, size_t K, uint64_t* const* candidates, size_t n,
                                      int launches, size_t* best, float* ms, void* stream) {
  if (!ctx || !candidates || !best || !n || launches < 1) return SHELFI_ERR_ARG;
  return guarded([&] {
    DeviceGuard g(ctx->device);
    hipStream_t s = (hipStream_t)stream;
    struct Events {
      hipEvent_t a = nullptr, b = nullptr;
      ~Events() {
        if (a) (void)hipEventDestroy(a);
        if (b) (void)hipEventDestroy(b);
      }
    } ev;
    SHELFI_HIP(hipEventCreate(&ev.a));
    SHELFI_HIP(hipEventCreate(&ev.b));
    auto run = [&](uint64_t* out) {
      const int rc = shelfi_dev_wavg_arena(ctx, arena_dev, w, C, K, out, stream);
      if (rc) throw Error{rc, shelfi_last_error()};
    };
    float best_ms = 0.f;
    for (size_t i = 0; i < n; ++i) {
      if (!candidates[i]) throw Error{SHELFI_ERR_ARG, "null candidate buffer"};
      run(candidates[i]);  // warm-up
      SHELFI_HIP(hipEventRecord(ev.a, s));
      for (int l = 0; l < launches; ++l) run(candidates[i]);
      SHELFI_HIP(hipEventRecord(ev.b, s));
      SHELFI_HIP(hipEventSynchronize(ev.b));
      float t = 0.f;
      SHELFI_HIP(hipEventElapsedTime(&t, ev.a, ev.b));
      t /= (float)launches;
      if (ms) ms[i] = t;
      if (i == 0 || t < best_ms) {
        best_ms = t;
        *best = i;
      }
    }
  });
}

int shelfi_dev_modq(shelfi_ctx* ctx, uint64_t* buf_dev, size_t K, void* stream) {
  if (!ctx || !buf_dev) return SHELFI_ERR_ARG;
  return guarded([&] {
    DeviceGuard g(ctx->device);
    hipStream_t s = (hipStream_t)stream;  // 0 = legacy default stream
    launch_modq(buf_dev, (uint64_t)K * 2 * ctx->p.L, ctx->p.L, ctx->p.logN, ctx->dt.tc, s);
  });
}

// Ciphertexts per launch chain of the device-resident encrypt/decrypt: as many as a
// 4 GiB scratch holds (1149 at N = 2^15, L = 4: one chain for a ResNet-18 learner),
// split into equal chunks, so no launch runs a short tail chunk.
// SHELFI_DEV_CHUNK_MIB overrides the budget (A/B probe switch).
static uint64_t dev_chunk(uint64_t K, size_t scratch_per_ct) {
  const uint64_t mib = switches().dev_chunk_mib;
  const uint64_t cap = std::max<uint64_t>(1, (mib << 20) / scratch_per_ct);
  const uint64_t n = (K + cap - 1) / cap;
  return n ? (K + n - 1) / n : 1;
}

int shelfi_dev_encrypt(shelfi_ctx* ctx, const double* x_dev, size_t n, uint64_t* ct_dev,
                       void* stream) {
  if (!ctx || (n && (!x_dev || !ct_dev))) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    require_keys(ctx);
    DeviceGuard g(ctx->device);
    const Params& p = ctx->p;
    hipStream_t s = (hipStream_t)stream;  // 0 = legacy default stream
    const uint64_t K = (n + p.batch - 1) / p.batch;
    if (!K) return;
    uint32_t key[8];
    uint64_t g0;
    draw_key(ctx, K, key, &g0);
    const uint64_t kc_max = dev_chunk(K, encrypt_scratch_bytes(p, 1));
    void* scratch = ensure(ctx->scratch, ctx->scratch_bytes, encrypt_scratch_bytes(p, kc_max));
    const GenFlag fl = next_gen_flag(ctx);
    const size_t ct_words = 2ull * p.L * p.N;
    bool approx = false;
    for (int pass = 0; pass < 2; ++pass) {
      for (uint64_t k0 = 0; k0 < K; k0 += kc_max) {
        const uint64_t kc = std::min(kc_max, K - k0);
        const uint64_t xs = k0 * p.batch, xn = std::min<uint64_t>(n - xs, kc * p.batch);
        if (approx)
          launch_encrypt_approx(p, ctx->dt, ctx->dk, x_dev + xs, xn, kc, ct_dev + k0 * ct_words, scratch, key,
                                g0 + k0, s);
        else
          launch_encrypt(p, ctx->dt, ctx->dk, x_dev + xs, xn, kc, ct_dev + k0 * ct_words, scratch,
                         key, g0 + k0, fl, s);
      }
      if (approx) break;
      SHELFI_HIP(hipStreamSynchronize(s));  // scratch is reused by the next call
      bool redo;
      try {
        redo = encode_needs_approx(ctx, fl);
      } catch (...) {
        std::memset(key, 0, sizeof(key));
        throw;
      }
      if (!redo) break;
      approx = true;  // some |x Delta| > 2^61: redo the call on the large-value path
    }
    std::memset(key, 0, sizeof(key));
  });
}

// decrypt K ciphertexts of `towers` RNS towers (the context's L, or fewer after ModReduce)
// (sum_in: residues are uint64 sums of <= 16 canonical residues, folded on load)
static int dev_decrypt(shelfi_ctx* ctx, const uint64_t* ct_dev, size_t K, uint32_t towers, double scale,
                       size_t n, double* out_dev, void* stream, bool sum_in = false) {
  if (!ctx || (n && (!ct_dev || !out_dev))) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    require_keys(ctx);
    DeviceGuard g(ctx->device);
    if (towers < 1 || towers > ctx->p.L) throw Error{SHELFI_ERR_ARG, "tower count out of range for this context"};
    if (n > (uint64_t)K * ctx->p.batch) throw Error{SHELFI_ERR_ARG, "n exceeds the slots in K ciphertexts"};
    hipStream_t s = (hipStream_t)stream;  // 0 = legacy default stream
    const uint64_t Kn = (n + ctx->p.batch - 1) / ctx->p.batch;
    if (!Kn) return;
    const size_t ct_words = 2ull * towers * ctx->p.N;
    const GenFlag fl = next_gen_flag(ctx);
    DecodeNoise dn = decode_noise_begin(ctx, Kn, fl);
    const uint64_t g0 = dn.g0;
    // one pass over the call: the decode's tower prefix with the fast CRT, or (exact) every tower
    // through crt_exact_kernel
    const auto run = [&](bool exact) {
      Params p = ctx->p;
      p.L = exact ? towers : decode_towers(ctx->p, towers);  // Q' = q_0 .. q_{p.L-1}; the secret key's first towers
      const DeviceTables& dt = p.L == ctx->p.L ? ctx->dt : level_tables(ctx, p.L);
      const uint64_t kc_max = dev_chunk(Kn, decrypt_scratch_bytes(p, 1));
      void* scratch = ensure(ctx->scratch, ctx->scratch_bytes, decrypt_scratch_bytes(p, kc_max));
      dn.reset = 1;
      for (uint64_t k0 = 0; k0 < Kn; k0 += kc_max) {
        const uint64_t kc = std::min(kc_max, Kn - k0);
        const uint64_t o0 = k0 * p.batch, on = std::min<uint64_t>(n - o0, kc * p.batch);
        dn.g0 = g0 + k0;
        launch_decrypt(p, dt, ctx->dk, ct_dev + k0 * ct_words, kc, scale, on, out_dev + o0, scratch, s, &dn,
                       sum_in, towers, fl, exact);
        dn.reset = 0;  // the flags are reset by the first chunk's flooding only
      }
      decode_noise_readback(ctx, dn, s);
    };
    if (ctx->decode_exact) {
      run(true);
    } else {
      run(false);
      SHELFI_HIP(hipStreamSynchronize(s));
      if (gen_flag_raised(ctx, fl, 2)) run(true);  // a value outside the fast CRT's range: the call again, exactly
    }
    SHELFI_HIP(hipStreamSynchronize(s));  // scratch is reused by the next call
    decode_noise_end(ctx, dn);
  });
}

int shelfi_dev_decrypt(shelfi_ctx* ctx, const uint64_t* ct_dev, size_t K, double scale, size_t n,
                       double* out_dev, void* stream) {
  return dev_decrypt(ctx, ct_dev, K, ctx ? ctx->p.L : 0, scale, n, out_dev, stream);
}

int shelfi_dev_decrypt_level(shelfi_ctx* ctx, const uint64_t* ct_dev, size_t K, uint32_t towers, double scale,
                             size_t n, double* out_dev, void* stream) {
  return dev_decrypt(ctx, ct_dev, K, towers, scale, n, out_dev, stream);
}

int shelfi_dev_decrypt_sum(shelfi_ctx* ctx, const uint64_t* ct_dev, size_t K, uint32_t terms, double scale,
                           size_t n, double* out_dev, void* stream) {
  if (terms < 1 || terms > (uint32_t)kMaxCommRanks) {
    set_error("decrypt_sum: the residues must be sums of 1..16 canonical residues");
    return SHELFI_ERR_ARG;
  }
  return dev_decrypt(ctx, ct_dev, K, ctx ? ctx->p.L : 0, scale, n, out_dev, stream, true);
}

int shelfi_dev_ntt(shelfi_ctx* ctx, uint64_t* polys_dev, size_t P, int inverse, void* stream) {
  if (!ctx || (P && !polys_dev)) return SHELFI_ERR_ARG;
  return guarded([&] {
    DeviceGuard g(ctx->device);
    hipStream_t s = (hipStream_t)stream;  // 0 = legacy default stream
    launch_ntt(polys_dev, P, ctx->p.L, ctx->p.logN, inverse != 0, ctx->dt, s);
  });
}

int shelfi_fft_twiddles(uint32_t slots, double* ir, double* ii, double* fr, double* fi) {
  if (!slots || (slots & (slots - 1)) || !ir || !ii || !fr || !fi) return SHELFI_ERR_ARG;
  fft_twiddles(slots, ir, ii, fr, fi);
  return SHELFI_OK;
}

int shelfi_gauss_cdt(double sigma, uint64_t* cdt, int max_entries) {
  if (!cdt) return SHELFI_ERR_ARG;
  return gauss_cdt(sigma, cdt, max_entries);
}

}  // extern "C"

// ------------------------------------------------- PALISADE wire format ----
int shelfi_set_wire_format(shelfi_ctx* ctx, int format) {
  if (!ctx || format < 0 || format > 2) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return guarded([&] {
    if (format == 1 && ctx->pal_ctx_obj.empty())
      throw Error{SHELFI_ERR_STATE, "PALISADE wire format needs keys loaded from PALISADE files"};
    ctx->wire = format;
  });
}

int shelfi_get_wire_format(const shelfi_ctx* ctx) {
  if (!ctx) return -1;
  std::lock_guard<std::mutex> lk(ctx_mutex(ctx));
  return ctx->wire;
}

int shelfi_palisade_parse(const uint8_t* archive, size_t len, shelfi_palisade_info* info,
                          uint64_t* residues) {
  if (!archive || !info) return SHELFI_ERR_ARG;
  return guarded([&] {
    const PalisadeArchive A = palisade_parse_archive(archive, len);
    std::memset(info, 0, sizeof(*info));
    info->ring_dim = A.N;
    info->num_towers = A.L;
    info->num_cts = A.K;
    for (uint32_t t = 0; t < A.L; ++t) info->moduli[t] = A.q[t];
    info->depth = A.depth;
    info->level = A.level;
    info->scale = A.scale;
    info->encoding = A.encoding;
    info->vector_archive = A.vector_archive ? 1 : 0;
    info->ctx_offset = A.ctx_off;
    info->ctx_length = A.ctx_len;
    std::memcpy(info->keytag, A.keytag.data(), std::min<size_t>(A.keytag.size(), 256));
    if (residues)
      for (size_t i = 0; i < A.tower_off.size(); ++i)
        std::memcpy(residues + i * (size_t)A.N, archive + A.tower_off[i], (size_t)A.N * 8);
  });
}

int shelfi_palisade_write(const uint8_t* ctx_obj, size_t ctx_len, const char* keytag,
                          uint32_t ring_dim, uint32_t num_towers, const uint64_t* moduli,
                          uint64_t num_cts, const uint64_t* residues, uint64_t depth, uint64_t level,
                          double scale, int flags, uint8_t** out, size_t* out_len) {
  if (!ctx_obj || !keytag || !moduli || !out || !out_len || (num_cts && !residues) ||
      num_towers < 1 || num_towers > (uint32_t)kMaxTowers)
    return SHELFI_ERR_ARG;
  *out = nullptr;
  *out_len = 0;
  return guarded([&] {
    const std::string obj((const char*)ctx_obj, ctx_len), tag(keytag);
    const bool vec = (flags & SHELFI_PAL_VECTOR) != 0, kp = (flags & SHELFI_PAL_KEY_PARAMS) != 0;
    size_t total = 0;
    palisade_layout(obj, tag, ring_dim, num_towers, moduli, num_cts, depth, level, scale, 4, vec, kp,
                    nullptr, &total);
    uint8_t* buf = (uint8_t*)std::malloc(total);
    if (!buf) throw std::bad_alloc();
    const std::vector<size_t> off = palisade_layout(obj, tag, ring_dim, num_towers, moduli, num_cts,
                                                    depth, level, scale, 4, vec, kp, buf, &total);
    for (size_t i = 0; i < off.size(); ++i)
      std::memcpy(buf + off[i], residues + i * (size_t)ring_dim, (size_t)ring_dim * 8);
    *out = buf;
    *out_len = total;
  });
}

static void take_string(const std::string& s, uint8_t** out, size_t* out_len) {
  uint8_t* buf = (uint8_t*)std::malloc(s.size() ? s.size() : 1);
  if (!buf) throw std::bad_alloc();
  std::memcpy(buf, s.data(), s.size());
  *out = buf;
  *out_len = s.size();
}

int shelfi_palisade_context_file(uint32_t ring_dim, uint32_t num_towers, const uint64_t* moduli,
                                 const uint64_t* roots, uint32_t scale_bits, uint32_t batch,
                                 uint8_t** out, size_t* out_len) {
  if (!moduli || !roots || !out || !out_len || num_towers < 1 || num_towers > (uint32_t)kMaxTowers)
    return SHELFI_ERR_ARG;
  *out = nullptr;
  return guarded([&] {
    PalisadeCtxParams cp;
    cp.N = ring_dim;
    cp.L = num_towers;
    cp.q.assign(moduli, moduli + num_towers);
    cp.psi.assign(roots, roots + num_towers);
    cp.plaintext_modulus = scale_bits;
    cp.batch = batch;
    take_string(palisade_context_file(cp), out, out_len);
  });
}

int shelfi_palisade_key_file(const uint8_t* ctx_obj, size_t ctx_len, const char* keytag,
                             const uint64_t* polys, int is_public, uint8_t** out, size_t* out_len) {
  if (!ctx_obj || !keytag || !polys || !out || !out_len) return SHELFI_ERR_ARG;
  *out = nullptr;
  return guarded([&] {
    uint32_t id0 = 0;
    const PalisadeCtxParams cp =
        palisade_parse_context_object(std::string((const char*)ctx_obj, ctx_len), &id0);
    if (id0 != 3) throw Error{SHELFI_ERR_FORMAT, "context object must be in embedded form (ids from 3)"};
    take_string(palisade_key_file(cp, keytag, polys, is_public != 0), out, out_len);
  });
}

int shelfi_palisade_key_context(const uint8_t* pub, size_t len, uint8_t** ctx_obj, size_t* ctx_len,
                                char* keytag) {
  if (!pub || !ctx_obj || !ctx_len || !keytag) return SHELFI_ERR_ARG;
  *ctx_obj = nullptr;
  return guarded([&] {
    std::string obj, tag;
    palisade_key_context(std::string((const char*)pub, len), obj, tag);
    uint8_t* buf = (uint8_t*)std::malloc(obj.size());
    if (!buf) throw std::bad_alloc();
    std::memcpy(buf, obj.data(), obj.size());
    *ctx_obj = buf;
    *ctx_len = obj.size();
    std::memset(keytag, 0, 257);
    std::memcpy(keytag, tag.data(), std::min<size_t>(tag.size(), 256));
  });
}

int shelfi_palisade_embed_context(const uint8_t* ctxfile, size_t len, uint8_t** out,
                                  size_t* out_len) {
  if (!ctxfile || !out || !out_len) return SHELFI_ERR_ARG;
  *out = nullptr;
  return guarded([&] {
    const std::string obj = palisade_embed_context(std::string((const char*)ctxfile, len));
    uint8_t* buf = (uint8_t*)std::malloc(obj.size());
    if (!buf) throw std::bad_alloc();
    std::memcpy(buf, obj.data(), obj.size());
    *out = buf;
    *out_len = obj.size();
  });
}

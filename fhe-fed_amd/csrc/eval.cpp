// eval.cpp — C ABI of SURVEY §8 f4: EvalMultKeyGen, EvalMult (ct x ct) with HYBRID
// relinearization, ModReduce, and the per-level tables they (and decrypt at a level) use.
//
// None of this is on the reference's aggregation path (ckks.cpp:26 fixes multDepth = 1 and
// computeWeightedAverage only multiplies by constants); it is the general-circuit part of
// the PALISADE 1.11 CKKS scheme the reference builds its contexts with.  Host code only
// precomputes constants and moves keys; every per-ciphertext step is in keyswitch.hip.
#include <algorithm>
#include <cstring>
#include <fstream>
#include <sstream>

#include "api_util.h"
#include "palisade_codec.h"
#include "shelfi_internal.h"

namespace shelfi {

constexpr int kMaxDigits = 3;  // ComputeNumLargeDigits never exceeds 3

struct LevelState {
  bool built = false;  // key-switching state (ext, dtf, ks, args)
  bool q_built = false;
  bool own_q = false;  // q tables built here (levels below L); level L uses ctx->dt
  DeviceTables q;      // Q_l: NTT + CRT tables (decrypt at this level)
  DeviceTables ext;    // Q_l u P (key switching)
  DeviceTables dtf[kMaxDigits];  // per digit: its foreign towers (Q_l minus the digit, then P)
  uint64_t* ks = nullptr;
  KsArgs args{};
};

struct EvalState {
  uint32_t dnum = 0, alpha = 0, kP = 0;
  uint64_t p[kMaxTowers] = {0}, ppsi[kMaxTowers] = {0};
  std::string ks_error;        // why this chain cannot key-switch ("" = it can)
  uint64_t* evk = nullptr;     // [2][dnum][L + kP][N] (b-vector, a-vector)
  uint64_t* evk_sh = nullptr;  // Shoup companions
  std::vector<uint64_t> evk_host;
  LevelState lv[kMaxTowers + 1];  // index = towers Ll
};

static uint64_t mm(uint64_t a, uint64_t b, uint64_t q) { return (uint64_t)(((u128)a * b) % q); }

// key-switching state of a level (its Q_l tables stay: decrypt at the level uses them)
static void free_level_ks(LevelState& l) {
  free_ntt_tables(l.ext);
  for (auto& d : l.dtf) free_ntt_tables(d);
  dfree_t(l.ks);
  l.ext = DeviceTables{};
  for (auto& d : l.dtf) d = DeviceTables{};
  l.args = KsArgs{};
  l.built = false;
}

static void free_level(LevelState& l) {
  if (l.own_q) free_ntt_tables(l.q);
  free_level_ks(l);
  l = LevelState{};
}

void eval_release(shelfi_ctx* ctx, bool keys_only) {
  EvalState* ev = ctx->ev;
  if (!ev) return;
  dfree_t(ev->evk);
  dfree_t(ev->evk_sh);
  ev->evk_host.clear();
  if (keys_only) return;
  for (auto& l : ev->lv) free_level(l);
  delete ev;
  ctx->ev = nullptr;
}

// Per-context level state.  The special primes are derived here, but a chain that cannot
// key-switch (L + kP > 16) only fails EvalMult: decrypt and ModReduce at any level need
// nothing but the Q_l tables.
static EvalState& eval_state(shelfi_ctx* ctx) {
  if (ctx->ev) return *ctx->ev;
  const Params& p = ctx->p;
  auto ev = new EvalState();
  try {
    special_primes(p.N, p.L, p.q, &ev->dnum, &ev->alpha, &ev->kP, ev->p, ev->ppsi);
    if (p.L + ev->kP > (uint32_t)kMaxTowers) ev->ks_error = "EvalMult needs num_towers + special primes <= 16";
  } catch (const Error& e) {
    ev->ks_error = e.msg;
  }
  ctx->ev = ev;
  return *ev;
}

// NTT + CRT tables of Q_l = q_0 .. q_{Ll-1} (decrypt at a level): built on first use, no
// key-switching state.
static const DeviceTables& level_q(shelfi_ctx* ctx, uint32_t Ll) {
  EvalState& ev = eval_state(ctx);
  const Params& P0 = ctx->p;
  if (Ll < 1 || Ll > P0.L) throw Error{SHELFI_ERR_ARG, "tower count out of range for this context"};
  LevelState& l = ev.lv[Ll];
  if (l.q_built) return l.q;
  if (Ll == P0.L) {
    l.q = ctx->dt;
    l.own_q = false;
  } else {
    Params pl = P0;
    pl.L = Ll;
    DeviceTables q;
    try {
      build_ntt_tables(pl, q);
    } catch (...) {
      free_ntt_tables(q);
      throw;
    }
    l.q = q;
    l.own_q = true;
    l.q.fft_inv = ctx->dt.fft_inv;  // shared, owned by the context
    l.q.fft_fwd = ctx->dt.fft_fwd;
    l.q.cdt = ctx->dt.cdt;
    l.q.cdt_len = ctx->dt.cdt_len;
  }
  l.q_built = true;
  return l.q;
}

// Tables and key-switching constants for ciphertexts of Ll towers (Q_l = q_0 .. q_{Ll-1}).
static LevelState& level(shelfi_ctx* ctx, uint32_t Ll) {
  EvalState& ev = eval_state(ctx);
  if (!ev.ks_error.empty()) throw Error{SHELFI_ERR_ARG, ev.ks_error};
  const Params& P0 = ctx->p;
  level_q(ctx, Ll);
  LevelState& l = ev.lv[Ll];
  if (l.built) return l;
  const uint32_t kP = ev.kP, T = Ll + kP, al = ev.alpha, dn = (Ll + al - 1) / al;
  try {
    Params pe = P0;
    pe.L = T;
    for (uint32_t m = 0; m < kP; ++m) {
      pe.q[Ll + m] = ev.p[m];
      pe.psi[Ll + m] = ev.ppsi[m];
    }
    build_ntt_tables(pe, l.ext);
    if (dn > (uint32_t)kMaxDigits) throw Error{SHELFI_ERR_ARG, "EvalMult: more than 3 digits"};
    for (uint32_t j = 0; j < dn; ++j) {  // digit j's foreign towers, in ModUp's order
      const uint32_t s = j * al, cnt = std::min(al, Ll - s);
      Params pf = P0;
      pf.L = T - cnt;
      for (uint32_t t = 0, u = 0; t < T; ++t)
        if (t < s || t >= s + cnt) {
          pf.q[u] = pe.q[t];
          pf.psi[u] = pe.psi[t];
          ++u;
        }
      build_ntt_tables(pf, l.dtf[j]);
    }
    // constants: mu_inv | mu_inv_sh [dn][al] | mu_hat [dn][al][T] | md_inv | md_inv_sh [kP] |
    // md_hat [kP][Ll] | pinv | pinv_sh [Ll]
    const size_t o_mi = 0, o_mis = o_mi + dn * al, o_mh = o_mis + dn * al, o_di = o_mh + (size_t)dn * al * T,
                 o_dis = o_di + kP, o_dh = o_dis + kP, o_pi = o_dh + (size_t)kP * Ll, o_pis = o_pi + Ll,
                 total = o_pis + Ll;
    std::vector<uint64_t> c(total, 0);
    for (uint32_t j = 0; j < dn; ++j) {
      const uint32_t s = j * al, cnt = std::min(al, Ll - s);
      for (uint32_t i = 0; i < cnt; ++i) {
        const uint64_t qi = pe.q[s + i];
        uint64_t h = 1;
        for (uint32_t u = 0; u < cnt; ++u)
          if (u != i) h = mm(h, pe.q[s + u] % qi, qi);
        const uint64_t inv = invmod(h, qi);
        c[o_mi + j * al + i] = inv;
        c[o_mis + j * al + i] = shoup(inv, qi);
        for (uint32_t t = 0; t < T; ++t) {
          const uint64_t qt = pe.q[t];
          uint64_t v = 1;
          for (uint32_t u = 0; u < cnt; ++u)
            if (u != i) v = mm(v, pe.q[s + u] % qt, qt);
          c[o_mh + ((size_t)j * al + i) * T + t] = v;
        }
      }
    }
    for (uint32_t m = 0; m < kP; ++m) {
      const uint64_t pm = ev.p[m];
      uint64_t h = 1;
      for (uint32_t u = 0; u < kP; ++u)
        if (u != m) h = mm(h, ev.p[u] % pm, pm);
      const uint64_t inv = invmod(h, pm);
      c[o_di + m] = inv;
      c[o_dis + m] = shoup(inv, pm);
      for (uint32_t t = 0; t < Ll; ++t) {
        const uint64_t qt = P0.q[t];
        uint64_t v = 1;
        for (uint32_t u = 0; u < kP; ++u)
          if (u != m) v = mm(v, ev.p[u] % qt, qt);
        c[o_dh + (size_t)m * Ll + t] = v;
      }
    }
    for (uint32_t t = 0; t < Ll; ++t) {
      const uint64_t qt = P0.q[t];
      uint64_t pm = 1;
      for (uint32_t u = 0; u < kP; ++u) pm = mm(pm, ev.p[u] % qt, qt);
      const uint64_t inv = invmod(pm, qt);
      c[o_pi + t] = inv;
      c[o_pis + t] = shoup(inv, qt);
    }
    l.ks = upload(c.data(), total);
    KsArgs& a = l.args;
    a.Ll = Ll;
    a.kP = kP;
    a.T = T;
    a.dn = dn;
    a.alpha = al;
    a.logN = P0.logN;
    a.Lfull = P0.L;
    a.dnFull = ev.dnum;
    a.mu_inv = l.ks + o_mi;
    a.mu_inv_sh = l.ks + o_mis;
    a.mu_hat = l.ks + o_mh;
    a.md_inv = l.ks + o_di;
    a.md_inv_sh = l.ks + o_dis;
    a.md_hat = l.ks + o_dh;
    a.pinv = l.ks + o_pi;
    a.pinv_sh = l.ks + o_pis;
    a.tq = ctx->dt.tc;  // q / Shoup constants only: the context's prefix serves every level
    a.te = l.ext.tc;
  } catch (...) {
    free_level_ks(l);
    throw;
  }
  l.built = true;
  return l;
}

// tables of Q_l for decrypt at a level (api.cpp): the Q_l tables alone
const DeviceTables& level_tables(shelfi_ctx* ctx, uint32_t Ll) { return level_q(ctx, Ll); }

static void install_evk(shelfi_ctx* ctx, EvalState& ev, const uint64_t* evk) {
  const Params& p = ctx->p;
  if (!ev.ks_error.empty()) throw Error{SHELFI_ERR_ARG, ev.ks_error};
  const uint32_t T0 = p.L + ev.kP;
  const size_t TN = (size_t)T0 * p.N, words = 2ull * ev.dnum * TN;
  std::vector<uint64_t> sh(words);
  for (size_t i = 0; i < words; ++i) {
    const uint32_t t = (uint32_t)((i % TN) / p.N);
    const uint64_t q = t < p.L ? p.q[t] : ev.p[t - p.L];
    if (evk[i] >= q) throw Error{SHELFI_ERR_FORMAT, "evaluation key residue >= modulus"};
    sh[i] = shoup(evk[i], q);
  }
  dfree_t(ev.evk);
  dfree_t(ev.evk_sh);
  ev.evk_host.assign(evk, evk + words);
  ev.evk = upload(evk, words);
  ev.evk_sh = upload(sh.data(), words);
}

// key-eval-mult.txt metadata of this context's evaluation key (PALISADE keys required: the
// file embeds the context object and key tag of key-public.txt)
static PalisadeEvalKey evalkey_meta(const shelfi_ctx* ctx, const EvalState& ev) {
  if (ctx->pal_ctx_obj.empty() || ctx->pal_keytag.empty())
    throw Error{SHELFI_ERR_STATE, "evaluation-key files need PALISADE keys (loadCryptoParams or keygen)"};
  const Params& p = ctx->p;
  PalisadeEvalKey K;
  uint32_t id0 = 0;
  K.ctx = palisade_parse_context_object(ctx->pal_ctx_obj, &id0, 1);
  K.keytag = ctx->pal_keytag;
  K.N = p.N;
  K.T = p.L + ev.kP;
  K.dnum = ev.dnum;
  for (uint32_t t = 0; t < K.T; ++t) {
    K.q.push_back(t < p.L ? p.q[t] : ev.p[t - p.L]);
    K.psi.push_back(t < p.L ? p.psi[t] : ev.ppsi[t - p.L]);
  }
  // class versions as in the reference's own key-eval-mult.txt
  for (auto& v : K.poly_versions) v = 0;
  return K;
}

static std::string slurp(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw Error{SHELFI_ERR_IO, "cannot read " + path};
  std::ostringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// install a parsed PALISADE evaluation key after checking it belongs to these keys / params
static void load_evalkey(shelfi_ctx* ctx, const std::string& file) {
  EvalState& ev = eval_state(ctx);
  const PalisadeEvalKey K = palisade_parse_evalmult_key((const uint8_t*)file.data(), file.size());
  const Params& p = ctx->p;
  if (ctx->pal_keytag.empty() || K.keytag != ctx->pal_keytag)
    throw Error{SHELFI_ERR_FORMAT, "evaluation key belongs to another key pair (key tag)"};
  if (K.N != p.N || K.T != p.L + ev.kP || K.dnum != ev.dnum)
    throw Error{SHELFI_ERR_FORMAT, "evaluation key was made for other parameters"};
  for (uint32_t t = 0; t < K.T; ++t)
    if (K.q[t] != (t < p.L ? p.q[t] : ev.p[t - p.L]))
      throw Error{SHELFI_ERR_FORMAT, "evaluation key towers differ from this context's Q and special primes"};
  if (K.tower_off.size() != 2ull * K.dnum * K.T) throw Error{SHELFI_ERR_FORMAT, "evaluation key tower count"};
  // residues: the key's roots may differ from ours for the special primes (PALISADE picks its
  // own); the EVALUATION order then differs, so only keys on the same roots are accepted
  for (uint32_t t = 0; t < K.T; ++t)
    if (K.psi[t] != (t < p.L ? p.psi[t] : ev.ppsi[t - p.L]))
      throw Error{SHELFI_ERR_FORMAT, "evaluation key roots of unity differ from this context's"};
  std::vector<uint64_t> polys(K.tower_off.size() * (size_t)K.N);
  for (size_t i = 0; i < K.tower_off.size(); ++i)
    std::memcpy(polys.data() + i * K.N, file.data() + K.tower_off[i], (size_t)K.N * 8);
  install_evk(ctx, ev, polys.data());
}

// shelfi_load: a key-eval-mult.txt beside PALISADE keys is loaded when it is theirs
void load_evalkey_if_present(shelfi_ctx* ctx, const std::string& dir) {
  std::string file;
  try {
    file = slurp(dir + "key-eval-mult.txt");
  } catch (const Error&) {
    return;  // optional file
  }
  try {
    load_evalkey(ctx, file);
  } catch (const Error&) {
    // another key pair's or another ring's key (e.g. palisade_pybind's resources): not ours
  }
}

static uint64_t chunk_of(uint64_t K, size_t per_ct) {
  const uint64_t cap = std::max<uint64_t>(1, (2048ull << 20) / std::max<size_t>(per_ct, 1));
  const uint64_t n = (K + cap - 1) / cap;
  return n ? (K + n - 1) / n : 1;
}

}  // namespace shelfi

using namespace shelfi;

extern "C" {

int shelfi_special_primes(uint32_t ring_dim, uint32_t num_towers, const uint64_t* moduli, uint32_t* dnum,
                          uint32_t* alpha, uint32_t* num_special, uint64_t* special, uint64_t* special_roots) {
  if (!moduli || !dnum || !alpha || !num_special || !special || num_towers < 1 ||
      num_towers > (uint32_t)kMaxTowers || ring_dim < 2 || (ring_dim & (ring_dim - 1)))
    return SHELFI_ERR_ARG;
  return guarded([&] {
    uint64_t p[kMaxTowers], r[kMaxTowers];
    special_primes(ring_dim, num_towers, moduli, dnum, alpha, num_special, p, r);
    for (uint32_t i = 0; i < *num_special; ++i) {
      special[i] = p[i];
      if (special_roots) special_roots[i] = r[i];
    }
  });
}

int shelfi_eval_key_info(const shelfi_ctx* ctx, uint32_t* dnum, uint32_t* alpha, uint32_t* num_special,
                         uint64_t* special, int* has_key) {
  if (!ctx || !dnum || !alpha || !num_special) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);
  return guarded([&] {
    uint64_t p[kMaxTowers];
    special_primes(ctx->p.N, ctx->p.L, ctx->p.q, dnum, alpha, num_special, p, nullptr);
    if (special)
      for (uint32_t i = 0; i < *num_special; ++i) special[i] = p[i];
    if (has_key) *has_key = (ctx->ev && ctx->ev->evk) ? 1 : 0;
  });
}

size_t shelfi_eval_key_words(const shelfi_ctx* ctx) {
  if (!ctx) return 0;
  uint32_t dn, al, kP;
  uint64_t p[kMaxTowers];
  special_primes(ctx->p.N, ctx->p.L, ctx->p.q, &dn, &al, &kP, p, nullptr);
  return 2ull * dn * (ctx->p.L + kP) * ctx->p.N;
}

int shelfi_eval_mult_keygen(shelfi_ctx* ctx) {
  if (!ctx) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);
  return guarded([&] {
    require_keys(ctx);
    DeviceGuard g(ctx->device);
    const Params& p = ctx->p;
    EvalState& ev = eval_state(ctx);
    LevelState& l = level(ctx, p.L);
    EvkGenConst gc{};
    gc.q0 = p.q[0];
    uint64_t P[kMaxTowers];
    for (uint32_t t = 0; t < p.L; ++t) {
      P[t] = 1;
      for (uint32_t m = 0; m < ev.kP; ++m) P[t] = mm(P[t], ev.p[m] % p.q[t], p.q[t]);
      gc.pmod[t] = P[t];
    }
    gc.L = p.L;
    gc.kP = ev.kP;
    gc.dnum = ev.dnum;
    gc.alpha = ev.alpha;
    gc.logN = p.logN;
    uint32_t key[8];
    if (ctx->seed)
      seed_to_key(ctx->seed, key);
    else
      os_random(key, 32);
    const size_t words = 2ull * ev.dnum * (p.L + ev.kP) * p.N;
    void* scratch = ensure(ctx->scratch, ctx->scratch_bytes, evk_scratch_bytes(p.L, ev.kP, p.N));
    uint64_t* evk_d = nullptr;
    SHELFI_HIP(hipMalloc((void**)&evk_d, words * 8));
    std::vector<uint64_t> host(words);
    try {
      launch_evk_keygen(gc, ctx->dt, l.ext, ctx->dt.cdt, ctx->dt.cdt_len, key, ctx->dk.sk, evk_d, scratch,
                        ctx->stream);
      SHELFI_HIP(hipMemcpyAsync(host.data(), evk_d, words * 8, hipMemcpyDeviceToHost, ctx->stream));
      SHELFI_HIP(hipStreamSynchronize(ctx->stream));
    } catch (...) {
      (void)hipFree(evk_d);
      throw;
    }
    (void)hipFree(evk_d);
    std::memset(key, 0, sizeof(key));
    install_evk(ctx, ev, host.data());
  });
}

int shelfi_get_eval_key(const shelfi_ctx* ctx, uint64_t* evk) {
  if (!ctx || !evk) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);  // against a concurrent keygen / load replacing it
  if (!ctx->ev || ctx->ev->evk_host.empty()) {
    set_error("no evaluation key: call shelfi_eval_mult_keygen first");
    return SHELFI_ERR_STATE;
  }
  std::memcpy(evk, ctx->ev->evk_host.data(), ctx->ev->evk_host.size() * 8);
  return SHELFI_OK;
}

int shelfi_set_eval_key(shelfi_ctx* ctx, const uint64_t* evk) {
  if (!ctx || !evk) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);
  return guarded([&] {
    DeviceGuard g(ctx->device);
    install_evk(ctx, eval_state(ctx), evk);
  });
}

int shelfi_palisade_evalkey_parse(const uint8_t* file, size_t len, shelfi_palisade_evk_info* info,
                                  uint64_t* polys) {
  if (!file || !info) return SHELFI_ERR_ARG;
  return guarded([&] {
    const PalisadeEvalKey K = palisade_parse_evalmult_key(file, len);
    std::memset(info, 0, sizeof(*info));
    info->ring_dim = K.N;
    info->num_towers = K.T;
    info->ctx_towers = K.ctx.L;
    info->dnum = K.dnum;
    for (uint32_t t = 0; t < K.T; ++t) {
      info->moduli[t] = K.q[t];
      info->roots[t] = K.psi[t];
    }
    std::memcpy(info->keytag, K.keytag.data(), std::min<size_t>(K.keytag.size(), 256));
    if (polys)
      for (size_t i = 0; i < K.tower_off.size(); ++i)
        std::memcpy(polys + i * (size_t)K.N, file + K.tower_off[i], (size_t)K.N * 8);
  });
}

int shelfi_palisade_evalkey_rewrite(const uint8_t* file, size_t len, const uint64_t* polys, uint8_t** out,
                                    size_t* out_len) {
  if (!file || !polys || !out || !out_len) return SHELFI_ERR_ARG;
  *out = nullptr;
  *out_len = 0;
  return guarded([&] {
    const PalisadeEvalKey K = palisade_parse_evalmult_key(file, len);
    const std::string w = palisade_evalmult_key_file(K, polys);
    uint8_t* buf = (uint8_t*)std::malloc(w.size());
    if (!buf) throw std::bad_alloc();
    std::memcpy(buf, w.data(), w.size());
    *out = buf;
    *out_len = w.size();
  });
}

int shelfi_save_eval_key(const shelfi_ctx* ctx, const char* path) {
  if (!ctx || !path) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);
  return guarded([&] {
    if (!ctx->ev || ctx->ev->evk_host.empty())
      throw Error{SHELFI_ERR_STATE, "no evaluation key: call evalMultKeyGen() first"};
    const std::string w = palisade_evalmult_key_file(evalkey_meta(ctx, *ctx->ev), ctx->ev->evk_host.data());
    std::ofstream f(path, std::ios::binary);
    if (!f || !f.write(w.data(), (std::streamsize)w.size()))
      throw Error{SHELFI_ERR_IO, std::string("cannot write ") + path};
  });
}

int shelfi_load_eval_key(shelfi_ctx* ctx, const char* path) {
  if (!ctx || !path) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);
  return guarded([&] {
    DeviceGuard g(ctx->device);
    load_evalkey(ctx, slurp(path));
  });
}

int shelfi_dev_mult(shelfi_ctx* ctx, const uint64_t* a_dev, const uint64_t* b_dev, size_t K, uint32_t towers,
                    uint64_t* out_dev, void* stream) {
  if (!ctx || (K && (!a_dev || !b_dev || !out_dev))) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);
  return guarded([&] {
    DeviceGuard g(ctx->device);
    if (!ctx->ev || !ctx->ev->evk)
      throw Error{SHELFI_ERR_STATE, "no evaluation key: call evalMultKeyGen() first"};
    LevelState& l = level(ctx, towers);
    if (!K) return;
    // out may alias a or b exactly (each workgroup reads its inputs before writing that
    // ciphertext's output); a shifted overlap would let one chunk's writes corrupt inputs
    // another has not read yet
    const uint64_t words = 2ull * towers * ctx->p.N * K;
    for (const uint64_t* in : {a_dev, b_dev})
      if (out_dev != in && out_dev < in + words && in < out_dev + words)
        throw Error{SHELFI_ERR_ARG, "EvalMult output must be an input exactly or not overlap the inputs"};
    const KsArgs& a = l.args;
    const uint32_t N = ctx->p.N;
    hipStream_t s = (hipStream_t)stream;
    const uint64_t kc_max = chunk_of(K, ks_scratch_bytes(a.Ll, a.kP, a.dn, a.alpha, N, 1));
    void* scratch =
        ensure(ctx->scratch, ctx->scratch_bytes, ks_scratch_bytes(a.Ll, a.kP, a.dn, a.alpha, N, kc_max));
    const uint64_t ctw = 2ull * towers * N;
    for (uint64_t k0 = 0; k0 < K; k0 += kc_max) {
      const uint64_t kc = std::min<uint64_t>(kc_max, K - k0);
      launch_eval_mult(a, ctx->dt, l.ext, l.dtf, ctx->ev->evk, ctx->ev->evk_sh, a_dev + k0 * ctw,
                       b_dev + k0 * ctw, kc, out_dev + k0 * ctw, scratch, s);
    }
    SHELFI_HIP(hipStreamSynchronize(s));  // scratch is reused by the next call
  });
}

int shelfi_dev_rescale(shelfi_ctx* ctx, const uint64_t* in_dev, size_t K, uint32_t towers, uint64_t* out_dev,
                       void* stream) {
  if (!ctx || (K && (!in_dev || !out_dev))) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);
  return guarded([&] {
    DeviceGuard g(ctx->device);
    const Params& p = ctx->p;
    if (towers < 2 || towers > p.L) throw Error{SHELFI_ERR_ARG, "ModReduce needs 2..L towers"};
    if (!K) return;
    const uint64_t in_words = 2ull * towers * p.N * K, out_words = 2ull * (towers - 1) * p.N * K;
    if (out_dev < in_dev + in_words && in_dev < out_dev + out_words)
      throw Error{SHELFI_ERR_ARG, "ModReduce input and output must not overlap"};
    RescaleConst rc{};
    rc.ql = p.q[towers - 1];
    for (uint32_t t = 0; t + 1 < towers; ++t) {
      rc.qlinv[t] = invmod(rc.ql % p.q[t], p.q[t]);
      rc.qlinv_sh[t] = shoup(rc.qlinv[t], p.q[t]);
    }
    hipStream_t s = (hipStream_t)stream;
    const uint64_t kc_max = chunk_of(K, rescale_scratch_bytes(towers, p.N, 1));
    void* scratch = ensure(ctx->scratch, ctx->scratch_bytes, rescale_scratch_bytes(towers, p.N, kc_max));
    for (uint64_t k0 = 0; k0 < K; k0 += kc_max) {
      const uint64_t kc = std::min<uint64_t>(kc_max, K - k0);
      launch_rescale(ctx->dt, towers, p.logN, rc, in_dev + k0 * 2ull * towers * p.N, kc,
                     out_dev + k0 * 2ull * (towers - 1) * p.N, scratch, s);
    }
    SHELFI_HIP(hipStreamSynchronize(s));
  });
}

}  // extern "C"

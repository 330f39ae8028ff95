// palisade_codec.cpp — PALISADE 1.11 vector<Ciphertext<DCRTPoly>> archives (see
// palisade_codec.h for the grammar).  Written from the cereal PortableBinary encoding
// rules and the reference's committed archives (CT1.txt, key-*.txt), not from
// PALISADE or cereal sources, which are not available here.
#include "palisade_codec.h"

#include <algorithm>
#include <cstring>

#include "shelfi_internal.h"

namespace shelfi {

namespace {

constexpr uint32_t kPoly = 0x40000000u;  // cereal: polymorphic pointer of the static type
constexpr uint32_t kNew = 0x80000000u;   // cereal: first occurrence of a shared pointer

[[noreturn]] void bad(const std::string& what) {
  throw Error{SHELFI_ERR_FORMAT, "PALISADE archive: " + what};
}

struct Cursor {
  const uint8_t* b;
  size_t len, p;
  void need(size_t n) const {
    if (p + n > len) bad("truncated");
  }
  template <class T>
  T get() {
    need(sizeof(T));
    T v;
    std::memcpy(&v, b + p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  uint32_t u32() { return get<uint32_t>(); }
  uint64_t u64() { return get<uint64_t>(); }
  void expect32(uint32_t v, const char* what) {
    if (u32() != v) bad(what);
  }
};

bool is_hex_tag(const uint8_t* s, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    const uint8_t c = s[i];
    if (!((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f'))) return false;
  }
  return true;
}

// Start of the key tag (u64 n | n hex chars | u64 2) after a context object at `from`.
size_t find_keytag(const uint8_t* b, size_t len, size_t from) {
  for (size_t p = from; p + 16 <= len; ++p) {
    uint64_t n;
    std::memcpy(&n, b + p, 8);
    if (n < 8 || n > 256 || p + 8 + n + 8 > len) continue;
    if (!is_hex_tag(b + p + 8, (size_t)n)) continue;
    uint64_t two;
    std::memcpy(&two, b + p + 8 + n, 8);
    if (two == 2) return p;
  }
  bad("no key tag after the context");
}

// New shared-pointer id sites inside a context object: a u32 with bit 31 set right
// after the polymorphic marker, or right after a polymorphic type-name record
// (u64 length | "lbcrypto::..."); returned in order of position.
std::vector<size_t> ptr_id_sites(const std::string& s) {
  std::vector<size_t> sites;
  auto rd32 = [&](size_t p) {
    uint32_t v;
    std::memcpy(&v, s.data() + p, 4);
    return v;
  };
  for (size_t p = 4; p + 4 <= s.size(); ++p) {
    if (rd32(p - 4) != kPoly) continue;
    const uint32_t v = rd32(p);
    if ((v & kNew) && (v & ~kNew) >= 1 && (v & ~kNew) < (1u << 20)) sites.push_back(p);
  }
  for (size_t s0 = s.find("lbcrypto::"); s0 != std::string::npos; s0 = s.find("lbcrypto::", s0 + 1)) {
    if (s0 < 8) continue;
    uint64_t n;
    std::memcpy(&n, s.data() + s0 - 8, 8);
    if (n < 10 || n > 512 || s0 + n + 4 > s.size()) continue;
    const size_t e = s0 + (size_t)n;
    const uint32_t v = rd32(e);
    if ((v & kNew) && (v & ~kNew) >= 1 && (v & ~kNew) < (1u << 20)) sites.push_back(e);
  }
  std::sort(sites.begin(), sites.end());
  sites.erase(std::unique(sites.begin(), sites.end()), sites.end());
  return sites;
}

// Ids of a context object: must be first, first+1, ... (cereal numbering).
std::vector<uint32_t> context_ids(const std::string& obj, uint32_t first) {
  std::vector<uint32_t> ids;
  for (size_t p : ptr_id_sites(obj)) {
    uint32_t v;
    std::memcpy(&v, obj.data() + p, 4);
    ids.push_back(v & ~kNew);
  }
  for (size_t i = 0; i < ids.size(); ++i)
    if (ids[i] != first + i) bad("context shared-pointer ids are not sequential");
  if (ids.size() < 4) bad("context object too small");
  return ids;
}

constexpr const char* kParamsName = "lbcrypto::LPCryptoParametersCKKS<lbcrypto::DCRTPoly>";
constexpr const char* kSchemeName = "lbcrypto::LPPublicKeyEncryptionSchemeCKKS<lbcrypto::DCRTPoly>";

struct Out {
  std::string s;
  void put(const void* v, size_t n) { s.append((const char*)v, n); }
  void u8(uint8_t v) { put(&v, 1); }
  void u16(uint16_t v) { put(&v, 2); }
  void u32(uint32_t v) { put(&v, 4); }
  void u64(uint64_t v) { put(&v, 8); }
  void f32(float v) { put(&v, 4); }
  void str(const std::string& v) {
    u64(v.size());
    s += v;
  }
};

// prod(q) as little-endian u32 limbs
std::vector<uint32_t> modulus_product(const std::vector<uint64_t>& q) {
  std::vector<uint32_t> r{1};
  for (uint64_t x : q) {
    const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    std::vector<uint32_t> t(r.size() + 2, 0);
    for (int half = 0; half < 2; ++half) {
      const uint64_t m = half ? hi : lo;
      uint64_t carry = 0;
      size_t i = 0;
      for (; i < r.size(); ++i) {
        const uint64_t v = (uint64_t)r[i] * m + t[i + half] + carry;
        t[i + half] = (uint32_t)v;
        carry = v >> 32;
      }
      for (size_t j = i + half; carry; ++j) {
        const uint64_t v = (uint64_t)t[j] + carry;
        t[j] = (uint32_t)v;
        carry = v >> 32;
      }
    }
    while (t.size() > 1 && !t.back()) t.pop_back();
    r.swap(t);
  }
  return r;
}

// BigIntegerFixedT<uint32_t, 3500>: limbs most significant first, then u16 bit length
void put_bigint(Out& o, const std::vector<uint32_t>& le, uint32_t nbytes) {
  const size_t nl = (nbytes - 2) / 4;
  size_t used = le.size();
  while (used && !le[used - 1]) --used;
  if (used > nl) bad("modulus product exceeds the BigInteger width");
  for (size_t i = 0; i < nl; ++i) {
    const size_t li = nl - 1 - i;
    o.u32(li < used ? le[li] : 0);
  }
  o.u16(used ? (uint16_t)(32 * (used - 1) + (32 - __builtin_clz(le[used - 1]))) : 0);
}

std::vector<uint32_t> read_bigint(Cursor& c, uint32_t nbytes) {
  const size_t nl = (nbytes - 2) / 4;
  std::vector<uint32_t> le(nl);
  for (size_t i = 0; i < nl; ++i) le[nl - 1 - i] = c.u32();
  c.get<uint16_t>();
  return le;
}

std::string get_str(Cursor& c, size_t max) {
  const uint64_t n = c.u64();
  if (n > max) bad("string length");
  c.need((size_t)n);
  std::string v((const char*)c.b + c.p, (size_t)n);
  c.p += (size_t)n;
  return v;
}

// A tower's ILNativeParams object body (after its pointer id; no class versions)
void put_tower_params(Out& o, uint32_t N, uint64_t q, uint64_t psi) {
  o.u32(2 * N);
  o.u32(N);
  o.u8(1);
  o.u64(q);
  o.u64(psi);
  o.u64(0);
  o.u64(0);
}

// The ILDCRTParams object body (after its pointer id; no class versions) with its
// towers given as references (the form a ciphertext archive uses for the key's
// parameters, whose towers were embedded at the first polynomial's residue vectors)
void put_dcrt_params_refs(Out& o, const PalisadeCtxParams& p, uint32_t tower_id0) {
  o.u32(2 * p.N);
  o.u32(p.N);
  o.u8(1);
  put_bigint(o, modulus_product(p.q), p.bigint_bytes);
  if (p.elem_bigints.size() == 3ull * p.bigint_bytes) {
    o.s += p.elem_bigints;
  } else {
    for (int i = 0; i < 3; ++i) put_bigint(o, {}, p.bigint_bytes);
  }
  o.u64(p.L);
  for (uint32_t t = 0; t < p.L; ++t) {
    o.u32(kPoly);
    o.u32(tower_id0 + t);
  }
  put_bigint(o, {}, p.bigint_bytes);  // originalModulus
}

}  // namespace

PalisadeCtxParams palisade_parse_context_object(const std::string& obj, uint32_t* first_id, uint32_t name0) {
  PalisadeCtxParams p;
  Cursor c{(const uint8_t*)obj.data(), obj.size(), 0};
  if (c.u32() != 1) bad("context version");
  if (c.u32() != (kNew | name0) || get_str(c, 256) != kParamsName) bad("crypto parameters type");
  const uint32_t id = c.u32();
  if (!(id & kNew)) bad("crypto parameters pointer");
  const uint32_t id0 = id & ~kNew;
  for (int i = 0; i < 3; ++i) c.u32();  // class versions
  c.expect32(kPoly, "element parameters pointer");
  if (c.u32() != (kNew | (id0 + 1))) bad("element parameters id");
  c.u32();
  c.u32();
  const uint32_t M = c.u32();
  p.N = c.u32();
  if (p.N < 2 || p.N > (1u << 17) || (p.N & (p.N - 1)) || M != 2 * p.N) bad("context ring dimension");
  c.get<uint8_t>();
  c.u32();  // BigInteger version
  // BigInteger width: the four element BigIntegers are followed by u64 L and the
  // first tower's new pointer
  uint32_t B = 0;
  for (uint32_t b = 10; b <= 4096; b += 4) {
    const size_t at = c.p + 4ull * b;
    if (at + 16 > obj.size()) break;
    uint64_t L;
    uint32_t m, t0;
    std::memcpy(&L, obj.data() + at, 8);
    std::memcpy(&m, obj.data() + at + 8, 4);
    std::memcpy(&t0, obj.data() + at + 12, 4);
    if (L >= 1 && L <= 64 && m == kPoly && t0 == (kNew | (id0 + 2))) {
      B = b;
      break;
    }
  }
  if (!B) bad("context BigInteger layout");
  p.bigint_bytes = B;
  const std::vector<uint32_t> Q = read_bigint(c, B);
  c.need(3ull * B);
  p.elem_bigints.assign(obj.data() + c.p, 3ull * B);
  c.p += 3ull * B;
  const uint64_t L = c.u64();
  if (L < 1 || L > (uint64_t)kMaxTowers) bad("context tower count");
  p.L = (uint32_t)L;
  for (uint32_t t = 0; t < p.L; ++t) {
    c.expect32(kPoly, "tower parameters pointer");
    if (c.u32() != (kNew | (id0 + 2 + t))) bad("tower parameters id");
    if (t == 0) {
      c.u32();
      c.u32();
    }
    if (c.u32() != M || c.u32() != p.N) bad("tower ring dimension");
    c.get<uint8_t>();
    if (t == 0) c.u32();  // NativeInteger version
    p.q.push_back(c.u64());
    p.psi.push_back(c.u64());
    c.u64();
    c.u64();
  }
  read_bigint(c, B);  // originalModulus
  c.expect32(kPoly, "encoding parameters pointer");
  if (c.u32() != (kNew | (id0 + 2 + p.L))) bad("encoding parameters id");
  c.u32();
  p.plaintext_modulus = c.u64();
  c.u64();
  c.u64();
  c.u64();
  c.u32();
  p.batch = c.u32();
  p.sigma = c.get<float>();
  p.assurance = c.get<float>();
  p.root_hermite = c.get<float>();
  p.fields.clear();
  for (;;) {
    const uint32_t v = c.u32();
    if (v == (kNew | (name0 + 1))) break;
    p.fields.push_back(v);
    if (p.fields.size() > 16) bad("crypto parameter fields");
  }
  if (get_str(c, 256) != kSchemeName) bad("scheme type");
  if (c.u32() != (kNew | (id0 + 3 + p.L))) bad("scheme id");
  c.u32();
  c.u32();
  p.enabled = c.u32();
  if (get_str(c, 64) != "CKKS") bad("scheme id string");
  if (c.p != obj.size()) bad("trailing bytes after the context");
  if (modulus_product(p.q) != [&] {
        std::vector<uint32_t> q = Q;
        while (q.size() > 1 && !q.back()) q.pop_back();
        return q;
      }())
    bad("context modulus is not the product of the towers");
  if (first_id) *first_id = id0;
  return p;
}

std::string palisade_context_object(const PalisadeCtxParams& p, uint32_t id0, uint32_t name0) {
  if (p.L < 1 || p.q.size() != p.L || p.psi.size() != p.L) bad("context parameters");
  Out o;
  o.u32(1);  // CryptoContextImpl version
  o.u32(kNew | name0);
  o.str(kParamsName);
  o.u32(kNew | id0);
  for (int i = 0; i < 3; ++i) o.u32(0);
  o.u32(kPoly);
  o.u32(kNew | (id0 + 1));
  o.u32(1);
  o.u32(1);
  o.u32(2 * p.N);
  o.u32(p.N);
  o.u8(1);
  o.u32(1);  // BigInteger version
  put_bigint(o, modulus_product(p.q), p.bigint_bytes);
  if (p.elem_bigints.size() == 3ull * p.bigint_bytes) {
    o.s += p.elem_bigints;
  } else {
    for (int i = 0; i < 3; ++i) put_bigint(o, {}, p.bigint_bytes);
  }
  o.u64(p.L);
  for (uint32_t t = 0; t < p.L; ++t) {
    o.u32(kPoly);
    o.u32(kNew | (id0 + 2 + t));
    if (t == 0) {
      o.u32(1);
      o.u32(1);
    }
    o.u32(2 * p.N);
    o.u32(p.N);
    o.u8(1);
    if (t == 0) o.u32(1);  // NativeInteger version
    o.u64(p.q[t]);
    o.u64(p.psi[t]);
    o.u64(0);
    o.u64(0);
  }
  put_bigint(o, {}, p.bigint_bytes);  // originalModulus
  o.u32(kPoly);
  o.u32(kNew | (id0 + 2 + p.L));
  o.u32(1);
  o.u64(p.plaintext_modulus);
  o.u64(0);
  o.u64(0);
  o.u64(0);
  o.u32(0);
  o.u32(p.batch);
  o.f32(p.sigma);
  o.f32(p.assurance);
  o.f32(p.root_hermite);
  for (uint32_t v : p.fields) o.u32(v);
  o.u32(kNew | (name0 + 1));
  o.str(kSchemeName);
  o.u32(kNew | (id0 + 3 + p.L));
  o.u32(0);
  o.u32(0);
  o.u32(p.enabled);
  o.str("CKKS");
  return o.s;
}

PalisadeCtxParams palisade_parse_context_file(const std::string& f) {
  uint32_t a, id, id0 = 0;
  if (f.size() < 64 || (uint8_t)f[0] != 0x01) bad("context file");
  std::memcpy(&a, f.data() + 1, 4);
  std::memcpy(&id, f.data() + 5, 4);
  if (a != kPoly || id != (kNew | 1u)) bad("context file header");
  PalisadeCtxParams p = palisade_parse_context_object(f.substr(9), &id0);
  if (id0 != 2) bad("context file ids");
  return p;
}

std::string palisade_context_file(const PalisadeCtxParams& p) {
  Out o;
  o.u8(0x01);
  o.u32(kPoly);
  o.u32(kNew | 1u);
  o.s += palisade_context_object(p, 2);
  return o.s;
}

std::string palisade_key_file(const PalisadeCtxParams& p, const std::string& keytag,
                              const uint64_t* polys, bool is_public) {
  const uint32_t N = p.N, L = p.L;
  Out o;
  o.u8(0x01);
  o.u32(kPoly);
  o.u32(kNew | 1u);
  for (int i = 0; i < 3; ++i) o.u32(0);  // LPPublicKeyImpl / LPPrivateKeyImpl, LPKey, CryptoObject
  o.u32(kPoly);
  o.u32(kNew | 2u);
  o.s += palisade_context_object(p, 3);
  o.str(keytag);
  const int nelem = is_public ? 2 : 1;
  if (is_public) o.u64(2);
  o.s.reserve(o.s.size() + (size_t)nelem * L * (N * 8 + 64) + 64);
  for (int e = 0; e < nelem; ++e) {
    if (e == 0) o.u32(1);  // DCRTPoly version
    o.u64(L);
    for (uint32_t t = 0; t < L; ++t) {
      if (e == 0 && t == 0) o.u32(1);  // PolyImpl version
      o.u32(kPoly);
      o.u8(0x01);
      if (e == 0 && t == 0) o.u32(1);  // NativeVector version
      o.u64(N);
      o.put(polys + ((size_t)e * L + t) * N, (size_t)N * 8);
      o.u64(p.q[t]);
      o.u32(0);  // EVALUATION
      o.u32(kPoly);
      o.u32(5 + t);  // the context's tower parameters (ids from 3: params, element, towers)
    }
    o.u32(0);
    o.u32(kPoly);
    o.u32(4);
  }
  return o.s;
}

bool palisade_looks_like_archive(const uint8_t* b, size_t len) {
  if (len < 9 || b[0] != 0x01) return false;
  uint32_t w;
  std::memcpy(&w, b + 1, 4);
  if (w == kPoly) return true;  // a single Ciphertext
  uint64_t count;
  std::memcpy(&count, b + 1, 8);
  if (count == 0) return len == 9;
  if (count > (1ull << 32) || len < 13) return false;
  std::memcpy(&w, b + 9, 4);
  return w == kPoly;
}

PalisadeArchive palisade_parse_archive(const uint8_t* b, size_t len) {
  PalisadeArchive A;
  Cursor c{b, len, 0};
  if (c.get<uint8_t>() != 0x01) bad("not a little-endian PortableBinary archive");
  uint32_t w;
  c.need(4);
  std::memcpy(&w, b + 1, 4);
  A.vector_archive = (w != kPoly);
  A.K = A.vector_archive ? c.u64() : 1;
  if (A.K > (1ull << 32)) bad("ciphertext count");
  bool seen_ct = false, seen_dcrt = false, seen_poly = false, seen_vec = false;
  uint32_t ctx_id = 0, elem_id = 0;
  std::vector<uint32_t> tower_ids;
  for (uint64_t k = 0; k < A.K; ++k) {
    c.expect32(kPoly, "ciphertext pointer");
    if (!(c.u32() & kNew)) bad("shared ciphertext pointers are not supported");
    if (!seen_ct) {
      c.u32();  // CiphertextImpl version
      c.u32();  // CryptoObject version
      seen_ct = true;
    }
    c.expect32(kPoly, "context pointer");
    const uint32_t cid = c.u32();
    if (cid & kNew) {
      if (k) bad("second embedded context");
      ctx_id = cid & ~kNew;
      A.ctx_off = c.p;
      c.p = find_keytag(b, len, c.p);
      A.ctx_len = c.p - A.ctx_off;
      context_ids(std::string((const char*)b + A.ctx_off, A.ctx_len), ctx_id + 1);
    } else if (!ctx_id || cid != ctx_id) {
      bad("context reference");
    }
    const uint64_t tl = c.u64();
    if (tl > 256) bad("key tag length");
    c.need((size_t)tl);
    const std::string tag((const char*)b + c.p, (size_t)tl);
    c.p += (size_t)tl;
    if (k == 0) A.keytag = tag;
    else if (tag != A.keytag) bad("ciphertexts under different keys");
    if (c.u64() != 2) bad("a ciphertext must have 2 elements");
    for (int e = 0; e < 2; ++e) {
      if (!seen_dcrt) {
        c.u32();
        seen_dcrt = true;
      }
      const uint64_t L = c.u64();
      if (L < 1 || L > (uint64_t)kMaxTowers) bad("tower count");
      if (k == 0 && e == 0) {
        A.L = (uint32_t)L;
        A.q.assign(L, 0);
        tower_ids.assign(L, 0);
      } else if (L != A.L) {
        bad("tower count differs between ciphertexts");
      }
      for (uint32_t t = 0; t < A.L; ++t) {
        if (!seen_poly) {
          c.u32();
          seen_poly = true;
        }
        c.expect32(kPoly, "residue vector pointer");
        if (c.get<uint8_t>() != 1) bad("empty residue vector");
        if (!seen_vec) {
          c.u32();
          seen_vec = true;
        }
        const uint64_t N = c.u64();
        if (N < 2 || N > (1u << 17) || (N & (N - 1))) bad("ring dimension");
        if (!A.N) A.N = (uint32_t)N;
        else if (N != A.N) bad("ring dimension differs");
        c.need((size_t)N * 8);
        A.tower_off.push_back(c.p);
        c.p += (size_t)N * 8;
        const uint64_t q = c.u64();
        if (k == 0 && e == 0) A.q[t] = q;
        else if (q != A.q[t]) bad("tower moduli differ");
        if (c.u32() != 0) bad("residues must be in EVALUATION format");
        c.expect32(kPoly, "tower params pointer");
        uint32_t pid = c.u32();
        if (pid & kNew) {  // the key's own tower parameters (palisade_layout key_params)
          if (k || e) bad("tower params object outside the first polynomial");
          pid &= ~kNew;
          if (c.u32() != 2 * A.N || c.u32() != A.N) bad("tower params ring dimension");
          c.get<uint8_t>();
          if (c.u64() != A.q[t]) bad("tower params modulus");
          c.u64();
          c.u64();
          c.u64();
        }
        if (k == 0 && e == 0) tower_ids[t] = pid;
        else if (pid != tower_ids[t]) bad("tower params reference");
      }
      if (c.u32() != 0) bad("element must be in EVALUATION format");
      c.expect32(kPoly, "element params pointer");
      uint32_t eid = c.u32();
      if (eid & kNew) {  // the key's own ILDCRTParams: towers by reference
        if (k || e) bad("element params object outside the first polynomial");
        eid &= ~kNew;
        if (!ctx_id || !A.ctx_len) bad("element params before the context");
        const PalisadeCtxParams cp = palisade_parse_context_object(
            std::string((const char*)b + A.ctx_off, A.ctx_len), nullptr);
        if (c.u32() != 2 * A.N || c.u32() != A.N) bad("element params ring dimension");
        c.get<uint8_t>();
        c.need(4ull * cp.bigint_bytes);
        c.p += 4ull * cp.bigint_bytes;
        if (c.u64() != A.L) bad("element params tower count");
        for (uint32_t t = 0; t < A.L; ++t) {
          c.expect32(kPoly, "element params tower pointer");
          if (c.u32() != tower_ids[t]) bad("element params tower reference");
        }
        c.need(cp.bigint_bytes);
        c.p += cp.bigint_bytes;
      }
      if (k == 0 && e == 0) elem_id = eid;
      else if (eid != elem_id) bad("element params reference");
    }
    const uint64_t depth = c.u64(), level = c.u64();
    const double scale = c.get<double>();
    const uint32_t enc = c.u32();
    if (k == 0) {
      A.depth = depth;
      A.level = level;
      A.scale = scale;
      A.encoding = enc;
    } else if (depth != A.depth || level != A.level || scale != A.scale || enc != A.encoding) {
      bad("ciphertexts with different depth / level / scale / encoding");
    }
    const uint32_t mid = c.u32();
    if (mid & kNew) {
      if (c.u64() != 0) bad("non-empty ciphertext metadata is not supported");
    }
  }
  if (c.p != len) bad("trailing bytes");
  // residues >= q are refused by the aggregation (wavg_kernel<false, true>); decrypt of a
  // malformed archive only yields a meaningless decode
  return A;
}

std::vector<size_t> palisade_layout(const std::string& ctx_obj, const std::string& keytag,
                                    uint32_t N, uint32_t L, const uint64_t* q, uint64_t K,
                                    uint64_t depth, uint64_t level, double scale, uint32_t encoding,
                                    bool vector_archive, bool key_params, uint8_t* buf,
                                    size_t* total) {
  if (!vector_archive && K != 1) bad("a single-ciphertext archive holds exactly one ciphertext");
  const std::vector<uint32_t> ids = context_ids(ctx_obj, 3);
  if (ids.size() < 2 + (size_t)L) bad("context has fewer tower parameter sets than towers");
  const uint32_t nctx = (uint32_t)ids.size(), elem_id = ids[1];
  PalisadeCtxParams kp;
  if (key_params) {
    uint32_t id0 = 0;
    kp = palisade_parse_context_object(ctx_obj, &id0);
    if (id0 != 3 || kp.N != N || kp.L != L) bad("context does not match the ciphertext parameters");
    for (uint32_t t = 0; t < L; ++t)
      if (kp.q[t] != q[t]) bad("context moduli do not match the ciphertext parameters");
  }
  // ids after the context: [the key's tower params x L, its ILDCRTParams], then per
  // ciphertext its metadata map (first) or pointer + metadata map (later ones)
  const uint32_t kid0 = 3 + nctx, extra = key_params ? L + 1 : 0;
  size_t pos = 0;
  auto put = [&](const void* v, size_t n) {
    if (buf) std::memcpy(buf + pos, v, n);
    pos += n;
  };
  auto p8 = [&](uint8_t v) { put(&v, 1); };
  auto p32 = [&](uint32_t v) { put(&v, 4); };
  auto p64 = [&](uint64_t v) { put(&v, 8); };
  std::string tower_obj[kMaxTowers], elem_obj;
  if (key_params) {
    for (uint32_t t = 0; t < L; ++t) {
      Out o;
      put_tower_params(o, N, kp.q[t], kp.psi[t]);
      tower_obj[t] = std::move(o.s);
    }
    Out o;
    put_dcrt_params_refs(o, kp, kid0);
    elem_obj = std::move(o.s);
  }
  std::vector<size_t> off;
  off.reserve(K * 2 * L);
  p8(0x01);
  if (vector_archive) p64(K);
  for (uint64_t k = 0; k < K; ++k) {
    const bool first = (k == 0);
    p32(kPoly);
    p32(kNew | (first ? 1u : (uint32_t)(2 + nctx + 2 * k + extra)));
    if (first) {
      p32(1);  // CiphertextImpl version (CT1.txt)
      p32(0);  // CryptoObject version
    }
    p32(kPoly);
    if (first) {
      p32(kNew | 2u);
      put(ctx_obj.data(), ctx_obj.size());
    } else {
      p32(2u);
    }
    p64(keytag.size());
    put(keytag.data(), keytag.size());
    p64(2);
    for (int e = 0; e < 2; ++e) {
      const bool embed = key_params && first && e == 0;
      if (first && e == 0) p32(1);  // DCRTPoly version
      p64(L);
      for (uint32_t t = 0; t < L; ++t) {
        if (first && e == 0 && t == 0) p32(1);  // PolyImpl version
        p32(kPoly);
        p8(0x01);
        if (first && e == 0 && t == 0) p32(1);  // NativeVector version
        p64(N);
        off.push_back(pos);
        pos += (size_t)N * 8;  // residues: written by the caller
        p64(q[t]);
        p32(0);  // EVALUATION
        p32(kPoly);
        if (embed) {
          p32(kNew | (kid0 + t));
          put(tower_obj[t].data(), tower_obj[t].size());
        } else {
          p32(key_params ? kid0 + t : ids[2 + t]);
        }
      }
      p32(0);
      p32(kPoly);
      if (embed) {
        p32(kNew | (kid0 + L));
        put(elem_obj.data(), elem_obj.size());
      } else {
        p32(key_params ? kid0 + L : elem_id);
      }
    }
    p64(depth);
    p64(level);
    put(&scale, 8);
    p32(encoding);
    p32(kNew | (uint32_t)(3 + nctx + 2 * k + extra));  // metadata map, empty
    p64(0);
  }
  *total = pos;
  return off;
}

void palisade_key_context(const std::string& pub, std::string& ctx_obj, std::string& keytag) {
  const uint8_t* b = (const uint8_t*)pub.data();
  Cursor c{b, pub.size(), 0};
  if (c.get<uint8_t>() != 0x01) bad("public key archive");
  c.expect32(kPoly, "public key pointer");
  if (c.u32() != (kNew | 1u)) bad("public key pointer id");
  // class versions of LPPublicKeyImpl and its bases, then the context pointer
  for (int i = 0; i < 8; ++i) {
    const uint32_t v = c.u32();
    if (v == kPoly) break;
    if (i == 7) bad("public key header");
  }
  if (c.u32() != (kNew | 2u)) bad("public key context id");
  const size_t start = c.p, tag = find_keytag(b, pub.size(), start);
  ctx_obj.assign(pub.data() + start, tag - start);
  context_ids(ctx_obj, 3);
  uint64_t n;
  std::memcpy(&n, b + tag, 8);
  keytag.assign(pub.data() + tag + 8, (size_t)n);
}

std::string palisade_embed_context(const std::string& f) {
  uint32_t a, id;
  if (f.size() < 64 || (uint8_t)f[0] != 0x01) bad("context file");
  std::memcpy(&a, f.data() + 1, 4);
  std::memcpy(&id, f.data() + 5, 4);
  if (a != kPoly || id != (kNew | 1u)) bad("context file header");
  std::string obj = f.substr(9);
  const std::vector<size_t> sites = ptr_id_sites(obj);
  context_ids(obj, 2);
  for (size_t p : sites) {
    uint32_t v;
    std::memcpy(&v, obj.data() + p, 4);
    v += 1;
    std::memcpy(&obj[p], &v, 4);
  }
  return obj;
}


// ------------------------------------------------ evaluation-key files (§8 f4) ----
namespace {
constexpr const char* kEvalKeyName = "lbcrypto::LPEvalKeyRelinImpl<lbcrypto::DCRTPoly>";
}

PalisadeEvalKey palisade_parse_evalmult_key(const uint8_t* b, size_t len) {
  PalisadeEvalKey K;
  Cursor c{b, len, 0};
  if (c.get<uint8_t>() != 0x01) bad("not a little-endian PortableBinary archive");
  if (c.u64() != 1) bad("evaluation-key map must hold one key tag");
  K.keytag = get_str(c, 256);
  if (c.u64() != 1) bad("evaluation-key vector must hold one key");
  if (c.u32() != (kNew | 1u) || get_str(c, 256) != kEvalKeyName) bad("evaluation key type");
  if (c.u32() != (kNew | 1u)) bad("evaluation key pointer");
  for (int i = 0; i < 4; ++i) K.key_versions[i] = c.u32();
  c.expect32(kPoly, "context pointer");
  if (c.u32() != (kNew | 2u)) bad("context id");
  // the context object ends at its "CKKS" scheme id string, followed by the key tag
  const size_t ctx0 = c.p;
  size_t ctx1 = std::string::npos;
  for (size_t p = ctx0; p + 12 <= len; ++p)
    if (std::memcmp(b + p, "\x04\0\0\0\0\0\0\0CKKS", 12) == 0) {
      ctx1 = p + 12;
      break;
    }
  if (ctx1 == std::string::npos) bad("context object end");
  K.ctx_obj.assign((const char*)b + ctx0, ctx1 - ctx0);
  uint32_t id0 = 0;
  K.ctx = palisade_parse_context_object(K.ctx_obj, &id0, 2);
  if (id0 != 3) bad("context ids");
  c.p = ctx1;
  if (get_str(c, 256) != K.keytag) bad("key tag differs from the map's");
  if (c.u64() != 2) bad("relinearization key must be (b, a) vectors");
  const uint32_t next_id = id0 + 4 + K.ctx.L;  // first id after the context's objects
  uint32_t dcrt_id = 0;
  for (int v = 0; v < 2; ++v) {
    const uint64_t dn = c.u64();
    if (dn < 1 || dn > 8 || (v == 1 && dn != K.dnum)) bad("digit count");
    K.dnum = (uint32_t)dn;
    for (uint32_t j = 0; j < K.dnum; ++j) {
      const bool first = v == 0 && j == 0;
      if (first) K.poly_versions[0] = c.u32();
      const uint64_t T = c.u64();
      if (T < 1 || T > (uint64_t)kMaxTowers || (!first && T != K.T)) bad("tower count");
      K.T = (uint32_t)T;
      for (uint32_t t = 0; t < K.T; ++t) {
        if (first && t == 0) K.poly_versions[1] = c.u32();
        c.expect32(kPoly, "residue vector pointer");
        if (c.get<uint8_t>() != 0x01) bad("residue vector marker");
        if (first && t == 0) K.poly_versions[2] = c.u32();
        const uint64_t N = c.u64();
        if (N < 2 || N > (1u << 17) || (N & (N - 1)) || (K.N && N != K.N)) bad("ring dimension");
        K.N = (uint32_t)N;
        c.need((size_t)N * 8);
        K.tower_off.push_back(c.p);
        c.p += (size_t)N * 8;
        const uint64_t q = c.u64();
        if (c.u32() != 0) bad("key polynomials must be in EVALUATION format");
        c.expect32(kPoly, "tower parameters pointer");
        const uint32_t pid = c.u32();
        if (first) {
          if (pid != (kNew | (next_id + t))) bad("tower parameters id");
          if (c.u32() != 2 * N || c.u32() != N || c.get<uint8_t>() != 1) bad("tower parameters");
          if (c.u64() != q) bad("tower parameters modulus");
          K.psi.push_back(c.u64());
          c.u64();
          c.u64();
          K.q.push_back(q);
        } else {
          if (pid != next_id + t || q != K.q[t]) bad("tower parameters reference");
        }
      }
      if (c.u32() != 0) bad("key polynomials must be in EVALUATION format");
      c.expect32(kPoly, "element parameters pointer");
      const uint32_t pid = c.u32();
      if (first) {
        dcrt_id = next_id + K.T;
        if (pid != (kNew | dcrt_id)) bad("element parameters id");
        if (c.u32() != 2 * K.N || c.u32() != K.N || c.get<uint8_t>() != 1) bad("element parameters");
        const uint32_t B = K.ctx.bigint_bytes;
        if (read_bigint(c, B) != [&] {
              std::vector<uint32_t> m = modulus_product(K.q);
              m.resize((B - 2) / 4, 0);
              return m;
            }())
          bad("element modulus is not the product of the key's towers");
        c.need(3ull * B);
        K.elem_bigints.assign((const char*)b + c.p, 3ull * B);
        c.p += 3ull * B;
        if (c.u64() != K.T) bad("element tower count");
        for (uint32_t t = 0; t < K.T; ++t) {
          c.expect32(kPoly, "element tower pointer");
          if (c.u32() != next_id + t) bad("element tower reference");
        }
        read_bigint(c, B);  // originalModulus
      } else if (pid != dcrt_id) {
        bad("element parameters reference");
      }
    }
  }
  if (c.p != len) bad("trailing bytes after the evaluation key");
  // Q's towers lead the key's (Q u P), the special towers follow
  if (K.T <= K.ctx.L) bad("no special towers");
  for (uint32_t t = 0; t < K.ctx.L; ++t)
    if (K.q[t] != K.ctx.q[t]) bad("key towers do not start with the context's");
  return K;
}

std::string palisade_evalmult_key_file(const PalisadeEvalKey& K, const uint64_t* polys) {
  const uint32_t N = K.N, T = K.T, B = K.ctx.bigint_bytes;
  if (K.q.size() != T || K.psi.size() != T || K.dnum < 1) bad("evaluation key parameters");
  Out o;
  o.u8(0x01);
  o.u64(1);
  o.str(K.keytag);
  o.u64(1);
  o.u32(kNew | 1u);
  o.str(kEvalKeyName);
  o.u32(kNew | 1u);
  for (int i = 0; i < 4; ++i) o.u32(K.key_versions[i]);
  o.u32(kPoly);
  o.u32(kNew | 2u);
  o.s += K.ctx_obj.empty() ? palisade_context_object(K.ctx, 3, 2) : K.ctx_obj;
  o.str(K.keytag);
  o.u64(2);
  const uint32_t next_id = 3 + 4 + K.ctx.L, dcrt_id = next_id + T;
  o.s.reserve(o.s.size() + 2ull * K.dnum * T * ((size_t)N * 8 + 64) + 4096);
  for (int v = 0; v < 2; ++v) {
    o.u64(K.dnum);
    for (uint32_t j = 0; j < K.dnum; ++j) {
      const bool first = v == 0 && j == 0;
      if (first) o.u32(K.poly_versions[0]);
      o.u64(T);
      for (uint32_t t = 0; t < T; ++t) {
        if (first && t == 0) o.u32(K.poly_versions[1]);
        o.u32(kPoly);
        o.u8(0x01);
        if (first && t == 0) o.u32(K.poly_versions[2]);
        o.u64(N);
        o.put(polys + (((size_t)v * K.dnum + j) * T + t) * N, (size_t)N * 8);
        o.u64(K.q[t]);
        o.u32(0);  // EVALUATION
        o.u32(kPoly);
        if (first) {
          o.u32(kNew | (next_id + t));
          put_tower_params(o, N, K.q[t], K.psi[t]);
        } else {
          o.u32(next_id + t);
        }
      }
      o.u32(0);
      o.u32(kPoly);
      if (first) {
        o.u32(kNew | dcrt_id);
        PalisadeCtxParams e = K.ctx;
        e.L = T;
        e.q = K.q;
        e.psi = K.psi;
        e.elem_bigints = K.elem_bigints.size() == 3ull * B ? K.elem_bigints : std::string();
        put_dcrt_params_refs(o, e, next_id);
      } else {
        o.u32(dcrt_id);
      }
    }
  }
  return o.s;
}

}  // namespace shelfi

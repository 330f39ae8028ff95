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

}  // namespace

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
        const uint32_t pid = c.u32();
        if (k == 0 && e == 0) tower_ids[t] = pid;
        else if (pid != tower_ids[t]) bad("tower params reference");
      }
      if (c.u32() != 0) bad("element must be in EVALUATION format");
      c.expect32(kPoly, "element params pointer");
      const uint32_t eid = c.u32();
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
  // every residue below its modulus is checked by the caller on the data it uses
  return A;
}

std::vector<size_t> palisade_layout(const std::string& ctx_obj, const std::string& keytag,
                                    uint32_t N, uint32_t L, const uint64_t* q, uint64_t K,
                                    uint64_t depth, uint64_t level, double scale, uint32_t encoding,
                                    bool vector_archive, uint8_t* buf, size_t* total) {
  if (!vector_archive && K != 1) bad("a single-ciphertext archive holds exactly one ciphertext");
  const std::vector<uint32_t> ids = context_ids(ctx_obj, 3);
  if (ids.size() < 2 + (size_t)L) bad("context has fewer tower parameter sets than towers");
  const uint32_t nctx = (uint32_t)ids.size(), elem_id = ids[1];
  size_t pos = 0;
  auto put = [&](const void* v, size_t n) {
    if (buf) std::memcpy(buf + pos, v, n);
    pos += n;
  };
  auto p8 = [&](uint8_t v) { put(&v, 1); };
  auto p32 = [&](uint32_t v) { put(&v, 4); };
  auto p64 = [&](uint64_t v) { put(&v, 8); };
  std::vector<size_t> off;
  off.reserve(K * 2 * L);
  p8(0x01);
  if (vector_archive) p64(K);
  for (uint64_t k = 0; k < K; ++k) {
    const bool first = (k == 0);
    p32(kPoly);
    p32(kNew | (first ? 1u : (uint32_t)(2 + nctx + 2 * k)));
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
        p32(ids[2 + t]);
      }
      p32(0);
      p32(kPoly);
      p32(elem_id);
    }
    p64(depth);
    p64(level);
    put(&scale, 8);
    p32(encoding);
    p32(kNew | (uint32_t)(3 + nctx + 2 * k));  // metadata map, empty
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

}  // namespace shelfi

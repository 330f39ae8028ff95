// palisade_io.cpp — loads the reference's PALISADE 1.11 key material.
//
// loadCryptoParams (ckks.cpp:11-23) deserializes three cereal PortableBinary files.
// Without the PALISADE/cereal sources only the structure needed here is decoded
// (SURVEY App. A):
//   * per RNS tower the context stores  u32 cyclotomic order (2N) | u32 ring dim (N) |
//     a few flag bytes | u64 modulus q | u64 root of unity psi;
//   * every NativeVector is  u64 length (N) | N x u64 residues | u64 modulus.
// Towers are located by those invariants (q prime, q = 1 mod 2N, psi^N = -1 mod q)
// and key vectors by (length == N, trailing modulus == q_t, all residues < q_t).
#include <cstring>

#include "palisade_codec.h"
#include "palisade_io.h"
#include "shelfi_internal.h"

namespace shelfi {

template <class T>
static T rd(const std::string& s, size_t off) {
  T v;
  std::memcpy(&v, s.data() + off, sizeof(T));
  return v;
}

// A tower as the context stores it: q prime, q = 1 mod 2N, psi a primitive 2N-th root (psi^N = -1).
static bool valid_tower(uint32_t N, uint64_t q, uint64_t psi) {
  return q > 2ull * N && q < (1ull << 60) && q % (2ull * N) == 1 && is_prime(q) && psi < q &&
         powmod(psi, N, q) == q - 1;
}

PalisadeContext palisade_read_context(const std::string& s) {
  if (s.size() < 64 || (uint8_t)s[0] != 0x01 || s.find("lbcrypto::") == std::string::npos)
    throw Error{SHELFI_ERR_FORMAT, "cryptocontext.txt is neither a SHELFI nor a PALISADE context"};
  PalisadeContext pc;
  // the structured grammar first (palisade_codec.h: every tower object in order, whatever the
  // moduli's size -- a 14-bit scale gives a 17-bit last tower, below the scan's guard)
  try {
    const PalisadeCtxParams cp = palisade_parse_context_file(s);
    bool ok = cp.L >= 1 && cp.L <= (uint32_t)kMaxTowers && cp.q.size() == cp.L && cp.psi.size() == cp.L;
    for (uint32_t t = 0; ok && t < cp.L; ++t) ok = valid_tower(cp.N, cp.q[t], cp.psi[t]);
    if (ok) {
      pc.N = cp.N;
      pc.q = cp.q;
      pc.psi = cp.psi;
      return pc;
    }
  } catch (const Error&) {
  }
  // other 1.11 layouts: locate the towers by their invariants (the scan's 2^20 floor on q keeps
  // stray byte patterns out)
  for (size_t off = 0; off + 16 <= s.size(); ++off) {
    const uint32_t M = rd<uint32_t>(s, off), N = rd<uint32_t>(s, off + 4);
    if (N < 1024 || N > (1u << 17) || (N & (N - 1)) || M != 2 * N) continue;
    if (pc.N && N != pc.N) continue;
    for (size_t gap = 0; gap < 12 && off + 8 + gap + 16 <= s.size(); ++gap) {
      const uint64_t q = rd<uint64_t>(s, off + 8 + gap), psi = rd<uint64_t>(s, off + 16 + gap);
      if (q < (1ull << 20) || q >= (1ull << 60) || q % M != 1) continue;
      bool dup = false;
      for (uint64_t x : pc.q) dup |= (x == q);
      if (dup || !is_prime(q) || psi >= q || powmod(psi, N, q) != q - 1) continue;
      pc.N = N;
      pc.q.push_back(q);
      pc.psi.push_back(psi);
      break;
    }
  }
  if (pc.q.empty() || pc.q.size() > (size_t)kMaxTowers)
    throw Error{SHELFI_ERR_FORMAT, "no RNS towers found in the PALISADE context"};
  return pc;
}

static std::vector<std::pair<uint64_t, size_t>> find_vectors(const std::string& s, uint32_t N,
                                                             const std::vector<uint64_t>& q) {
  std::vector<std::pair<uint64_t, size_t>> out;  // (modulus, residue offset)
  size_t off = 0;
  const size_t need = 8 + 8ull * N + 8;
  while (off + need <= s.size()) {
    if (rd<uint64_t>(s, off) == N) {
      const uint64_t mod = rd<uint64_t>(s, off + 8 + 8ull * N);
      bool known = false;
      for (uint64_t x : q) known |= (x == mod);
      if (known) {
        bool ok = true;
        for (uint32_t j = 0; j < N && ok; ++j) ok = rd<uint64_t>(s, off + 8 + 8ull * j) < mod;
        if (ok) {
          out.emplace_back(mod, off + 8);
          off += need;
          continue;
        }
      }
    }
    ++off;
  }
  return out;
}

void palisade_read_keys(const std::string& pub, const std::string& priv, uint32_t N,
                        const std::vector<uint64_t>& q, std::vector<uint64_t>& pk,
                        std::vector<uint64_t>& sk) {
  const size_t L = q.size();
  auto pv = find_vectors(pub, N, q);
  auto sv = find_vectors(priv, N, q);
  if (pv.size() != 2 * L) throw Error{SHELFI_ERR_FORMAT, "PALISADE public key: unexpected layout"};
  if (sv.size() != L) throw Error{SHELFI_ERR_FORMAT, "PALISADE secret key: unexpected layout"};
  pk.assign(2 * L * N, 0);
  sk.assign(L * N, 0);
  for (size_t i = 0; i < 2 * L; ++i) {  // element 0 = b (towers 0..L-1), element 1 = a
    if (pv[i].first != q[i % L]) throw Error{SHELFI_ERR_FORMAT, "PALISADE public key: tower order"};
    std::memcpy(&pk[i * N], pub.data() + pv[i].second, 8ull * N);
  }
  for (size_t i = 0; i < L; ++i) {
    if (sv[i].first != q[i]) throw Error{SHELFI_ERR_FORMAT, "PALISADE secret key: tower order"};
    std::memcpy(&sk[i * N], priv.data() + sv[i].second, 8ull * N);
  }
}

}  // namespace shelfi

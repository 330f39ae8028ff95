// palisade_codec.h — PALISADE 1.11 wire format of the SHELFI_FHE bytes API: the cereal
// PortableBinary archive of vector<Ciphertext<DCRTPoly>> that ckks.cpp:98-100 /
// :308-310 produce and :281 consumes.
//
// Grammar (pinned by the reference's CT1.txt and key files):
//   archive  := 0x01 [u64 count] ct*            (count absent: a single Ciphertext)
//   ct       := 0x40000000 id [ver ver]           CiphertextImpl, CryptoObject versions
//               0x40000000 ctxid [ctxobj]         context: new (object follows) or ref
//               u64 n  keytag[n]
//               u64 2  dcrt dcrt
//               u64 depth  u64 level  f64 scale  u32 encoding
//               metaid [u64 0]                    metadata map (new: empty map)
//   dcrt     := [ver] u64 L  tower^L  u32 format  0x40000000 u32 paramsid
//   tower    := [ver] 0x40000000 0x01 [ver] u64 N  u64[N]  u64 q  u32 format
//               0x40000000 u32 paramsid
// [ver] = u32 class version, present at a type's first occurrence only; new shared-ptr
// ids carry bit 31 and are numbered 1, 2, 3... in order of first appearance.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace shelfi {

struct PalisadeArchive {
  bool vector_archive = true;
  uint64_t K = 0;
  uint32_t N = 0, L = 0;
  std::vector<uint64_t> q;        // tower moduli (from the residue vectors)
  std::string keytag;
  uint64_t depth = 0, level = 0;
  double scale = 0.0;
  uint32_t encoding = 0;
  size_t ctx_off = 0, ctx_len = 0;  // the embedded context object (first ciphertext)
  std::vector<size_t> tower_off;    // [K][2][L] byte offsets of the N residues
};

// Parses and validates an archive (throws Error{SHELFI_ERR_FORMAT} on anything else).
PalisadeArchive palisade_parse_archive(const uint8_t* b, size_t len);
// True when the bytes start like a PALISADE archive (not a library blob).
bool palisade_looks_like_archive(const uint8_t* b, size_t len);

// Framing of an archive with K ciphertexts: writes everything but the residues into
// buf (nullptr: only sizes it), sets *total and returns the [K][2][L] tower offsets
// where the N residues of each tower go.  ctx_obj: an embedded context object whose
// shared-ptr ids start at 3 (from a public key archive or a parsed ciphertext archive).
std::vector<size_t> palisade_layout(const std::string& ctx_obj, const std::string& keytag,
                                    uint32_t N, uint32_t L, const uint64_t* q, uint64_t K,
                                    uint64_t depth, uint64_t level, double scale, uint32_t encoding,
                                    bool vector_archive, uint8_t* buf, size_t* total);

// key-public.txt (ckks.cpp:48): the embedded context object and the key tag.
void palisade_key_context(const std::string& pub, std::string& ctx_obj, std::string& keytag);

// A standalone context file (cryptocontext.txt) re-embedded one shared-ptr id later
// (what a key or ciphertext archive holds).  Exposed for the tests' pin.
std::string palisade_embed_context(const std::string& ctxfile);

}  // namespace shelfi

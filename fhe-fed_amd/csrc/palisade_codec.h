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
// key_params: the ciphertexts' polynomials carry their own element-parameter objects
// (embedded at the first ciphertext's c0), as every archive the reference's
// encrypt / computeWeightedAverage writes does: there the key is loaded from
// key-public.txt (ckks.cpp:16), so Encrypt's c0 = b*v + e0 + m and c1 = a*v + e1 inherit
// the key file's ILDCRTParams, a different object from the context's (pinned by
// code/params_results.csv:12-16, tests/test_palisade_codec.py).  false: they reference
// the context's parameters (CT1.txt, written where the keys were generated in-process).
std::vector<size_t> palisade_layout(const std::string& ctx_obj, const std::string& keytag,
                                    uint32_t N, uint32_t L, const uint64_t* q, uint64_t K,
                                    uint64_t depth, uint64_t level, double scale, uint32_t encoding,
                                    bool vector_archive, bool key_params, uint8_t* buf,
                                    size_t* total);

// The CryptoContext object: LPCryptoParametersCKKS (ILDCRTParams with one ILNativeParams
// per tower, EncodingParams, the RLWE fields) + LPPublicKeyEncryptionSchemeCKKS + "CKKS".
//   ctx      := u32 1  0x80000001 str(ParamsName)  new(id) u32 0 x3
//               elem   enc  f32 sigma  f32 assurance  f32 rootHermite  u32 field*
//               0x80000002 str(SchemeName)  new(id+3+L) u32 0 x2  u32 enabled  str("CKKS")
//   elem     := 0x40000000 new(id+1) [u32 1 u32 1] u32 2N u32 N u8 1 [u32 1]
//               big(Q) big(0) big(0) big(0)  u64 L  tower^L  big(0)
//   tower_t  := 0x40000000 new(id+2+t) [u32 1 u32 1] u32 2N u32 N u8 1 [u32 1] u64 q
//               u64 psi u64 0 u64 0
//   enc      := 0x40000000 new(id+2+L) [u32 1] u64 scaleBits u64 0 x3 u32 0 u32 batch
//   big(x)   := BigIntegerFixedT<u32, 3500>: 110 u32 limbs, most significant first,
//               then u16 bit length (442 bytes)
// [..] = class versions at a type's first occurrence; str = u64 length + chars.
struct PalisadeCtxParams {
  uint32_t N = 0, L = 0;
  std::vector<uint64_t> q, psi;
  uint64_t plaintext_modulus = 0;  // CKKS stores the scaling-factor bits here
  uint32_t batch = 0;
  float sigma = 3.19f, assurance = 9.0f, root_hermite = 1.006f;
  // u32 block after the floats: 9 fields in the benchmark's cryptoparams (1.11.7), 8 in
  // palisade_pybind's (an older 1.11 writer)
  std::vector<uint32_t> fields = {0, 1, 2, 0, 1, 0, 2, 1, 2};
  uint32_t enabled = 5;         // ENCRYPTION | SHE (ckks.cpp:34-35)
  uint32_t bigint_bytes = 442;  // BigIntegerFixedT<uint32_t, 3500>
  std::string elem_bigints;     // root, bigQ, bigRoot of the ILDCRTParams (parsed; else 0)
};

// Structured parse of a context object whose first shared-ptr id is *first_id
// (2: standalone cryptocontext.txt body, 3: embedded in a key or ciphertext archive).
// name0: the id of its first polymorphic type name (1 in context / key / ciphertext files, 2
// inside an evaluation-key file, whose key type name comes first)
PalisadeCtxParams palisade_parse_context_object(const std::string& obj, uint32_t* first_id,
                                                uint32_t name0 = 1);
std::string palisade_context_object(const PalisadeCtxParams& p, uint32_t first_id, uint32_t name0 = 1);
// Structured parse of a standalone cryptocontext.txt (throws on other layouts)
PalisadeCtxParams palisade_parse_context_file(const std::string& file);
// cryptocontext.txt as ckks.cpp:41 writes it (Serial::SerializeToFile of the context)
std::string palisade_context_file(const PalisadeCtxParams& p);
// key-public.txt (polys = [2][L][N]: b, a) or key-private.txt ([L][N]: s), ckks.cpp:48,53
std::string palisade_key_file(const PalisadeCtxParams& p, const std::string& keytag,
                              const uint64_t* polys, bool is_public);

// key-public.txt (ckks.cpp:48): the embedded context object and the key tag.
void palisade_key_context(const std::string& pub, std::string& ctx_obj, std::string& keytag);

// A standalone context file (cryptocontext.txt) re-embedded one shared-ptr id later
// (what a key or ciphertext archive holds).  Exposed for the tests' pin.
std::string palisade_embed_context(const std::string& ctxfile);

// key-eval-mult.txt (§8 f4): the cereal archive of EvalMultKeyGen's relinearization key as
// PALISADE 1.11 serializes the evaluation-key map (the reference's palisade_pybind/
// SHELFI_FHE/resources/cryptoparams/key-eval-mult.txt; grammar pinned by rewriting that file
// byte for byte, tests/test_palisade_codec.py):
//   file   := 0x01 u64 1 str(tag) u64 1  new-name(1) str(LPEvalKeyRelinImpl<DCRTPoly>) new(1)
//             u32 ver x4  0x40000000 new(2) ctxobj(ids from 3, names from 2)  str(tag)
//             u64 2 ( u64 dnum dcrt^dnum )^2                 m_rKey: b-vector, a-vector
//   dcrt   := [ver] u64 T tower^T u32 0 0x40000000 params    (Q u P towers, EVALUATION)
//   tower  := [ver] 0x40000000 0x01 [ver] u64 N u64[N] u64 q u32 0 0x40000000 tparams
// The first polynomial embeds the key's ILNativeParams per tower and its ILDCRTParams (new
// ids after the context's); the others reference them.
struct PalisadeEvalKey {
  std::string keytag;
  std::string ctx_obj;  // the embedded context object (empty when writing: synthesized from ctx)
  PalisadeCtxParams ctx;
  uint32_t N = 0, T = 0, dnum = 0;
  std::vector<uint64_t> q, psi;    // towers of the key polynomials: Q, then the special primes
  std::string elem_bigints;        // raw root / bigQ / bigRoot of the key's ILDCRTParams
  uint32_t key_versions[4] = {0, 0, 0, 0};   // LPEvalKeyRelinImpl, LPEvalKeyImpl, LPKey, CryptoObject
  uint32_t poly_versions[3] = {1, 1, 1};     // DCRTPoly, PolyImpl, NativeVector class versions
  std::vector<size_t> tower_off;   // parse: [2][dnum][T] byte offsets of the N residues
};
PalisadeEvalKey palisade_parse_evalmult_key(const uint8_t* b, size_t len);
std::string palisade_evalmult_key_file(const PalisadeEvalKey& k, const uint64_t* polys);

}  // namespace shelfi

/*
 * shelfi.h — C ABI of the MI355X-native CKKS weighted-average aggregator.
 *
 * Drop-in replacement for the compute behind the reference's pybind11 module
 * SHELFI_FHE (palisade_pybind/SHELFI_FHE/src/binding.cpp:14-31, class CKKS in
 * include/ckks.h:27-54 implementing Scheme in include/scheme.h:15-32).  Each
 * entry point below names the reference method it replaces.  Plain C: opaque
 * context, raw pointers and sizes, int status codes (0 = OK), a thread-local
 * message via shelfi_last_error().  Caller-owned inputs are never retained;
 * library-owned outputs are released with shelfi_free().
 *
 * All arithmetic runs in hand-written HIP kernels on an AMD Instinct MI355X
 * (gfx950).  There is no CPU compute path: on a host without a usable gfx950
 * device, shelfi_ctx_create() fails with SHELFI_ERR_DEVICE.
 */
#ifndef SHELFI_H_
#define SHELFI_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SHELFI_ABI_VERSION 1

/* status codes */
#define SHELFI_OK 0
#define SHELFI_ERR_ARG -1      /* bad argument (maps to ValueError) */
#define SHELFI_ERR_DEVICE -2   /* HIP / device failure (RuntimeError) */
#define SHELFI_ERR_IO -3       /* file read/write failure */
#define SHELFI_ERR_FORMAT -4   /* malformed / mismatched ciphertext or key blob */
#define SHELFI_ERR_STATE -5    /* keys not loaded, etc. */
#define SHELFI_ERR_RANGE -6    /* value outside the CKKS encoding/decoding range */
#define SHELFI_ERR_PRECISION -7 /* decode: approximation error too high (PALISADE math_error) */

typedef struct shelfi_ctx shelfi_ctx;

/* Parameters of a context (filled by shelfi_ctx_info). */
typedef struct shelfi_info {
  uint32_t ring_dim;       /* N */
  uint32_t num_towers;     /* L = multDepth + 1 */
  uint32_t batch;          /* slots per ciphertext (ckks.h:31 batchSize) */
  uint32_t scale_bits;     /* ckks.h:32 scaleFactorBits */
  uint32_t first_mod_bits; /* bits of q_0 */
  int32_t device;          /* HIP device ordinal */
  uint64_t moduli[16];     /* q_0 .. q_{L-1} */
  uint64_t roots[16];      /* minimal primitive 2N-th roots psi_t */
  double delta;            /* level-0 scaling factor = (double)q_{L-1} (EXACTRESCALE) */
  uint64_t key_id;         /* 0 until keys are loaded/generated */
  int32_t keys_loaded;
  int32_t palisade_keys;   /* 1 if the keys came from PALISADE-format files */
} shelfi_info;

/* ---- library ------------------------------------------------------------ */
int shelfi_abi_version(void);
/* Re-read the SHELFI_* A/B probe switches from the environment.  They are read
 * when a context is created and here, never by a launch; call between calls, not during one. */
void shelfi_reload_switches(void);
const char* shelfi_last_error(void);
void shelfi_free(void* p);

/* Host-only parameter generation (no device needed): PALISADE ParamsGen rule for
 * EXACTRESCALE chains, as called by ckks.cpp:28 genCryptoContextCKKS(multDepth,
 * scaleFactorBits, batchSize).  ring_dim = 0 picks the PALISADE ring dimension
 * (HE-standard 128-bit classic, N >= 2*batch).  Writes L moduli and roots. */
int shelfi_params_generate(uint32_t ring_dim, uint32_t num_towers, uint32_t scale_bits,
                           uint32_t first_mod_bits, uint32_t batch, uint32_t* ring_dim_out,
                           uint64_t* moduli_out, uint64_t* roots_out);

/* Host-only PALISADE reader (no device needed): parses a reference cryptodir
 * (cryptocontext.txt / key-public.txt / key-private.txt, ckks.cpp:11-23).  Call with
 * q/psi/pk/sk = NULL to query N and L first; q/psi hold 16 entries, pk 2*L*N, sk L*N. */
int shelfi_read_palisade(const char* cryptodir, uint32_t* ring_dim, uint32_t* num_towers,
                         uint64_t* moduli, uint64_t* roots, uint64_t* pk, uint64_t* sk);

/* ---- context lifecycle (ckks.cpp:5-9 CKKS::CKKS) -------------------------- */
/* num_towers = multDepth + 1 (reference: multDepth = 1, ckks.cpp:26). */
int shelfi_ctx_create(uint32_t ring_dim, uint32_t num_towers, uint32_t scale_bits,
                      uint32_t first_mod_bits, uint32_t batch, int device, shelfi_ctx** out);
void shelfi_ctx_destroy(shelfi_ctx* ctx);
int shelfi_ctx_info(const shelfi_ctx* ctx, shelfi_info* out);
/* Deterministic ("parity") mode: encryption/keygen randomness derived from `seed`
 * (ChaCha20 stream spec in DESIGN.md).  seed = 0 restores OS-entropy seeding. */
int shelfi_set_seed(shelfi_ctx* ctx, uint64_t seed);

/* ---- keys ----------------------------------------------------------------- */
/* ckks.cpp:25-59 genCryptoContextAndKeyGen: generates keys on the device and writes
 * cryptodir/{cryptocontext,key-public,key-private}.txt in PALISADE 1.11's cereal
 * PortableBinary format (ckks.cpp:41-55; byte-identical to what the reference writes for
 * the same parameters, keys and key tag).  cryptodir = "" or NULL: keys stay in memory. */
int shelfi_keygen(shelfi_ctx* ctx, const char* cryptodir);
/* ckks.cpp:11-23 loadCryptoParams: reads PALISADE 1.11 cereal-binary files (the
 * reference's code/resources/cryptoparams/, or shelfi_keygen's) and this library's
 * round-1 key files ("SHCC"/"SHPK"/"SHSK"). */
int shelfi_load(shelfi_ctx* ctx, const char* cryptodir);
/* Raw key import/export ([2][L][N] public (b, a), [L][N] secret, EVALUATION). */
int shelfi_set_keys(shelfi_ctx* ctx, const uint64_t* pk, const uint64_t* sk);
int shelfi_get_keys(const shelfi_ctx* ctx, uint64_t* pk, uint64_t* sk);

/* ---- bytes API (binding.cpp:26-31) ---------------------------------------- */
/* ckks.cpp:61-104 encrypt: n doubles -> blob of ceil(n/batch) ciphertexts. */
int shelfi_encrypt(shelfi_ctx* ctx, const double* x, size_t n, uint8_t** out, size_t* out_len);
/* Same into a caller-owned buffer (out = NULL: only *out_len); H2D, kernels and D2H
 * are pipelined over ciphertext chunks. */
int shelfi_encrypt_into(shelfi_ctx* ctx, const double* x, size_t n, uint8_t* out, size_t out_cap,
                        size_t* out_len);
/* ckks.cpp:264-320 computeWeightedAverage: C blobs, float32 weights (ckks.cpp:287). */
int shelfi_weighted_average(shelfi_ctx* ctx, const uint8_t* const* blobs, const size_t* lens,
                            const float* weights, size_t num_learners, uint8_t** out,
                            size_t* out_len);
/* Same, writing into a caller-owned buffer (out = NULL: only *out_len = result size).
 * Copies, aggregation and the copy-out are pipelined over ciphertext chunks. */
int shelfi_weighted_average_into(shelfi_ctx* ctx, const uint8_t* const* blobs, const size_t* lens,
                                 const float* weights, size_t num_learners, uint8_t* out,
                                 size_t out_cap, size_t* out_len);
/* ckks.cpp:170-213 decrypt: blob -> n doubles (caller-owned out[n]). */
int shelfi_decrypt(shelfi_ctx* ctx, const uint8_t* blob, size_t len, size_t n, double* out);

/* Decode noise flooding, PALISADE 1.11 CKKSPackedEncoding::Decode:
 * symmetrize, estimate sigma from the anti-symmetric part, add Gaussian noise of
 * stddev sqrt(m_factor + 1) * max(sigma, sqrt(N)/8) (m_factor = CKKS_M_FACTOR, 1 in
 * PALISADE), fail with SHELFI_ERR_PRECISION when log2 sigma > scale_bits - 5.  ON by
 * default with m_factor 1, like the Decrypt it replaces (ckks.cpp:189); enabled = 0 gives
 * the exact, deterministic decode (parity mode).  Applies to shelfi_decrypt and
 * shelfi_dev_decrypt.  Randomness: the ctx's seeded / OS-random ChaCha20 stream. */
int shelfi_set_decode_noise(shelfi_ctx* ctx, int enabled, double m_factor);
/* Decode range (round 6).  exact = 0 (default): decrypt reads the shortest tower prefix whose
 * modulus Q' exceeds 2^130 and reconstructs each coefficient exactly while its centred value is in
 * [-2^127, 2^127); a coefficient outside that range is detected and the call is redone over every
 * tower through an exact multi-word CRT, up to (Q - 1) / 2 (PALISADE's BigInteger decode,
 * ckks.cpp:189).  The prefix cannot see a value of |X| >= Q'/2 whose residue mod Q' falls inside
 * [-2^127, 2^127) (|X| >= 2^163 at 2^15 / L4).  exact = 1: every decrypt reads every tower and
 * decodes through the exact CRT (same output bits wherever both are defined; ~25% slower at
 * 2^15 / L4).  Applies to shelfi_decrypt and the shelfi_dev_decrypt* calls. */
int shelfi_set_decode_exact(shelfi_ctx* ctx, int exact);
/* logError of the last flooded decrypt (max over its ciphertexts; PALISADE
 * Plaintext::GetLogError), -1 if none.  Precision = scale_bits - logError. */
int shelfi_decode_log_error(shelfi_ctx* ctx, int* log_error);

/* Blob inspection: number of ciphertexts, depth, scale, key id. */
int shelfi_blob_info(const uint8_t* blob, size_t len, uint64_t* num_cts, uint32_t* depth,
                     double* scale, uint64_t* key_id);
/* Build a blob from raw residues [K][2][L][N] (host) with the given metadata. */
int shelfi_blob_pack(const shelfi_ctx* ctx, const uint64_t* residues, uint64_t num_cts,
                     uint32_t depth, double scale, uint8_t** out, size_t* out_len);
/* Offset of the residue payload inside a blob (64-byte header). */
size_t shelfi_blob_header_bytes(void);
/* Host-only: a blob's residues as [K][2][L][N] uint64 (out: K*2*L*N words) — a version-1 payload
 * copied, a version-2 (packed wire, shelfi_set_wire_format 2) payload unpacked. */
int shelfi_blob_unpack(const shelfi_ctx* ctx, const uint8_t* blob, size_t len, uint64_t* out);

/* ---- PALISADE 1.11 wire format -------------- */
/* The reference's bytes are cereal PortableBinary archives of
 * vector<Ciphertext<DCRTPoly>> (ckks.cpp:98-100, :281, :308-310).  With keys loaded from
 * the reference's PALISADE files, shelfi_set_wire_format(ctx, 1) makes encrypt produce
 * such archives; computeWeightedAverage and decrypt accept archives and blobs alike,
 * and computeWeightedAverage answers in its inputs' format. */
typedef struct {
  uint32_t ring_dim, num_towers;
  uint64_t num_cts;
  uint64_t moduli[16];
  uint64_t depth, level;
  double scale;
  uint32_t encoding;      /* 4 = CKKSPacked */
  int32_t vector_archive; /* 0: a single Ciphertext (e.g. mkhe's CT1.txt) */
  uint64_t ctx_offset, ctx_length; /* the embedded context object inside the archive */
  char keytag[257];
} shelfi_palisade_info;
/* 0 blob (the C ABI's default), 1 PALISADE archive (the Python / C++ front ends' default once keys
 * are generated or loaded in PALISADE's files, as ckks.cpp:98-103 writes them), 2 packed blob
 * (version 2: the residues at their moduli's widths, the arena's slice format with C = 1 — 218 of
 * 256 bits per coefficient at 2^15/L4, so a PCIe-bound upload carries 15% fewer bytes; DESIGN.md
 * §5.3).  Every entry that takes ciphertext bytes accepts all three. */
int shelfi_set_wire_format(shelfi_ctx* ctx, int format);
/* The format encrypt answers in right now (0, 1 or 2; -1 for a NULL context). */
int shelfi_get_wire_format(const shelfi_ctx* ctx);
/* Host-only: parse an archive; residues [K][2][L][N] copied out when non-NULL. */
int shelfi_palisade_parse(const uint8_t* archive, size_t len, shelfi_palisade_info* info,
                          uint64_t* residues);
/* Host-only: write an archive (free with shelfi_free) from residues [K][2][L][N] and an
 * embedded context object (shared-pointer ids from 3: shelfi_palisade_key_context).
 * flags: SHELFI_PAL_VECTOR = vector<Ciphertext> (else a single Ciphertext, K = 1);
 * SHELFI_PAL_KEY_PARAMS = the polynomials carry the key's own parameter objects, as in
 * every archive the reference's encrypt / computeWeightedAverage writes (its keys are
 * loaded from files); without it they reference the context's (CT1.txt). */
#define SHELFI_PAL_VECTOR 1
#define SHELFI_PAL_KEY_PARAMS 2
int shelfi_palisade_write(const uint8_t* ctx_obj, size_t ctx_len, const char* keytag,
                          uint32_t ring_dim, uint32_t num_towers, const uint64_t* moduli,
                          uint64_t num_cts, const uint64_t* residues, uint64_t depth, uint64_t level,
                          double scale, int flags, uint8_t** out, size_t* out_len);
/* Host-only: cryptocontext.txt as ckks.cpp:41 serializes the context of
 * genCryptoContextCKKS(multDepth = L - 1, scale_bits, batch) with these towers. */
int shelfi_palisade_context_file(uint32_t ring_dim, uint32_t num_towers, const uint64_t* moduli,
                                 const uint64_t* roots, uint32_t scale_bits, uint32_t batch,
                                 uint8_t** out, size_t* out_len);
/* Host-only: key-public.txt (is_public = 1, polys [2][L][N]: b, a) or key-private.txt
 * (polys [L][N]: s) around an embedded context object (ids from 3), ckks.cpp:48,53. */
int shelfi_palisade_key_file(const uint8_t* ctx_obj, size_t ctx_len, const char* keytag,
                             const uint64_t* polys, int is_public, uint8_t** out, size_t* out_len);
/* Host-only: the embedded context object (free with shelfi_free) and key tag of a
 * PALISADE key-public.txt (ckks.cpp:48). */
int shelfi_palisade_key_context(const uint8_t* pub, size_t len, uint8_t** ctx_obj, size_t* ctx_len,
                                char keytag[257]);
/* Host-only: a cryptocontext.txt's context object re-embedded one shared-pointer id
 * later (what key and ciphertext archives hold). */
int shelfi_palisade_embed_context(const uint8_t* ctxfile, size_t len, uint8_t** out,
                                  size_t* out_len);

/* ---- device-resident batch API (HBM in, HBM out; `stream` = hipStream_t) ---- */
/* Ciphertext batches are [K][2][L][N] uint64 in HBM (same order as the blob
 * payload).  Work is enqueued on `stream` exactly as given (NULL = the legacy
 * default stream, e.g. PyTorch's default stream); wavg/modq/ntt return without
 * syncing, encrypt/decrypt synchronise `stream` before returning (they reuse the
 * context's scratch arena). */

/* sum_c W_c * in[c] mod q_t, W_c = (int64)((double)w[c] * delta + 0.5) (EvalMult +
 * EvalAdd, ckks.cpp:286-297).  in_dev: host array of C device pointers. */
int shelfi_dev_wavg(shelfi_ctx* ctx, const uint64_t* const* in_dev, const float* w, size_t C,
                    size_t K, uint64_t* out_dev, void* stream);
/* Packed learner-interleaved arena: the aggregator's resident layout for C learners' K
 * ciphertexts.  Rows of 512 residues in [K][2][L][N] order; a row holds the C learners'
 * slices side by side, and every residue of tower t is packed to U_t bits (bitlength(q_t) when
 * that is 1 mod 4, else rounded up to a multiple of 4; >= 32): 60/53/52/53 at the reference's
 * 2^15/L4, 218 of 256 bits per coefficient, so one aggregation wave reads one contiguous C-slice
 * region and the launch moves 14% fewer bytes
 * (DESIGN.md §3).  The layout is opaque: size it with shelfi_arena_words() (uint64 words;
 * ciphertexts [k0, k1) of an arena start at word k0 * shelfi_arena_words(ctx, C, 1) and are
 * themselves an arena of k1 - k0 ciphertexts).  shelfi_dev_arena_put packs learner
 * `learner`'s [K][2][L][N] uint64 batch (device memory, or host memory if src_on_host) into
 * its slices. */
size_t shelfi_arena_words(const shelfi_ctx* ctx, size_t C, size_t K);
/* Every put validates what landed: one device pass over the learner's slices checks that
 * each residue is < q_t (the aggregation's carry-free limb sums assume canonical
 * residues), and the call returns after it (synchronises `stream`).  A refused slot
 * (SHELFI_ERR_FORMAT) stays marked: shelfi_dev_wavg_arena over a range of that arena
 * fails with SHELFI_ERR_STATE until a valid put replaces the slot. */
int shelfi_dev_arena_put(shelfi_ctx* ctx, const void* src, int src_on_host, size_t K, size_t learner,
                         size_t C, uint64_t* arena_dev, void* stream);
/* A learner's upload as it arrives over the wire — a library blob or a PALISADE archive
 * (ckks.cpp:276-281's per-learner bytes) — placed into its arena slot.  The header is
 * checked against the context before any byte is copied: ring dimension, towers and
 * moduli (params_id), the key (key_id / PALISADE keyTag, as EvalAdd refuses other keys,
 * SURVEY App. B.7), the CKKS-packed encoding and the length; the batch must hold exactly
 * K ciphertexts.  Refusals are SHELFI_ERR_FORMAT; the residues are then validated as
 * for shelfi_dev_arena_put.  A refused header marks the slot refused as well (its previous
 * contents are not aggregated as if the upload had landed). */
int shelfi_dev_arena_put_blob(shelfi_ctx* ctx, const uint8_t* blob, size_t len, size_t K, size_t learner,
                              size_t C, uint64_t* arena_dev, void* stream);
/* Forget the refusal marks of an arena's memory [arena_dev, arena_dev + words) before it is
 * freed or reused (no reference counterpart: the reference has no resident arena).  A put
 * into a differently shaped arena over the same memory, and a parameter or key reload, drop
 * stale marks by themselves. */
int shelfi_dev_arena_release(shelfi_ctx* ctx, const uint64_t* arena_dev, size_t words);
/* Host-synchronous check that every residue of a [K][2][L][N] device batch is < q_t
 * (SHELFI_ERR_FORMAT otherwise): the upload check of SHELFI_FHE.device.Arena's uint64 layout, which
 * small launches aggregate with shelfi_dev_wavg (the packed arena checks while packing). */
int shelfi_dev_check_residues(shelfi_ctx* ctx, const uint64_t* ct_dev, size_t K, void* stream);
/* shelfi_dev_wavg over an arena of C learners (same arithmetic and result). */
int shelfi_dev_wavg_arena(shelfi_ctx* ctx, const uint64_t* arena_dev, const float* w, size_t C,
                          size_t K, uint64_t* out_dev, void* stream);
/* The same aggregation written packed: K ciphertexts in the arena's slice format with C = 1
 * (shelfi_arena_words(ctx, 1, K) uint64 words at out_packed), the packed exchange's send form. */
int shelfi_dev_wavg_arena_packed(shelfi_ctx* ctx, const uint64_t* arena_dev, const float* w, size_t C,
                                 size_t K, uint64_t* out_packed, void* stream);
/* sum_g x_g mod q_t of G <= 16 packed (C = 1) batches of K ciphertexts stacked stride_words uint64
 * words apart (>= shelfi_arena_words(ctx, 1, K)) -> out_dev [K][2][L][N], canonical residues: the
 * packed exchange's receive side (EvalAdd of the ranks' partial aggregates). */
int shelfi_dev_sum_packed(shelfi_ctx* ctx, const uint64_t* stacked, size_t G, size_t K, size_t stride_words,
                          uint64_t* out_dev, void* stream);
/* Output placement for a resident arena (no reference counterpart: a property of where
 * the aggregate lands in HBM).  The arena launch's time depends on the physical
 * placement of its output buffer relative to the arena (up to 12%,
 * reproducible per buffer pair).  Runs shelfi_dev_wavg_arena into each of the n
 * candidate [K][2][L][N] buffers (1 warm-up + `launches` timed launches each, HIP
 * events on `stream`), writes each one's mean launch time to ms[i] (if ms), and the
 * index of the fastest to *best.  Every candidate ends up holding the aggregate. */
int shelfi_dev_wavg_arena_pick_output(shelfi_ctx* ctx, const uint64_t* arena_dev, const float* w,
                                      size_t C, size_t K, uint64_t* const* candidates, size_t n,
                                      int launches, size_t* best, float* ms, void* stream);
/* Folds a collective's uint64 SUM of G <= 15 reduced partial sums back into [0, q_t)
 * (multi-GPU combine: local shelfi_dev_wavg -> RCCL reduce/reduce_scatter -> this). */
int shelfi_dev_modq(shelfi_ctx* ctx, uint64_t* buf_dev, size_t K, void* stream);
/* ---- multi-GPU combine over RCCL (one process per GPU, SURVEY §8 e) --------
 * Each rank aggregates its own learners with shelfi_dev_wavg / _arena into a partial
 * of K ciphertexts; these calls combine the partials exactly (uint64 SUM over <= 16
 * ranks, then the mod-q fold of shelfi_dev_modq), bit-identical to aggregating every
 * learner on one GPU.  Collective: every rank of the communicator makes the same call
 * in the same order.  Replaces, for the multi-GPU path, the serial EvalAdd loop of
 * CKKS::computeWeightedAverage (ckks.cpp:291-297). */
#define SHELFI_COMM_ID_BYTES 128
/* rank 0 makes the 128-byte id and hands it to every rank out of band */
int shelfi_comm_unique_id(uint8_t* id_out);
/* bind a communicator of `world` (<= 16) ranks to ctx (its device), replacing any previous one */
int shelfi_comm_init(shelfi_ctx* ctx, const uint8_t* id, int rank, int world);
int shelfi_comm_destroy(shelfi_ctx* ctx);
/* rank/world of ctx's communicator (-1 / 0 if none) */
int shelfi_comm_info(const shelfi_ctx* ctx, int* rank, int* world);
/* in place: the combined aggregate lands on `root` (other ranks' buffers are scratch) */
int shelfi_dev_reduce(shelfi_ctx* ctx, uint64_t* partial_dev, size_t K, int root, void* stream);
/* in place: the combined aggregate on every rank */
int shelfi_dev_allreduce(shelfi_ctx* ctx, uint64_t* partial_dev, size_t K, void* stream);
/* rank r receives ciphertexts [r K/W, (r+1) K/W) of the combined aggregate in out_dev
 * (K % W == 0): each rank then decrypts its own slice, nothing is gathered */
int shelfi_dev_reduce_scatter(shelfi_ctx* ctx, const uint64_t* partial_dev, size_t K,
                              uint64_t* out_dev, void* stream);
/* The whole learner-sharded step in one call, pipelined: this rank's arena of C learners
 * (K ciphertexts each) is aggregated piece by piece on `stream`, and each piece's
 * ncclReduceScatter runs on the context's own comm stream (ordered by HIP events) while the
 * next piece is aggregated.  Rank r receives the combined aggregate of global ciphertexts
 * [r Ks, min(K, (r+1) Ks)), Ks = shelfi_combine_share_cts(ctx, K) = ceil(K / W), contiguous in
 * share_dev (Ks ciphertexts; slots past K are zero).  send_dev is scratch of W * Ks
 * ciphertexts.  fold = 1 folds each piece into [0, q_t) on the comm stream; fold = 0 leaves
 * the uint64 sums of W residues for shelfi_dev_decrypt_sum, which folds them on load (no
 * separate pass).  Returns with the work enqueued: `stream` is ordered after the share. */
size_t shelfi_combine_share_cts(const shelfi_ctx* ctx, size_t K);
int shelfi_dev_combine_arena(shelfi_ctx* ctx, const uint64_t* arena_dev, const float* w, size_t C, size_t K,
                             size_t pieces, uint64_t* send_dev, uint64_t* share_dev, int fold, void* stream);
/* The same step with the packed share exchange (no reference counterpart): each
 * piece's partial is written packed (the arena's slice format with C = 1, sum_t U_t bits per
 * coefficient) into send_dev, exchanged by one grouped ncclSend/ncclRecv all-to-all into
 * recv_dev, and summed on the comm stream with unit weights (the mod-q fold included) into
 * share_dev.  (W - 1) / W of the packed partial crosses xGMI per rank instead of the uint64 one.
 * send_dev and recv_dev hold shelfi_arena_words(ctx, 1, W * Ks) uint64 words each. */
int shelfi_dev_combine_arena_packed(shelfi_ctx* ctx, const uint64_t* arena_dev, const float* w, size_t C,
                                    size_t K, size_t pieces, uint64_t* send_dev, uint64_t* recv_dev,
                                    uint64_t* share_dev, void* stream);

/* encode + encrypt n doubles (device) into K = ceil(n/batch) ciphertexts. */
int shelfi_dev_encrypt(shelfi_ctx* ctx, const double* x_dev, size_t n, uint64_t* ct_dev,
                       void* stream);
/* decrypt + decode K ciphertexts of scaling factor `scale` into n doubles (device). */
int shelfi_dev_decrypt(shelfi_ctx* ctx, const uint64_t* ct_dev, size_t K, double scale,
                       size_t n, double* out_dev, void* stream);
/* negacyclic NTT of P polys [P][N] whose tower is (p % L) (PALISADE order). */
int shelfi_dev_ntt(shelfi_ctx* ctx, uint64_t* polys_dev, size_t P, int inverse, void* stream);

/* ---- EvalMult (ct x ct), relinearization, ModReduce ---------- *
 * The general-circuit part of the PALISADE 1.11 CKKS scheme behind the reference's
 * contexts (ckks.cpp:28 genCryptoContextCKKS: ks = HYBRID, rs = EXACTRESCALE, dnum from
 * multDepth; the reference's own evaluation key is palisade_pybind/SHELFI_FHE/resources/
 * cryptoparams/key-eval-mult.txt).  Not on the aggregation path (ckks.cpp:26 multDepth = 1).
 * A ciphertext of `towers` RNS towers holds q_0 .. q_{towers-1} (towers = L - level). */
/* Host-only: PALISADE's HYBRID key-switching parameters for a chain: dnum digits of alpha
 * towers and num_special special primes (special/special_roots hold 16). */
int shelfi_special_primes(uint32_t ring_dim, uint32_t num_towers, const uint64_t* moduli, uint32_t* dnum,
                          uint32_t* alpha, uint32_t* num_special, uint64_t* special, uint64_t* special_roots);
/* The context's key-switching parameters; *has_key = 1 once an evaluation key is installed. */
int shelfi_eval_key_info(const shelfi_ctx* ctx, uint32_t* dnum, uint32_t* alpha, uint32_t* num_special,
                         uint64_t* special, int* has_key);
/* cc->EvalMultKeyGen(sk) on the device: the relinearization key s^2 -> s, layout
 * [2][dnum][L + num_special][N] (b-vector, a-vector; EVALUATION), seeded like keygen. */
int shelfi_eval_mult_keygen(shelfi_ctx* ctx);
size_t shelfi_eval_key_words(const shelfi_ctx* ctx); /* 2 * dnum * (L + num_special) * N */
int shelfi_get_eval_key(const shelfi_ctx* ctx, uint64_t* evk);
int shelfi_set_eval_key(shelfi_ctx* ctx, const uint64_t* evk);
/* PALISADE key-eval-mult.txt (cereal archive of the evaluation-key map, as the reference's
 * palisade_pybind/SHELFI_FHE/resources/cryptoparams/key-eval-mult.txt).  save: this context's
 * key (PALISADE keys required: the file embeds their context and key tag); load: a file made
 * for this key pair and these parameters (shelfi_load also picks up a matching
 * key-eval-mult.txt beside the key files). */
int shelfi_save_eval_key(const shelfi_ctx* ctx, const char* path);
int shelfi_load_eval_key(shelfi_ctx* ctx, const char* path);
typedef struct {
  uint32_t ring_dim, num_towers, ctx_towers, dnum; /* num_towers = Q's ctx_towers + special */
  uint64_t moduli[16], roots[16];
  char keytag[257];
} shelfi_palisade_evk_info;
/* Host-only: parse a key-eval-mult.txt; polys [2][dnum][num_towers][ring_dim] when non-NULL. */
int shelfi_palisade_evalkey_parse(const uint8_t* file, size_t len, shelfi_palisade_evk_info* info,
                                  uint64_t* polys);
/* Host-only: the same file re-serialized around other residues (the format's pin). */
int shelfi_palisade_evalkey_rewrite(const uint8_t* file, size_t len, const uint64_t* polys, uint8_t** out,
                                    size_t* out_len);
/* cc->EvalMult(ct_a, ct_b): tensor product + HYBRID relinearization, a, b, out
 * [K][2][towers][N] in HBM (out may be a or b).  Result depth 2, scale = scale_a scale_b. */
int shelfi_dev_mult(shelfi_ctx* ctx, const uint64_t* a_dev, const uint64_t* b_dev, size_t K, uint32_t towers,
                    uint64_t* out_dev, void* stream);
/* cc->ModReduce / Rescale: [K][2][towers][N] -> [K][2][towers-1][N] (no overlap), dividing by
 * q_{towers-1} with rounding; scale / q_{towers-1}. */
int shelfi_dev_rescale(shelfi_ctx* ctx, const uint64_t* in_dev, size_t K, uint32_t towers, uint64_t* out_dev,
                       void* stream);
/* shelfi_dev_decrypt for ciphertexts of `towers` <= L towers (after ModReduce). */
int shelfi_dev_decrypt_level(shelfi_ctx* ctx, const uint64_t* ct_dev, size_t K, uint32_t towers, double scale,
                             size_t n, double* out_dev, void* stream);
/* shelfi_dev_decrypt of a multi-GPU combine's unfolded share: every residue is a uint64 sum of
 * `terms` (1..16) canonical residues (shelfi_dev_combine_arena with fold = 0); the mod-q fold
 * happens inside decrypt's first pass. */
int shelfi_dev_decrypt_sum(shelfi_ctx* ctx, const uint64_t* ct_dev, size_t K, uint32_t terms, double scale,
                           size_t n, double* out_dev, void* stream);

/* ---- test hooks (host-visible tables) ------------------------------------- */
/* CKKS special-FFT twiddles (flat, index lenh + j) as used by the kernels. */
int shelfi_fft_twiddles(uint32_t slots, double* inv_re, double* inv_im, double* fwd_re,
                        double* fwd_im);
/* Gaussian CDT thresholds used by the samplers; returns the entry count. */
int shelfi_gauss_cdt(double sigma, uint64_t* cdt, int max_entries);

#ifdef __cplusplus
}
#endif
#endif /* SHELFI_H_ */

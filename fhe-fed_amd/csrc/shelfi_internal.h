// shelfi_internal.h — shared host-side declarations of libshelfi (not installed).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/shelfi.h"

namespace shelfi {

typedef unsigned __int128 u128;

// ---------------------------------------------------------------- errors ----
void set_error(const std::string& msg);
struct Error {
  int code;
  std::string msg;
};
#define SHELFI_HIP(expr)                                                             \
  do {                                                                               \
    hipError_t _e = (expr);                                                          \
    if (_e != hipSuccess)                                                            \
      throw ::shelfi::Error{SHELFI_ERR_DEVICE, std::string(#expr) + ": " +           \
                                                 hipGetErrorString(_e)};             \
  } while (0)

// ----------------------------------------------------------- host params ----
constexpr int kMaxTowers = 16;
constexpr int kMaxCommRanks = 16;  // W partials below q < 2^60 sum exactly in a uint64
constexpr int kFftBlockLog = 10;     // complex f64 block staged in LDS by FFT pass 2
constexpr int kFftBlockLogBig = 11;  // batch >= 2^15: 32 KiB blocks keep pass 1 at 16 columns
inline uint32_t fft_block_log(uint32_t logS) {
  const uint32_t b = logS >= 15 ? (uint32_t)kFftBlockLogBig : (uint32_t)kFftBlockLog;
  return logS < b ? logS : b;
}
constexpr int kNttBlockLog = 11;     // u64 block staged in LDS by NTT pass 2 (N <= 2^16)
constexpr int kNttBlockLogBig = 12;  // N >= 2^17: 32 KiB blocks keep pass 1 at 32 columns
// 2^16 runs 2^11 blocks + a 32-column pass 1: 5% faster encrypt and decrypt than 2^12
// blocks at L = 6 (A/B in one box, tools/enc_variant_probe.py); 2^17 is a tie.
// SHELFI_NTT_BLOCK_LOG_BIG=11|12 overrides the block size for N >= 2^16 in a whole
// process (read once: tables and launches must agree; A/B runs use separate processes).
inline uint32_t ntt_block_log(uint32_t logN) {
  static const uint32_t ovr = [] {
    const char* e = std::getenv("SHELFI_NTT_BLOCK_LOG_BIG");
    const int v = e ? std::atoi(e) : 0;
    return (uint32_t)((v == 11 || v == 12) ? v : 0);
  }();
  uint32_t b = logN >= 17 ? (uint32_t)kNttBlockLogBig : (uint32_t)kNttBlockLog;
  if (ovr && logN >= 16) b = ovr;
  return logN < b ? logN : b;
}

// A/B probe switches (none changes an output bit), process-wide: read from the
// environment when a context is created and by shelfi_reload_switches() -- never on a launch path --
// and published as an immutable snapshot (api.cpp), so concurrent calls never see a torn struct.
struct Switches {
  bool xcd_order = true;       // SHELFI_XCD_ORDER=0: natural block order in the NTT block passes
  bool ntt_wl = true;          // SHELFI_NTT_WL=0: a workgroup barrier at every block-pass exchange
  bool fft_ct = true;          // SHELFI_FFT_CT=0: LDS-loop FFT block passes
  bool fft_whole = true;       // SHELFI_FFT_WHOLE=0: separate columns / blocks FFT passes at 2^14 slots
  bool enc_fused = true;       // SHELFI_ENC_FUSED_COLS=0: enc_prep_kernel + three column passes
  bool enc_pp = true;          // SHELFI_ENC_PP=0: one-shot encrypt block pass
  bool dec_pp = true;          // SHELFI_DEC_PP=0: one-shot decrypt block pass
  bool enc_nored = true;       // SHELFI_ENC_NORED=0: reductions in every tower
  bool enc_tab = true;         // SHELFI_ENC_TAB=0: butterflies for v's / e1's first column stages
  bool enc_vt = true;          // SHELFI_ENC_VT=0: v's columns pass in enc_cols_fused, not enc_vtab sums
  int enc_ts = -1;             // SHELFI_ENC_TS=0|1: enc_cols_fused's one-wave-per-tower form (-1: by K)
  bool dec_all_towers = false; // SHELFI_DEC_ALL_TOWERS=1: decode over every tower
  bool stage_trace = false;    // SHELFI_STAGE_TRACE=1: the bytes-API aggregation prints its call split
  bool enc_x5 = true;          // SHELFI_ENC_X5=0: nlogR = 5 encrypt through enc_prep_kernel + three column passes
  int pack_kernel = 0;         // SHELFI_PACK_KERNEL=r3|v4 (0: by shape)
  int pack_unroll = 0;         // SHELFI_PACK_UNROLL=1|2|4|8 (0: by shape)
  int pack_waves = 0;          // SHELFI_PACK_WAVES=2|8 (0: 4 rows per block)
  int wavg_rows = 0;           // SHELFI_WAVG_ROWS=1|2 (0: by shape)
  uint32_t wavg_strands = 0;   // SHELFI_WAVG_STRANDS=n: wavg_packed's blocks in n interleaved strands (0: in order)
  int arena_stager = -1;       // SHELFI_ARENA_STAGER=0|1 (-1: by upload shape)
  uint64_t dev_chunk_mib = 4096;  // SHELFI_DEV_CHUNK_MIB: device encrypt / decrypt scratch per chain
  uint64_t wavg_chunk_mib = 0;    // SHELFI_WAVG_CHUNK_MIB: bytes-API aggregation chunk per learner group
                                  // (0: 32 MiB per learner with direct uploads, 128 per group through the ring)
  uint64_t stage_slot_mib = 16;   // SHELFI_STAGE_SLOT_MIB: pinned staging-ring slot (DMA granule)
  bool h2d_direct = false;        // SHELFI_H2D_DIRECT=1: bytes-API uploads straight from pageable memory
  bool h2d_two = true;            // SHELFI_H2D_TWO=0: direct uploads from the calling thread only
};
const Switches& switches();
void reload_switches();

struct Params {
  uint32_t N = 0, logN = 0, L = 0, batch = 0, gap = 0, scale_bits = 0, first_mod_bits = 0;
  uint64_t q[kMaxTowers] = {0};
  uint64_t psi[kMaxTowers] = {0};
  double delta = 0.0;  // (double)q[L-1]
  double sigma = 3.19;
};

uint64_t powmod(uint64_t a, uint64_t e, uint64_t q);
uint64_t invmod(uint64_t a, uint64_t q);
uint64_t shoup(uint64_t w, uint64_t q);  // floor(w * 2^64 / q)
uint64_t mod_signed(int64_t v, uint64_t q);
bool is_prime(uint64_t n);
uint32_t default_ring_dim(uint32_t L, uint32_t scale_bits, uint32_t first_mod_bits, uint32_t batch);
uint32_t hybrid_dnum(uint32_t L);
double ring_dim_qbound(uint32_t L, uint32_t scale_bits, uint32_t first_mod_bits);
void generate_chain(uint32_t N, uint32_t L, uint32_t scale_bits, uint32_t first_mod_bits,
                    uint64_t* q, uint64_t* psi);
uint64_t min_root(uint64_t m, uint64_t q);
void special_primes(uint32_t N, uint32_t L, const uint64_t* q, uint32_t* dnum, uint32_t* alpha,
                    uint32_t* kP, uint64_t* p, uint64_t* ppsi);
void fft_twiddles(uint32_t slots, double* inv_re, double* inv_im, double* fwd_re, double* fwd_im);
int gauss_cdt(double sigma, uint64_t* cdt, int max_entries);
uint64_t fnv1a(const void* data, size_t n, uint64_t h = 1469598103934665603ull);

// ------------------------------------------------------- device constants ----
// Per-tower constants, laid out for scalar (SGPR) loads in the kernels.
struct TowerConst {
  uint64_t q;
  uint64_t one_shoup;     // floor(2^64 / q): x mod q for any u64 x via Shoup-by-1
  uint64_t r30, r30_shoup;  // 2^30 mod q
  uint64_t r60, r60_shoup;  // 2^60 mod q
  uint64_t r64, r64_shoup;  // 2^64 mod q
  uint64_t ninv, ninv_shoup;  // N^-1 mod q
  uint64_t qhat_inv, qhat_inv_shoup;  // (Q/q_t)^-1 mod q_t
  double inv_q;               // 1.0 / q (crt_exact_value's k estimate)
  uint64_t nq, n4q, n8q;      // 2^64 - q, - 4q, - 8q (borrow-free conditional subtractions)
  // any u64 x -> [0, 2q): k = (x_hi * red_r) >> (32 + red_sh), x - k q (red_any; needs
  // q >= 2^40, red_ok): red_r = floor(2^(32 + E) / q) < 2^32, E = bitlength(q) - 1
  uint32_t red_r, red_sh, red_ok;
  // the CRT's k in binary32 (crt_value): y_t >> crt_sh < 2^32 (crt_sh = max(0, E - 31)) times
  // inv_q32 = 2^crt_sh / q
  uint32_t crt_sh;
  float inv_q32;
  uint32_t pad32;
  uint64_t bq62;  // floor(2^62 / q) q: v + bq62 in [0, 2^63) for |v| <= 2^61 + 2^7 (encrypt's m + e0)
  uint64_t ninv_qhat, ninv_qhat_shoup;  // N^-1 (Q/q_t)^-1 mod q_t (INTT scale fused with the CRT)
  uint64_t ninv_qhat_w1, ninv_qhat_w1_shoup;  // ninv_qhat * psi^-bitrev(1): the last INTT stage's twiddle, scaled
  // the CRT in 30-bit limbs (crt_value, L <= 7): (Q/q_t) mod 2^210 and (2^210 - Q) mod 2^210
  // (the same in every tower), limbs 0..6 of 30 bits; a launch uses the first DeviceTables::crt_nc
  uint32_t crt30[7], nq30[7];
};

constexpr int kEncVTab = 4 * 81, kEncETab = 128, kEncTab = kEncVTab + kEncETab;

struct DeviceTables {
  TowerConst* tc = nullptr;         // [L]
  uint64_t* psi_rev = nullptr;      // [L][N]  psi^bitrev(i)
  uint64_t* psi_rev_sh = nullptr;   // [L][N]  Shoup companions
  uint64_t* ipsi_rev = nullptr;     // [L][N]  psi^-bitrev(i)
  uint64_t* ipsi_rev_sh = nullptr;  // [L][N]
  // per-block {w, w'} twiddle slices for the compile-time block passes: [L][nb][2^BL],
  // entry 2^l + i of block b = index 2^(sstart + l) + b 2^l + i of psi_rev / ipsi_rev
  // (BL = ntt_block_log(logN), sstart = logN - BL, nb = 2^sstart)
  ulonglong2* tw_fwd_blk = nullptr;
  ulonglong2* tw_inv_blk = nullptr;
  bool red_ok = false;  // every tower has TowerConst::red_ok (q >= 2^40): *_ct kernels usable
  double2* fft_inv = nullptr;       // [B] flat special-FFT twiddles (FFTSpecialInv)
  double2* fft_fwd = nullptr;       // [B] (FFTSpecial)
  uint64_t* cdt = nullptr;          // Gaussian CDT [64]
  // encrypt's first column stages of its small polynomials (enc_cols_fused), per tower
  // [L][kEncTab]: the radix-4 outputs of 4 ternary inputs (stages 0-1, 4 x 81) and W0 e for e1's
  // stage 0 (e + 64, |e| <= 63), all canonical
  uint64_t* enc_tab = nullptr;
  // encrypt's NTT(v) without the columns pass (round 5, kernels.hip ntt_fwd_blocks_enc_pp<VT>): for a
  // 16-row columns pass (logN - BL = 4), [L][16 rows][4 groups][81]: output row r of the 4 column
  // stages applied to v restricted to rows g, g + 4, g + 8, g + 12 with ternary pattern p (base 3),
  // canonical; the row's value is the sum over the 4 groups.  nullptr for other shapes.
  uint64_t* enc_vtab = nullptr;
  int cdt_len = 0;
  // Decode's CRT (round 6).  crt_nc: 30-bit columns crt_value needs to hold sum_t y_t (Q/q_t) - k Q
  // exactly (ceil((bits(Q) + bits(L) + 1) / 30), at least 5), or 0 when that exceeds 7 or L > 7: such
  // tower sets always decode through crt_exact_kernel.  crt_mw: that kernel's table (uint32 words):
  // [0] NL limbs, [1] NW 64-bit words of |X|, [2..3] 0, then (Q/q_t) [L][NL], 2^(30 NL) - Q [NL],
  // (Q - 1) / 2 [NL], all in 30-bit limbs.
  uint32_t crt_nc = 0;
  uint32_t* crt_mw = nullptr;
};
constexpr int kCrtMwMaxLimbs = 36;  // crt_exact_kernel: 16 towers below 2^60, times L, plus sign

// NTT / CRT tables of an arbitrary tower list p.q[0..p.L) (api.cpp); free_ntt_tables frees
// only what build_ntt_tables allocates (not the FFT / Gaussian tables of a context).
void build_ntt_tables(const Params& p, DeviceTables& dt);
void free_ntt_tables(DeviceTables& dt);
// A view of towers [t0, t0 + n) of dt for launch_ntt (pointers offset, nothing owned).
inline DeviceTables tower_view(const DeviceTables& dt, uint32_t t0, uint32_t N) {
  DeviceTables v;
  v.tc = dt.tc + t0;
  v.psi_rev = dt.psi_rev + (size_t)t0 * N;
  v.psi_rev_sh = dt.psi_rev_sh + (size_t)t0 * N;
  v.ipsi_rev = dt.ipsi_rev + (size_t)t0 * N;
  v.ipsi_rev_sh = dt.ipsi_rev_sh + (size_t)t0 * N;
  v.tw_fwd_blk = dt.tw_fwd_blk + (size_t)t0 * N;
  v.tw_inv_blk = dt.tw_inv_blk + (size_t)t0 * N;
  v.red_ok = dt.red_ok;
  return v;
}

struct DeviceKeys {
  uint64_t* pk = nullptr;     // [2][L][N]
  uint64_t* pk_sh = nullptr;  // [2][L][N]
  uint64_t* sk = nullptr;     // [L][N]
  uint64_t* sk_sh = nullptr;  // [L][N]
};

}  // namespace shelfi

namespace shelfi {
class Stager;
class AsyncDrain;
class AsyncUpload;
struct EvalState;  // eval.cpp: relinearization key + per-level tables
}

struct shelfi_ctx {
  mutable std::mutex mu;  // serializes calls on this context
  shelfi::Params p;
  int device = 0;
  hipStream_t stream = nullptr;   // copy / default work stream
  hipStream_t stream2 = nullptr;  // compute stream of the pipelined bytes API
  hipStream_t stream3 = nullptr;  // copy-out stream of the pipelined bytes API
  shelfi::Stager* stage = nullptr;  // pinned staging rings (host_stage.h), lazily created
  shelfi::AsyncDrain* drain = nullptr;  // background output scatter of the direct-upload aggregation
  shelfi::AsyncUpload* up2 = nullptr;   // second uploading thread of the direct-upload aggregation
  hipStream_t stream4 = nullptr;        // its upload stream
  shelfi::DeviceTables dt;
  shelfi::DeviceKeys dk;
  std::vector<uint64_t> pk_host, sk_host;
  bool keys_loaded = false;
  bool palisade_keys = false;
  uint64_t key_id = 0;
  uint64_t params_id = 0;
  uint64_t seed = 0;          // 0 -> OS entropy per call
  uint64_t enc_counter = 0;   // global ciphertext index for the sampler stream
  uint32_t* host_flag = nullptr; // pinned host mirror of dev_flag (async readback before one sync)
  uint32_t* map_flag_host = nullptr;  // GenFlag words in pinned host memory (encode range, decode CRT range)
  uint32_t* map_flag_dev = nullptr;   // the same words as the device addresses them
  uint32_t map_gen = 0;               // the last call generation handed out (never 0)
  uint32_t* dev_flag = nullptr;  // device flags: [0] encode range (before round 6), [1] decode precision,
                                 // [2] max decode logError (noise flooding), [3] bytes-API
                                 // upload residue >= q, [4] arena upload residue >= q, [5] the
                                 // packed wire's pack check, [6] shelfi_dev_check_residues,
                                 // (round 6: the encode and decode-CRT range flags are GenFlag words)
  // arena slots whose last upload was refused (shelfi_dev_arena_put*): an aggregation
  // over an arena range holding one fails instead of summing the refused residues
  // (an entry names the arena by its base, its shelfi_arena_words(C, K) span and C, so a later
  // put into a differently shaped arena over the same memory -- the old one was freed -- drops it;
  // shelfi_dev_arena_release and a parameter/key reload drop entries explicitly)
  struct ArenaRefusal {
    const uint64_t* arena;
    size_t words;  // shelfi_arena_words(C, K) of that arena
    size_t C;
    size_t learner;
  };
  std::vector<ArenaRefusal> arena_refused;
  int decode_noise = 1;          // shelfi_set_decode_noise (PALISADE floods every decode)
  double decode_m_factor = 1.0;
  int decode_exact = 0;          // shelfi_set_decode_exact: every decrypt over every tower, exact CRT
  int last_log_error = -1;       // of the last flooded decrypt, -1 if none
  bool log_error_pending = false;  // dev_flag[2] holds a newer one, read on demand (shelfi_decode_log_error)
  std::string pal_ctx_obj;       // PALISADE keys: embedded context object (§8 f1)
  std::string pal_keytag;        // PALISADE keys: key tag
  int wire = 0;                  // encrypt output: 0 blob, 1 PALISADE archive
  // device weight-limb buffers of wavg_packed (ring; reused while weights repeat)
  static constexpr int kWeightRing = 8;
  uint32_t* wl_dev[kWeightRing] = {};
  size_t wl_cap[kWeightRing] = {};
  hipEvent_t wl_done[kWeightRing] = {};
  std::vector<uint32_t> wl_host[kWeightRing];
  int wl_next = 0, wl_last_slot = -1;
  uint32_t* unit_wl = nullptr;   // [16][kMaxTowers][2] limbs (1, 0): the packed exchange's unit-weight sum
  // scratch arena (grown on demand, never shrunk)
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  void* io = nullptr;            // bytes-API staging arena (inputs/outputs)
  size_t io_bytes = 0;
  uint64_t* gather_host = nullptr;  // pinned run-offset table of a bytes-API aggregation of archives (gather_cap words)
  size_t gather_cap = 0;
  shelfi::EvalState* ev = nullptr;  // EvalMult / ModReduce state (eval.cpp), lazily created
  // RCCL communicator of the multi-GPU combine (comm.cpp; ncclComm_t, opaque here)
  void* comm = nullptr;
  int comm_rank = 0, comm_world = 0;
  hipStream_t comm_stream = nullptr;     // the pipelined combine's collectives (comm.cpp)
  std::vector<hipEvent_t> comm_events;   // piece-ready events of the pipelined combine
};

namespace shelfi {

// device-side launchers (kernels.hip)
constexpr int kWavgMaxLearners = 16;  // per launch (limb sums stay < 2^64)
constexpr int kArenaChunk = 512;      // residues per (row, learner) slice of an arena
struct WavgArgs {
  const uint64_t* ptrs[kWavgMaxLearners];          // learner batches [K][2][L][N]
  uint32_t wl[kWavgMaxLearners][kMaxTowers][2];    // 30-bit limbs of W_{c,t}
  uint64_t* out;
  uint64_t rows;  // K * 2 * L
  uint32_t C, L, logN, accumulate;
  uint32_t* bad;  // device flag set when an input residue is >= q (or null)
};
void launch_wavg(const WavgArgs& a, const TowerConst* tc, hipStream_t s);
// Packed arena (round 3): the aggregator's resident layout.  Tower t's residues are
// stored at U_t bits instead of 64: U_t = bitlength(q_t) when that is 1 mod 4 (a field of U_t - 1
// bits + the top bit in a flag plane), else 4 ceil(bitlength(q_t) / 4); at least 32, at most 60.
// Rows of 512 residues of one (ct, poly, tower) in natural order, each row holding the C learners'
// slices side by side, a slice 16 U_t dwords (lane l of a wave owns residues 2l, 2l + 1 (+128 g,
// g < 4), packed into 16-byte / 8-byte / 4-byte field planes and a byte flag plane, see kernels.hip).
struct ArenaPack {
  uint32_t w[kMaxTowers];    // U_t
  uint32_t pre[kMaxTowers];  // sum of U_t' for t' < t
  uint32_t sum;              // sum of U_t
};
ArenaPack arena_pack(const Params& p);                 // api.cpp
uint64_t arena_ct_words(const Params& p, uint64_t C);  // uint64 words per ciphertext of C learners
// sum_c W_c x_c over C learners (any C: groups of 16 folded into a running sum), weight limbs
// wl_dev [C][L][2]; rows = K * 2 * L ciphertext polynomials
void launch_wavg_packed(const uint64_t* arena, const uint32_t* wl_dev, uint32_t C, uint64_t rows, uint32_t L,
                        uint32_t logN, const ArenaPack& ap, const TowerConst* tc, uint64_t* out, hipStream_t s);
// The general form: C inputs whose rows are laid out for `crow` learners (C for an arena; 1 for C
// stacked C = 1 packed batches lstride dwords apart -- lstride 0 = the arena's adjacent slices);
// the result as uint64 [K][2][L][N] at out, or (pout != null) packed in the C = 1 layout.
void launch_wavg_packed_ex(const uint32_t* in, const uint32_t* wl_dev, uint32_t C, uint32_t crow, uint64_t lstride,
                           uint64_t rows, uint32_t L, uint32_t logN, const ArenaPack& ap, const TowerConst* tc,
                           uint64_t* out, uint32_t* pout, hipStream_t s);
// Packs rows [row0, row0 + rows) of learner `learner`'s [K][2][L][N] batch (src holds exactly those
// rows' residues, 512 per row) into its arena slices; *bad |= 1 when a residue is >= q_t.
void launch_arena_pack(const uint64_t* src, uint64_t row0, uint64_t rows, uint32_t C, uint32_t learner,
                       uint32_t L, uint32_t logN, const ArenaPack& ap, const TowerConst* tc, uint64_t* arena,
                       uint32_t* bad, hipStream_t s);
// Packed wire blobs: K ciphertexts [K][2][L][N] <-> the arena's slice format with C = 1 (ap from the
// towers the buffer holds); pack flags *bad when a residue is >= q_t.
void launch_blob_pack(const uint64_t* src, uint64_t K, uint32_t L, uint32_t logN, const ArenaPack& ap,
                      const TowerConst* tc, uint32_t* dst, uint32_t* bad, hipStream_t s);
void launch_blob_unpack(const uint32_t* src, uint64_t K, uint32_t L, uint32_t logN, const ArenaPack& ap,
                        uint64_t* dst, hipStream_t s);
// Residue runs of an upload landed raw (a PALISADE archive's byte range with its tower headers): run j is
// run_bytes bytes at raw + src_off[j] (any alignment) -> dst + j * run_bytes (16-B aligned)
void launch_gather_runs(const uint8_t* raw, const uint64_t* src_off, uint64_t runs, uint32_t run_bytes, uint8_t* dst,
                        hipStream_t s);
void launch_modq(uint64_t* buf, uint64_t rows, uint32_t L, uint32_t logN, const TowerConst* tc,
                 hipStream_t s);
// *bad |= 1 when a residue of the [rows / (2 L)][2][L][N] batch is >= its tower's q
void launch_check_residues(const uint64_t* ct, uint64_t rows, uint32_t L, uint32_t logN, const TowerConst* tc,
                           uint32_t* bad, hipStream_t s);
void launch_ntt(uint64_t* polys, uint64_t P, uint32_t L, uint32_t logN, bool inverse,
                const DeviceTables& dt, hipStream_t s);
void launch_ntt_cols(uint64_t* polys, uint64_t P, uint32_t L, uint32_t logN, bool inverse,
                     const DeviceTables& dt, hipStream_t s);
// A flag in pinned host memory the kernels write directly (round 6): word i holds the generation of the
// last call that raised it, so a call compares it with its own generation after its one synchronisation --
// no reset before a call and no readback copy after it (each was a ~2-4 us copy-engine op plus its launch
// gap on every device encrypt / decrypt).  Words: [0] an encode value out of the fast range, [1] a
// non-finite one, [2] a decode coefficient outside the fast CRT's range, [3] a flooded decode's precision
// failure.  Written with system-scope
// stores; p == nullptr: no flag.
struct GenFlag {
  uint32_t* p = nullptr;
  uint32_t gen = 0;
};
void launch_encrypt(const Params& p, const DeviceTables& dt, const DeviceKeys& dk,
                    const double* x, uint64_t n, uint64_t K, uint64_t* ct, void* scratch,
                    const uint32_t key[8], uint64_t g0, GenFlag flag, hipStream_t s);
// encode's large-value path (|x Delta| > 2^61 somewhere in the call; PALISADE's approxFactor): the
// same ciphertexts' encryption redone with per-ciphertext scale-down exponents (kernels.hip)
void launch_encrypt_approx(const Params& p, const DeviceTables& dt, const DeviceKeys& dk, const double* x,
                           uint64_t n, uint64_t K, uint64_t* ct, void* scratch, const uint32_t key[8],
                           uint64_t g0, hipStream_t s);
size_t encrypt_scratch_bytes(const Params& p, uint64_t K);
// Decode noise flooding (PALISADE 1.11 Decode); off = exact decode.
struct DecodeNoise {
  int enabled = 0;
  double m_factor = 1.0;   // CKKS_M_FACTOR
  uint32_t p_bits = 52;    // PALISADE plaintext modulus of CKKS = scale bits
  uint32_t key[8] = {};    // ChaCha20 key, nonce (3 << 56) | (g0 + ciphertext)
  uint64_t g0 = 0;
  uint32_t* flags = nullptr;  // device: [2] = max logError
  GenFlag fail;               // word 3: the precision failure (PALISADE's Decode throws)
  int reset = 1;              // the launch's flooding resets flags [1], [2] first (a call's first chunk)
};
void launch_decrypt(const Params& p, const DeviceTables& dt, const DeviceKeys& dk,
                    const uint64_t* ct, uint64_t K, double scale, uint64_t n, double* out,
                    void* scratch, hipStream_t s, const DecodeNoise* dn = nullptr, bool sum_in = false,
                    uint32_t ct_L = 0,  // ct_L: towers of the ciphertexts (0 = p.L; >= p.L)
                    GenFlag crt_flag = GenFlag{}, bool exact = false);
// crt_flag: the fast CRT (crt_value) sets word 2 to crt_flag.gen when a coefficient's centred value is not
// in (-2^127, 2^127) over these towers -- the caller redoes the call with every tower and exact =
// true (crt_exact_kernel, any |X| <= (Q - 1) / 2).  A fast-path launch needs crt_flag.
size_t decrypt_scratch_bytes(const Params& p, uint64_t K);
void launch_keygen(const Params& p, const DeviceTables& dt, const uint32_t key[8], uint64_t* sk,
                   uint64_t* pk, void* scratch, hipStream_t s);
size_t keygen_scratch_bytes(const Params& p);

// api.cpp: the arena aggregation (ctx lock held, weights checked), refused-slot check, weights
void wavg_arena_enqueue(shelfi_ctx* ctx, const uint64_t* arena_dev, const float* w, size_t C, size_t K,
                        uint64_t* out_dev, hipStream_t s);
void wavg_arena_enqueue_packed(shelfi_ctx* ctx, const uint64_t* arena_dev, const float* w, size_t C, size_t K,
                               uint64_t* out_packed, hipStream_t s);
void sum_packed_enqueue(shelfi_ctx* ctx, const uint64_t* stacked, size_t G, size_t K, size_t stride,
                        uint64_t* out, hipStream_t s);
void arena_require_valid_locked(const shelfi_ctx* ctx, const uint64_t* a, size_t words);
void check_wavg_weights(const float* w, size_t C, double delta);
// comm.cpp: drop the context's RCCL communicator (if any)
void comm_release(shelfi_ctx* ctx);
// eval.cpp: drop the relinearization key (keys_only) or all EvalMult / ModReduce state
void eval_release(shelfi_ctx* ctx, bool keys_only);
// eval.cpp: install cryptodir's key-eval-mult.txt when it belongs to the loaded keys
void load_evalkey_if_present(shelfi_ctx* ctx, const std::string& dir);
// eval.cpp: NTT / CRT tables of Q_l (towers q_0 .. q_{Ll-1}) for decrypt at a level
const DeviceTables& level_tables(shelfi_ctx* ctx, uint32_t Ll);
// api.cpp helpers shared with eval.cpp
void seed_to_key(uint64_t seed, uint32_t key[8]);
void os_random(void* buf, size_t n);
void require_keys(const shelfi_ctx* ctx);

// ---- EvalMult (ct x ct) + relinearization, ModReduce (keyswitch.hip) ----
// PALISADE 1.11 HYBRID key switching: Q_l split into digits of alpha towers, special
// primes P = p_0 .. p_{kP-1}; the key is [2][dnum][L + kP][N] (b-vector, a-vector).
struct KsArgs {
  uint32_t Ll, kP, T, dn, alpha, logN, Lfull, dnFull;
  const uint64_t* mu_inv;     // [dn][alpha] ((Q_j / q_i) mod q_i)^-1 mod q_i
  const uint64_t* mu_inv_sh;  // Shoup companions
  const uint64_t* mu_hat;     // [dn][alpha][T] (Q_j / q_i) mod target tower t
  const uint64_t* md_inv;     // [kP] ((P / p_m) mod p_m)^-1 mod p_m
  const uint64_t* md_inv_sh;
  const uint64_t* md_hat;     // [kP][Ll] (P / p_m) mod q_t
  const uint64_t* pinv;       // [Ll] P^-1 mod q_t
  const uint64_t* pinv_sh;
  const TowerConst* tq;       // towers of Q_l (the context's, prefix)
  const TowerConst* te;       // towers of Q_l u P (extended tables)
};
// out = relinearized (a x b): tensor, ModUp per digit, inner product with the key,
// ModDown.  a, b, out [K][2][Ll][N] (out may alias a or b); scratch = ks_scratch_bytes(.., K).
// dtq: tables of Q (prefix Q_l used); dte: Q_l u P; dtf[j]: digit j's foreign towers.
size_t ks_scratch_bytes(uint32_t Ll, uint32_t kP, uint32_t dn, uint32_t alpha, uint32_t N, uint64_t K);
void launch_eval_mult(const KsArgs& a, const DeviceTables& dtq, const DeviceTables& dte,
                      const DeviceTables* dtf, const uint64_t* evk, const uint64_t* evk_sh, const uint64_t* x,
                      const uint64_t* y, uint64_t K, uint64_t* out, void* scratch, hipStream_t s);
// ModReduce: in [K][2][Ll][N] -> out [K][2][Ll-1][N] (EVAL); qlinv[t] = q_{Ll-1}^-1 mod q_t
struct RescaleConst {
  uint64_t ql;  // the dropped modulus q_{Ll-1}
  uint64_t qlinv[kMaxTowers], qlinv_sh[kMaxTowers];
};
size_t rescale_scratch_bytes(uint32_t Ll, uint32_t N, uint64_t K);
void launch_rescale(const DeviceTables& dt, uint32_t Ll, uint32_t logN, const RescaleConst& rc,
                    const uint64_t* in, uint64_t K, uint64_t* out, void* scratch, hipStream_t s);
// EvalMultKeyGen on the device: dte = tables of Q u P (T0 = L + kP towers), sk [L][N] EVAL
struct EvkGenConst {
  uint64_t q0;                // s is read centred from tower 0
  uint64_t pmod[kMaxTowers];  // P mod q_t
  uint32_t L, kP, dnum, alpha, logN;
};
size_t evk_scratch_bytes(uint32_t L, uint32_t kP, uint32_t N);
void launch_evk_keygen(const EvkGenConst& g, const DeviceTables& dtq, const DeviceTables& dte,
                       const uint64_t* cdt, int cdt_len, const uint32_t key[8], const uint64_t* sk,
                       uint64_t* evk, void* scratch, hipStream_t s);

}  // namespace shelfi

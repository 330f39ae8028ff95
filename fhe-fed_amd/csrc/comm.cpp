// comm.cpp — the C-ABI multi-GPU combine over RCCL (SURVEY §8 b/e): per-context
// communicator, and the uint64 SUM reduce / allreduce / reduce-scatter of per-rank
// partial aggregates followed by the mod-q fold.
//
// Why this is exact: each rank's partial is sum_{c in rank} W_c ct_c mod q_t, a residue
// below q_t < 2^60; a uint64 sum of W <= 16 of them stays below 2^64, and EvalAdd is
// order-independent, so RCCL's reduction order (ring, tree) cannot change the result.
// The fold back into [0, q_t) is launch_modq (kernels.hip).
//
// RCCL is opened with dlopen(RTLD_LOCAL | RTLD_DEEPBIND) on first use, from the ROCm
// install this library's HIP runtime comes from: a PyTorch process already carries its
// own librccl (same soname, built against its own HIP runtime), and a stream of ours
// must not reach a communicator of theirs.  Nothing here runs unless a communicator is
// created, so single-GPU users never load RCCL.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/shelfi.h"
#include "shelfi_internal.h"

namespace shelfi {
namespace {

struct Rccl {
  void* handle = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclReduce) reduce = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  std::string load_error;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* env = getenv("SHELFI_RCCL_LIB");
    const char* cands[] = {env, "/opt/rocm/lib/librccl.so.1", "librccl.so.1"};
    for (const char* path : cands) {
      if (!path || !*path) continue;
      r.handle = dlopen(path, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
      if (r.handle) break;
      r.load_error = dlerror();
    }
    if (!r.handle) return;
#define SHELFI_SYM(field, name)                                                  \
  r.field = reinterpret_cast<decltype(r.field)>(dlsym(r.handle, #name));          \
  if (!r.field) {                                                                \
    r.load_error = std::string("librccl lacks ") + #name;                        \
    r.handle = nullptr;                                                          \
    return;                                                                      \
  }
    SHELFI_SYM(get_unique_id, ncclGetUniqueId)
    SHELFI_SYM(comm_init_rank, ncclCommInitRank)
    SHELFI_SYM(comm_destroy, ncclCommDestroy)
    SHELFI_SYM(reduce, ncclReduce)
    SHELFI_SYM(all_reduce, ncclAllReduce)
    SHELFI_SYM(reduce_scatter, ncclReduceScatter)
    SHELFI_SYM(error_string, ncclGetErrorString)
    SHELFI_SYM(send, ncclSend)
    SHELFI_SYM(recv, ncclRecv)
    SHELFI_SYM(group_start, ncclGroupStart)
    SHELFI_SYM(group_end, ncclGroupEnd)
#undef SHELFI_SYM
  });
  if (!r.handle) throw Error{SHELFI_ERR_DEVICE, "RCCL unavailable: " + r.load_error};
  return r;
}

void check(ncclResult_t rc, const char* what) {
  if (rc != ncclSuccess)
    throw Error{SHELFI_ERR_DEVICE, std::string(what) + ": " + rccl().error_string(rc)};
}

template <class F>
int guarded_comm(F&& f) {
  try {
    f();
    return SHELFI_OK;
  } catch (const Error& e) {
    set_error(e.msg);
    return e.code;
  } catch (const std::exception& e) {
    set_error(e.what());
    return SHELFI_ERR_DEVICE;
  }
}

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    SHELFI_HIP(hipSetDevice(dev));
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

ncclComm_t comm_of(shelfi_ctx* ctx) {
  if (!ctx->comm) throw Error{SHELFI_ERR_STATE, "no communicator: call shelfi_comm_init first"};
  return reinterpret_cast<ncclComm_t>(ctx->comm);
}

}  // namespace

void comm_release(shelfi_ctx* ctx) {
  if (!ctx) return;
  if (ctx->comm_stream) (void)hipStreamSynchronize(ctx->comm_stream);
  if (ctx->comm) {
    (void)rccl().comm_destroy(reinterpret_cast<ncclComm_t>(ctx->comm));
    ctx->comm = nullptr;
    ctx->comm_rank = 0;
    ctx->comm_world = 0;
  }
  for (hipEvent_t e : ctx->comm_events) (void)hipEventDestroy(e);
  ctx->comm_events.clear();
  if (ctx->comm_stream) (void)hipStreamDestroy(ctx->comm_stream);
  ctx->comm_stream = nullptr;
}

}  // namespace shelfi

using namespace shelfi;

extern "C" {

int shelfi_comm_unique_id(uint8_t* id_out) {
  if (!id_out) return SHELFI_ERR_ARG;
  return guarded_comm([&] {
    static_assert(sizeof(ncclUniqueId) == SHELFI_COMM_ID_BYTES, "unique id size");
    ncclUniqueId id;
    check(rccl().get_unique_id(&id), "ncclGetUniqueId");
    std::memcpy(id_out, &id, sizeof(id));
  });
}

int shelfi_comm_init(shelfi_ctx* ctx, const uint8_t* id, int rank, int world) {
  if (!ctx || !id || world < 1 || rank < 0 || rank >= world) return SHELFI_ERR_ARG;
  if (world > kMaxCommRanks) {
    set_error("world size above 16: a uint64 sum of the partial aggregates could wrap");
    return SHELFI_ERR_ARG;
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  return guarded_comm([&] {
    comm_release(ctx);
    DevGuard g(ctx->device);
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclComm_t c = nullptr;
    check(rccl().comm_init_rank(&c, world, uid, rank), "ncclCommInitRank");
    ctx->comm = c;
    ctx->comm_rank = rank;
    ctx->comm_world = world;
  });
}

int shelfi_comm_destroy(shelfi_ctx* ctx) {
  if (!ctx) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);
  return guarded_comm([&] {
    DevGuard g(ctx->device);
    comm_release(ctx);
  });
}

int shelfi_dev_reduce(shelfi_ctx* ctx, uint64_t* partial_dev, size_t K, int root, void* stream) {
  if (!ctx || (K && !partial_dev)) return SHELFI_ERR_ARG;
  // comm_init/comm_destroy replace the communicator under ctx->mu
  std::lock_guard<std::mutex> lk(ctx->mu);
  return guarded_comm([&] {
    ncclComm_t c = comm_of(ctx);
    if (root < 0 || root >= ctx->comm_world) throw Error{SHELFI_ERR_ARG, "root outside the communicator"};
    if (!K) return;
    DevGuard g(ctx->device);
    const Params& p = ctx->p;
    hipStream_t s = (hipStream_t)stream;
    const size_t words = K * 2ull * p.L * p.N;
    check(rccl().reduce(partial_dev, partial_dev, words, ncclUint64, ncclSum, root, c, s), "ncclReduce");
    if (ctx->comm_rank == root) launch_modq(partial_dev, (uint64_t)K * 2 * p.L, p.L, p.logN, ctx->dt.tc, s);
  });
}

int shelfi_dev_allreduce(shelfi_ctx* ctx, uint64_t* partial_dev, size_t K, void* stream) {
  if (!ctx || (K && !partial_dev)) return SHELFI_ERR_ARG;
  // comm_init/comm_destroy replace the communicator under ctx->mu
  std::lock_guard<std::mutex> lk(ctx->mu);
  return guarded_comm([&] {
    ncclComm_t c = comm_of(ctx);
    if (!K) return;
    DevGuard g(ctx->device);
    const Params& p = ctx->p;
    hipStream_t s = (hipStream_t)stream;
    const size_t words = K * 2ull * p.L * p.N;
    check(rccl().all_reduce(partial_dev, partial_dev, words, ncclUint64, ncclSum, c, s), "ncclAllReduce");
    launch_modq(partial_dev, (uint64_t)K * 2 * p.L, p.L, p.logN, ctx->dt.tc, s);
  });
}

int shelfi_dev_reduce_scatter(shelfi_ctx* ctx, const uint64_t* partial_dev, size_t K, uint64_t* out_dev,
                              void* stream) {
  if (!ctx || (K && (!partial_dev || !out_dev))) return SHELFI_ERR_ARG;
  // comm_init/comm_destroy replace the communicator under ctx->mu
  std::lock_guard<std::mutex> lk(ctx->mu);
  return guarded_comm([&] {
    ncclComm_t c = comm_of(ctx);
    const size_t W = (size_t)ctx->comm_world;
    if (K % W) throw Error{SHELFI_ERR_ARG, "reduce_scatter needs K divisible by the world size"};
    if (!K) return;
    DevGuard g(ctx->device);
    const Params& p = ctx->p;
    hipStream_t s = (hipStream_t)stream;
    const size_t Ks = K / W, words = Ks * 2ull * p.L * p.N;
    check(rccl().reduce_scatter(partial_dev, out_dev, words, ncclUint64, ncclSum, c, s), "ncclReduceScatter");
    launch_modq(out_dev, (uint64_t)Ks * 2 * p.L, p.L, p.logN, ctx->dt.tc, s);
  });
}

size_t shelfi_combine_share_cts(const shelfi_ctx* ctx, size_t K) {
  if (!ctx || !ctx->comm || ctx->comm_world < 1) return 0;
  const size_t W = (size_t)ctx->comm_world;
  return (K + W - 1) / W;
}

// The pipelined learner-sharded combine (SURVEY §8 e): rank r owns the global ciphertexts
// [r Ks, (r+1) Ks), Ks = ceil(K / W).  Piece j covers sub-slice j (Kp = ceil(Ks / P)
// ciphertexts) of EVERY rank's slice: the local arena aggregation of those W runs is written
// to a [W][kp] send region on the caller's stream, an event hands it to the context's comm
// stream, and one ncclReduceScatter delivers this rank's sub-slice straight into
// share[j Kp ..] while piece j+1 is being aggregated.  The share comes out contiguous, as
// the unpipelined reduce_scatter's would.  fold = 1: the mod-q fold of each piece follows its
// collective on the comm stream; fold = 0: left to the consumer (shelfi_dev_decrypt_sum).
int shelfi_dev_combine_arena(shelfi_ctx* ctx, const uint64_t* arena_dev, const float* w, size_t C, size_t K,
                             size_t pieces, uint64_t* send_dev, uint64_t* share_dev, int fold, void* stream) {
  if (!ctx || !w || !C || (K && (!arena_dev || !send_dev || !share_dev))) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);
  return guarded_comm([&] {
    ncclComm_t c = comm_of(ctx);
    check_wavg_weights(w, C, ctx->p.delta);
    const Params& p = ctx->p;
    const size_t ctw = 2ull * p.L * p.N;
    const size_t acw = (size_t)arena_ct_words(p, C);  // arena words per ciphertext (packed, all learners)
    arena_require_valid_locked(ctx, arena_dev, acw * K);
    if (!K) return;
    DevGuard g(ctx->device);
    const size_t W = (size_t)ctx->comm_world;
    const size_t Ks = (K + W - 1) / W;
    const size_t P = std::max<size_t>(1, std::min(pieces ? pieces : 1, Ks));
    const size_t Kp = (Ks + P - 1) / P;
    hipStream_t s = (hipStream_t)stream;
    if (!ctx->comm_stream) SHELFI_HIP(hipStreamCreateWithFlags(&ctx->comm_stream, hipStreamNonBlocking));
    while (ctx->comm_events.size() < P + 1) {
      hipEvent_t e = nullptr;
      SHELFI_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      ctx->comm_events.push_back(e);
    }
    hipStream_t cs = ctx->comm_stream;
    // the comm stream must not overwrite a share the caller's stream may still be reading
    SHELFI_HIP(hipEventRecord(ctx->comm_events[P], s));
    SHELFI_HIP(hipStreamWaitEvent(cs, ctx->comm_events[P], 0));
    for (size_t j = 0; j < P; ++j) {
      const size_t kj0 = j * Kp;
      if (kj0 >= Ks) break;
      const size_t kn = std::min(Kp, Ks - kj0);
      uint64_t* send = send_dev + W * kj0 * ctw;  // [W][kn] ciphertexts
      for (size_t gr = 0; gr < W; ++gr) {
        const size_t a = gr * Ks + kj0;
        const size_t cnt = a < K ? std::min(kn, K - a) : 0;
        if (cnt) wavg_arena_enqueue(ctx, arena_dev + a * acw, w, C, cnt, send + gr * kn * ctw, s);
        if (cnt < kn)  // padding past K: zero, the additive identity
          SHELFI_HIP(hipMemsetAsync(send + (gr * kn + cnt) * ctw, 0, (kn - cnt) * ctw * 8, s));
      }
      SHELFI_HIP(hipEventRecord(ctx->comm_events[j], s));
      SHELFI_HIP(hipStreamWaitEvent(cs, ctx->comm_events[j], 0));
      uint64_t* dst = share_dev + kj0 * ctw;
      check(rccl().reduce_scatter(send, dst, kn * ctw, ncclUint64, ncclSum, c, cs), "ncclReduceScatter");
      if (fold) launch_modq(dst, (uint64_t)kn * 2 * p.L, p.L, p.logN, ctx->dt.tc, cs);
    }
    SHELFI_HIP(hipEventRecord(ctx->comm_events[P], cs));
    SHELFI_HIP(hipStreamWaitEvent(s, ctx->comm_events[P], 0));  // the share is ready on `stream`
  });
}

// The packed share exchange (round 4): the same pieces as
// shelfi_dev_combine_arena, but each rank's partial of piece j is written PACKED (the C = 1 slice
// format, sum_t U_t bits per coefficient: 218 of 256 at 2^15 / L4) into send [W][kn], exchanged by
// one grouped ncclSend / ncclRecv all-to-all (rank h's block of every rank lands in recv [W][kn]),
// and summed locally with unit weights (sum_packed_enqueue: the mod-q fold included) into share.
// The xGMI bytes per rank are (W - 1) / W of the packed partial instead of the uint64 one (0.85x at
// 2^15 / L4); the local sum reads W packed blocks and writes the uint64 share.  Bit-identical to the
// reduce-scatter combine (EvalAdd is order-independent).  send and recv hold W * Ks packed
// ciphertexts (shelfi_arena_words(ctx, 1, W * Ks) uint64 words each).
int shelfi_dev_combine_arena_packed(shelfi_ctx* ctx, const uint64_t* arena_dev, const float* w, size_t C, size_t K,
                                    size_t pieces, uint64_t* send_dev, uint64_t* recv_dev, uint64_t* share_dev,
                                    void* stream) {
  if (!ctx || !w || !C || (K && (!arena_dev || !send_dev || !recv_dev || !share_dev))) return SHELFI_ERR_ARG;
  std::lock_guard<std::mutex> lk(ctx->mu);
  return guarded_comm([&] {
    ncclComm_t c = comm_of(ctx);
    check_wavg_weights(w, C, ctx->p.delta);
    const Params& p = ctx->p;
    const size_t ctw = 2ull * p.L * p.N;
    const size_t pcw = (size_t)arena_ct_words(p, 1);  // packed uint64 words per ciphertext (C = 1)
    const size_t acw = (size_t)arena_ct_words(p, C);
    arena_require_valid_locked(ctx, arena_dev, acw * K);
    if (!K) return;
    DevGuard g(ctx->device);
    const size_t W = (size_t)ctx->comm_world;
    const size_t Ks = (K + W - 1) / W;
    const size_t P = std::max<size_t>(1, std::min(pieces ? pieces : 1, Ks));
    const size_t Kp = (Ks + P - 1) / P;
    hipStream_t s = (hipStream_t)stream;
    if (!ctx->comm_stream) SHELFI_HIP(hipStreamCreateWithFlags(&ctx->comm_stream, hipStreamNonBlocking));
    while (ctx->comm_events.size() < P + 1) {
      hipEvent_t e = nullptr;
      SHELFI_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      ctx->comm_events.push_back(e);
    }
    hipStream_t cs = ctx->comm_stream;
    SHELFI_HIP(hipEventRecord(ctx->comm_events[P], s));
    SHELFI_HIP(hipStreamWaitEvent(cs, ctx->comm_events[P], 0));
    for (size_t j = 0; j < P; ++j) {
      const size_t kj0 = j * Kp;
      if (kj0 >= Ks) break;
      const size_t kn = std::min(Kp, Ks - kj0);
      uint64_t* send = send_dev + W * kj0 * pcw;  // [W][kn] packed ciphertexts
      uint64_t* recv = recv_dev + W * kj0 * pcw;
      for (size_t gr = 0; gr < W; ++gr) {
        const size_t a = gr * Ks + kj0;
        const size_t cnt = a < K ? std::min(kn, K - a) : 0;
        if (cnt) wavg_arena_enqueue_packed(ctx, arena_dev + a * acw, w, C, cnt, send + gr * kn * pcw, s);
        if (cnt < kn)  // padding past K: packed zeros, the additive identity
          SHELFI_HIP(hipMemsetAsync(send + (gr * kn + cnt) * pcw, 0, (kn - cnt) * pcw * 8, s));
      }
      SHELFI_HIP(hipEventRecord(ctx->comm_events[j], s));
      SHELFI_HIP(hipStreamWaitEvent(cs, ctx->comm_events[j], 0));
      check(rccl().group_start(), "ncclGroupStart");
      for (size_t h = 0; h < W; ++h) {
        check(rccl().send(send + h * kn * pcw, kn * pcw, ncclUint64, (int)h, c, cs), "ncclSend");
        check(rccl().recv(recv + h * kn * pcw, kn * pcw, ncclUint64, (int)h, c, cs), "ncclRecv");
      }
      check(rccl().group_end(), "ncclGroupEnd");
      sum_packed_enqueue(ctx, recv, W, kn, kn * pcw, share_dev + kj0 * ctw, cs);
    }
    SHELFI_HIP(hipEventRecord(ctx->comm_events[P], cs));
    SHELFI_HIP(hipStreamWaitEvent(s, ctx->comm_events[P], 0));  // the share is ready on `stream`
  });
}

int shelfi_comm_info(const shelfi_ctx* ctx, int* rank, int* world) {
  if (!ctx) return SHELFI_ERR_ARG;
  if (rank) *rank = ctx->comm ? ctx->comm_rank : -1;
  if (world) *world = ctx->comm ? ctx->comm_world : 0;
  return SHELFI_OK;
}

}  // extern "C"

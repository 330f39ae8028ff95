// Pinned staging rings + parallel memcpy for the bytes API (see host_stage.h).
#include "host_stage.h"

#include <immintrin.h>
#include <sched.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "shelfi_internal.h"

namespace shelfi {

int default_copy_threads() {
  if (const char* e = std::getenv("SHELFI_COPY_THREADS")) {
    const int v = std::atoi(e);
    if (v >= 1) return std::min(v, 64);
  }
  cpu_set_t set;
  int n = 1;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
  return std::max(1, std::min(8, n));
}

int default_h2d_copy_threads() {
  if (const char* e = std::getenv("SHELFI_H2D_COPY_THREADS")) {
    const int v = std::atoi(e);
    if (v >= 1) return std::min(v, 64);
  }
  return 4;
}

void advise_huge(void* p, size_t n) {
  const uintptr_t kHuge = 2u << 20;
  if (n < 2 * kHuge) return;
  const uintptr_t a = ((uintptr_t)p + kHuge - 1) & ~(kHuge - 1);
  const uintptr_t b = ((uintptr_t)p + n) & ~(kHuge - 1);
  if (b > a) (void)madvise((void*)a, b - a, MADV_HUGEPAGE);  // advice only; failure is harmless
}

// Copy with non-temporal (streaming) stores: the destination of a staging copy is read
// next by a DMA engine or by the caller much later, so the stores skip the read-for-
// ownership of every destination line and do not evict the source from the cache.
__attribute__((target("avx512f"))) static void copy_nt512(uint8_t* d, const uint8_t* s, size_t n) {
  const size_t head = std::min(n, (size_t)((64 - ((uintptr_t)d & 63)) & 63));
  std::memcpy(d, s, head);
  d += head;
  s += head;
  n -= head;
  const size_t body = n & ~(size_t)255;
  for (size_t i = 0; i < body; i += 256) {
    const __m512i a = _mm512_loadu_si512(s + i), b = _mm512_loadu_si512(s + i + 64),
                  c = _mm512_loadu_si512(s + i + 128), e = _mm512_loadu_si512(s + i + 192);
    _mm512_stream_si512((__m512i*)(d + i), a);
    _mm512_stream_si512((__m512i*)(d + i + 64), b);
    _mm512_stream_si512((__m512i*)(d + i + 128), c);
    _mm512_stream_si512((__m512i*)(d + i + 192), e);
  }
  _mm_sfence();
  std::memcpy(d + body, s + body, n - body);
}

static bool use_nt_copy() {
  if (const char* e = std::getenv("SHELFI_NT_COPY")) return std::atoi(e) != 0;
  return true;
}

void copy_bytes(uint8_t* d, const uint8_t* s, size_t n, bool nt) {
  static const bool has512 = __builtin_cpu_supports("avx512f");
  if (nt && has512 && n >= (64u << 10)) copy_nt512(d, s, n);
  else std::memcpy(d, s, n);
}

// ------------------------------------------------------------- CopyPool ----
CopyPool::CopyPool(int threads) : parts_(std::max(1, threads)), nt_(use_nt_copy()) {
  workers_.reserve(parts_ - 1);
  for (int i = 1; i < parts_; ++i) workers_.emplace_back([this, i] { run(i); });
}

CopyPool::~CopyPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_.store(true);
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
}

// Share `id` of the current list: bytes [id T/P, (id+1) T/P) of the concatenated
// jobs, page-aligned so first-touch faults of a fresh destination land on different
// threads.
void CopyPool::share(int id) {
  if (id >= active_) return;
  const size_t per = ((total_ / active_) + 4095) & ~size_t(4095);
  const size_t a = std::min(total_, per * (size_t)id), b = std::min(total_, per * (size_t)(id + 1));
  size_t base = 0;
  for (size_t j = 0; j < njobs_ && base < b; ++j) {
    const CopyJob& J = jobs_[j];
    const size_t lo = std::max(a, base), hi = std::min(b, base + J.n);
    if (hi > lo) copy_bytes(J.dst + (lo - base), J.src + (lo - base), hi - lo, nt_);
    base += J.n;
  }
}

void CopyPool::run(int id) {
  uint64_t seen = 0;
  for (;;) {
    uint64_t g = gen_.load(std::memory_order_acquire);
    for (int spin = 0; g == seen && spin < (1 << 14) && !stop_.load(std::memory_order_relaxed); ++spin) {
      __builtin_ia32_pause();
      g = gen_.load(std::memory_order_acquire);
    }
    if (g == seen) {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_.load() || gen_.load(std::memory_order_acquire) != seen; });
      g = gen_.load(std::memory_order_acquire);
    }
    if (stop_.load()) return;
    seen = g;
    share(id);
    pending_.fetch_sub(1, std::memory_order_acq_rel);
  }
}

void CopyPool::copy_many(const CopyJob* jobs, size_t njobs, int parts) {
  size_t total = 0;
  for (size_t j = 0; j < njobs; ++j) total += jobs[j].n;
  if (total == 0) return;
  const int active = (parts >= 1 && parts < parts_) ? parts : parts_;
  if (workers_.empty() || active == 1 || total < (512u << 10)) {
    for (size_t j = 0; j < njobs; ++j) copy_bytes(jobs[j].dst, jobs[j].src, jobs[j].n, nt_);
    return;
  }
  jobs_ = jobs;
  njobs_ = njobs;
  total_ = total;
  active_ = active;
  pending_.store((int)workers_.size(), std::memory_order_relaxed);
  {
    std::lock_guard<std::mutex> lk(mu_);  // no lost wake-up for a worker about to sleep
    gen_.fetch_add(1, std::memory_order_release);
  }
  cv_.notify_all();
  share(0);
  while (pending_.load(std::memory_order_acquire) != 0) __builtin_ia32_pause();
}

void CopyPool::copy(void* dst, const void* src, size_t n) {
  const CopyJob j{(uint8_t*)dst, (const uint8_t*)src, n};
  copy_many(&j, 1);
}

// --------------------------------------------------------------- Stager ----
Stager::Stager(size_t slot_bytes, int n_in, int n_out, int threads)
    : slot_bytes_(slot_bytes), in_(n_in), out_(n_out), pool_(threads),
      h2d_parts_(std::min(pool_.threads(), default_h2d_copy_threads())) {
  if (const char* e = std::getenv("SHELFI_STAGE_TRACE")) trace_ = std::atoi(e) != 0;
  try {
    for (auto* ring : {&in_, &out_})
      for (Slot& s : *ring) {
        SHELFI_HIP(hipHostMalloc((void**)&s.host, slot_bytes_, hipHostMallocDefault));
        SHELFI_HIP(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
      }
  } catch (...) {
    for (auto* ring : {&in_, &out_})
      for (Slot& s : *ring) {
        if (s.host) (void)hipHostFree(s.host);
        if (s.ev) (void)hipEventDestroy(s.ev);
      }
    throw;
  }
}

Stager::~Stager() {
  abort();
  for (auto* ring : {&in_, &out_})
    for (Slot& s : *ring) {
      if (s.host) (void)hipHostFree(s.host);
      if (s.ev) (void)hipEventDestroy(s.ev);
    }
}

// Drain the oldest pending output if its DMA is done (or wait for it when `block`).
bool Stager::drain_front(bool block) {
  if (pending_.empty()) return false;
  Slot& s = out_[pending_.front()];
  if (block) {
    SHELFI_HIP(hipEventSynchronize(s.ev));
  } else {
    const hipError_t e = hipEventQuery(s.ev);
    if (e == hipErrorNotReady) return false;
    if (e != hipSuccess)
      throw Error{SHELFI_ERR_DEVICE, std::string("staged copy: ") + hipGetErrorString(e)};
  }
  const auto t0 = std::chrono::steady_clock::now();
  pool_.copy_many(s.out_jobs.data(), s.out_jobs.size());
  if (trace_) t_drain_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  s.out_jobs.clear();
  s.pending = false;
  pending_.pop_front();
  return true;
}

void Stager::poll() {
  while (drain_front(false)) {
  }
}

// Wait until an input slot's previous DMA has read it, draining outputs meanwhile.
void Stager::wait_in_slot(Slot& sl) {
  if (!sl.used) return;
  const auto t0 = std::chrono::steady_clock::now();
  struct Acc {
    bool on;
    double& t;
    std::chrono::steady_clock::time_point t0;
    ~Acc() {
      if (on) t += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
  } acc{trace_, t_wait_, t0};
  for (;;) {
    const hipError_t e = hipEventQuery(sl.ev);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady)
      throw Error{SHELFI_ERR_DEVICE, std::string("staged copy: ") + hipGetErrorString(e)};
    if (!drain_front(false)) std::this_thread::yield();
  }
}

void Stager::h2dv(void* dev, const HostPiece* pieces, size_t np, hipStream_t s) {
  uint8_t* dst = (uint8_t*)dev;
  size_t pi = 0, po = 0;  // current piece, offset inside it
  std::vector<CopyJob> jobs;
  while (pi < np) {
    Slot& sl = in_[in_next_++ % in_.size()];
    wait_in_slot(sl);
    size_t fill = 0;
    jobs.clear();
    const size_t cap = ramp_ < 2 ? slot_bytes_ >> (2 - ramp_) : slot_bytes_;
    while (pi < np && fill < cap) {
      const size_t take = std::min(pieces[pi].n - po, cap - fill);
      if (take) jobs.push_back(CopyJob{sl.host + fill, pieces[pi].p + po, take});
      fill += take;
      po += take;
      if (po == pieces[pi].n) {
        ++pi;
        po = 0;
      }
    }
    if (!fill) break;
    if (ramp_ < 2) ++ramp_;
    const auto t0 = std::chrono::steady_clock::now();
    pool_.copy_many(jobs.data(), jobs.size(), h2d_parts_);
    if (trace_) {
      t_fill_ += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      b_in_ += fill;
    }
    SHELFI_HIP(hipMemcpyAsync(dst, sl.host, fill, hipMemcpyHostToDevice, s));
    SHELFI_HIP(hipEventRecord(sl.ev, s));
    sl.used = true;
    dst += fill;
  }
}

void Stager::h2d(void* dev, const void* host, size_t n, hipStream_t s) {
  const HostPiece p{(uint8_t*)host, n};
  h2dv(dev, &p, 1, s);
}

void Stager::d2hv(const HostPiece* pieces, size_t np, const void* dev, hipStream_t s) {
  const uint8_t* src = (const uint8_t*)dev;
  size_t pi = 0, po = 0;
  while (pi < np) {
    const size_t idx = out_next_++ % out_.size();
    Slot& sl = out_[idx];
    while (sl.pending) drain_front(true);  // FIFO: the oldest pending is drained first
    size_t fill = 0;
    sl.out_jobs.clear();
    while (pi < np && fill < slot_bytes_) {
      const size_t take = std::min(pieces[pi].n - po, slot_bytes_ - fill);
      if (take) sl.out_jobs.push_back(CopyJob{pieces[pi].p + po, sl.host + fill, take});
      fill += take;
      po += take;
      if (po == pieces[pi].n) {
        ++pi;
        po = 0;
      }
    }
    if (!fill) break;
    SHELFI_HIP(hipMemcpyAsync(sl.host, src, fill, hipMemcpyDeviceToHost, s));
    SHELFI_HIP(hipEventRecord(sl.ev, s));
    sl.used = true;
    sl.pending = true;
    pending_.push_back(idx);
    src += fill;
  }
}

void Stager::d2h(void* host, const void* dev, size_t n, hipStream_t s) {
  const HostPiece p{(uint8_t*)host, n};
  d2hv(&p, 1, dev, s);
}

void Stager::finish() {
  while (drain_front(true)) {
  }
  for (Slot& sl : in_)
    if (sl.used) SHELFI_HIP(hipEventSynchronize(sl.ev));
  if (trace_ && (b_in_ || t_drain_ > 0)) {
    std::fprintf(stderr, "[stage] in %.1f MB: fill %.2f ms (%.1f GB/s), wait in-slot %.2f ms, drain %.2f ms\n",
                 b_in_ / 1e6, t_fill_ * 1e3, t_fill_ > 0 ? b_in_ / t_fill_ / 1e9 : 0.0, t_wait_ * 1e3,
                 t_drain_ * 1e3);
    t_fill_ = t_wait_ = t_drain_ = 0;
    b_in_ = 0;
  }
}

void Stager::abort() noexcept {
  for (auto* ring : {&in_, &out_})
    for (Slot& sl : *ring) {
      if (sl.used) (void)hipEventSynchronize(sl.ev);
      sl.pending = false;
      sl.out_jobs.clear();
    }
  pending_.clear();
}

// ------------------------------------------------------------ AsyncDrain ----
AsyncDrain::AsyncDrain(int threads) : pool_(threads) { worker_ = std::thread([this] { run(); }); }

AsyncDrain::~AsyncDrain() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  worker_.join();
  for (int i = 0; i < 2; ++i)
    if (buf_[i]) (void)hipHostFree(buf_[i]);
}

uint8_t* AsyncDrain::buffer(int slot, size_t bytes) {
  wait_slot(slot);
  if (cap_[slot] < bytes) {
    if (buf_[slot]) SHELFI_HIP(hipHostFree(buf_[slot]));
    buf_[slot] = nullptr;
    cap_[slot] = 0;
    SHELFI_HIP(hipHostMalloc((void**)&buf_[slot], bytes, hipHostMallocDefault));
    cap_[slot] = bytes;
  }
  return buf_[slot];
}

void AsyncDrain::wait_slot(int slot) {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&] { return busy_[slot] == 0; });
}

void AsyncDrain::post(int slot, hipEvent_t ev, std::vector<HostPiece> pieces) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    ++busy_[slot];
    q_.push_back(Job{slot, ev, std::move(pieces)});
  }
  cv_.notify_all();
}

void AsyncDrain::prefault(uint8_t* p, size_t n) {
  if (!n) return;
  {
    std::lock_guard<std::mutex> lk(mu_);
    ++prefaults_;
    q_.push_back(Job{-1, nullptr, std::vector<HostPiece>{HostPiece{p, n}}});
  }
  cv_.notify_all();
}

void AsyncDrain::finish() {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&] { return busy_[0] == 0 && busy_[1] == 0 && prefaults_ == 0; });
  if (!err_.empty()) {
    const std::string e = err_;
    err_.clear();
    throw Error{SHELFI_ERR_DEVICE, e};
  }
}

void AsyncDrain::run() {
  std::vector<CopyJob> jobs;
  for (;;) {
    Job j;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;  // stop_ with nothing left
      j = std::move(q_.front());
      q_.pop_front();
    }
    if (j.slot < 0) {  // prefault: one write per 4 KiB page (the bytes are overwritten by the drains)
      for (const HostPiece& h : j.pieces)
        for (size_t o = 0; o < h.n; o += 4096) reinterpret_cast<volatile uint8_t*>(h.p)[o] = 0;
      {
        std::lock_guard<std::mutex> lk(mu_);
        --prefaults_;
      }
      cv_.notify_all();
      continue;
    }
    const hipError_t e = hipEventSynchronize(j.ev);
    if (e == hipSuccess) {
      jobs.clear();
      size_t off = 0;
      for (const HostPiece& h : j.pieces) {
        jobs.push_back(CopyJob{h.p, buf_[j.slot] + off, h.n});
        off += h.n;
      }
      pool_.copy_many(jobs.data(), jobs.size());
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (e != hipSuccess && err_.empty()) err_ = std::string("staged copy: ") + hipGetErrorString(e);
      --busy_[j.slot];
    }
    cv_.notify_all();
  }
}

// ----------------------------------------------------------- AsyncUpload ----
AsyncUpload::AsyncUpload() { worker_ = std::thread([this] { run(); }); }

AsyncUpload::~AsyncUpload() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  worker_.join();
}

void AsyncUpload::post(void* dst, const void* src, size_t n, hipStream_t stream) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    ++pending_;
    q_.push_back(Job{dst, src, n, stream});
  }
  cv_.notify_all();
}

void AsyncUpload::wait() {
  std::unique_lock<std::mutex> lk(mu_);
  cv_.wait(lk, [&] { return pending_ == 0; });
  if (!err_.empty()) {
    const std::string e = err_;
    err_.clear();
    throw Error{SHELFI_ERR_DEVICE, e};
  }
}

void AsyncUpload::run() {
  for (;;) {
    Job j;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;
      j = q_.front();
      q_.pop_front();
    }
    const hipError_t e = hipMemcpyAsync(j.dst, j.src, j.n, hipMemcpyHostToDevice, j.stream);
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (e != hipSuccess && err_.empty()) err_ = std::string("upload: ") + hipGetErrorString(e);
      --pending_;
    }
    cv_.notify_all();
  }
}

}  // namespace shelfi

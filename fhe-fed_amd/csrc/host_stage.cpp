// Pinned staging rings + parallel memcpy for the bytes API (see host_stage.h).
#include "host_stage.h"

#include <sched.h>
#include <sys/mman.h>

#include <algorithm>
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

void advise_huge(void* p, size_t n) {
  const uintptr_t kHuge = 2u << 20;
  if (n < 2 * kHuge) return;
  const uintptr_t a = ((uintptr_t)p + kHuge - 1) & ~(kHuge - 1);
  const uintptr_t b = ((uintptr_t)p + n) & ~(kHuge - 1);
  if (b > a) (void)madvise((void*)a, b - a, MADV_HUGEPAGE);  // advice only; failure is harmless
}

// ------------------------------------------------------------- CopyPool ----
CopyPool::CopyPool(int threads) : parts_(std::max(1, threads)) {
  workers_.reserve(parts_ - 1);
  for (int i = 1; i < parts_; ++i) workers_.emplace_back([this, i] { run(i); });
}

CopyPool::~CopyPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_go_.notify_all();
  for (auto& t : workers_) t.join();
}

// Share `id` of the current job: page-aligned pieces so first-touch faults of a fresh
// destination land on different threads.
static void piece(uint8_t* dst, const uint8_t* src, size_t n, int id, int parts) {
  const size_t per = ((n / parts) + 4095) & ~size_t(4095);
  const size_t a = std::min(n, per * (size_t)id), b = std::min(n, per * (size_t)(id + 1));
  if (b > a) std::memcpy(dst + a, src + a, b - a);
}

void CopyPool::run(int id) {
  uint64_t seen = 0;
  for (;;) {
    uint8_t* dst;
    const uint8_t* src;
    size_t n;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_go_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      dst = dst_;
      src = src_;
      n = n_;
    }
    piece(dst, src, n, id, threads());
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) cv_done_.notify_one();
    }
  }
}

void CopyPool::copy(void* dst, const void* src, size_t n) {
  if (n == 0) return;
  if (workers_.empty() || n < (512u << 10)) {
    std::memcpy(dst, src, n);
    return;
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    dst_ = (uint8_t*)dst;
    src_ = (const uint8_t*)src;
    n_ = n;
    pending_ = (int)workers_.size();
    ++gen_;
  }
  cv_go_.notify_all();
  piece((uint8_t*)dst, (const uint8_t*)src, n, 0, threads());
  std::unique_lock<std::mutex> lk(mu_);
  cv_done_.wait(lk, [&] { return pending_ == 0; });
}

// --------------------------------------------------------------- Stager ----
Stager::Stager(size_t slot_bytes, int n_in, int n_out, int threads)
    : slot_bytes_(slot_bytes), in_(n_in), out_(n_out), pool_(threads) {
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
  pool_.copy(s.dst, s.host, s.len);
  s.dst = nullptr;
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
  for (;;) {
    const hipError_t e = hipEventQuery(sl.ev);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady)
      throw Error{SHELFI_ERR_DEVICE, std::string("staged copy: ") + hipGetErrorString(e)};
    if (!drain_front(false)) std::this_thread::yield();
  }
}

void Stager::h2d(void* dev, const void* host, size_t n, hipStream_t s) {
  const uint8_t* src = (const uint8_t*)host;
  uint8_t* dst = (uint8_t*)dev;
  while (n) {
    const size_t len = std::min(n, slot_bytes_);
    Slot& sl = in_[in_next_++ % in_.size()];
    wait_in_slot(sl);
    pool_.copy(sl.host, src, len);
    SHELFI_HIP(hipMemcpyAsync(dst, sl.host, len, hipMemcpyHostToDevice, s));
    SHELFI_HIP(hipEventRecord(sl.ev, s));
    sl.used = true;
    src += len;
    dst += len;
    n -= len;
  }
}

void Stager::d2h(void* host, const void* dev, size_t n, hipStream_t s) {
  uint8_t* dst = (uint8_t*)host;
  const uint8_t* src = (const uint8_t*)dev;
  while (n) {
    const size_t len = std::min(n, slot_bytes_);
    const size_t idx = out_next_++ % out_.size();
    Slot& sl = out_[idx];
    while (sl.dst) drain_front(true);  // FIFO: the oldest pending is drained first
    SHELFI_HIP(hipMemcpyAsync(sl.host, src, len, hipMemcpyDeviceToHost, s));
    SHELFI_HIP(hipEventRecord(sl.ev, s));
    sl.used = true;
    sl.dst = dst;
    sl.len = len;
    pending_.push_back(idx);
    dst += len;
    src += len;
    n -= len;
  }
}

void Stager::finish() {
  while (drain_front(true)) {
  }
  for (Slot& sl : in_)
    if (sl.used) SHELFI_HIP(hipEventSynchronize(sl.ev));
}

void Stager::abort() noexcept {
  for (auto* ring : {&in_, &out_})
    for (Slot& sl : *ring) {
      if (sl.used) (void)hipEventSynchronize(sl.ev);
      sl.dst = nullptr;
    }
  pending_.clear();
}

}  // namespace shelfi

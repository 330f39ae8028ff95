// Host <-> HBM staging for the bytes API.
//
// The bytes API hands over pageable Python buffers.  A hipMemcpyAsync from pageable memory
// returns only once the runtime has moved the data (the calling thread waits), and a freshly
// allocated output (a new bytes object) first-touch faults on the copy thread at ~16 GB/s.
// The Stager owns rings of pinned slots: pageable data is memcpy'd into a slot by a pool of
// threads (faults spread over the cores) and the slot is DMA'd asynchronously; outputs are
// DMA'd into pinned slots and drained into the destination by the same pool while later DMAs
// run.  Round 5: for large contiguous uploads the runtime's own pageable path is faster (55.6
// GB/s in 32 MiB copies vs ~44 through the ring, tools/h2d_pageable_probe.py), so the
// aggregation uploads directly and drains its outputs on an AsyncDrain worker instead, which
// keeps the uploading thread free.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace shelfi {

// memcpy, with non-temporal stores when `nt` and the CPU has AVX-512 (n >= 64 KiB).
void copy_bytes(uint8_t* d, const uint8_t* s, size_t n, bool nt);

// One memcpy of a scatter/gather list.
struct CopyJob {
  uint8_t* dst;
  const uint8_t* src;
  size_t n;
};

// Persistent workers splitting one copy list at a time (the caller takes a share
// too): the list is treated as one byte stream cut into page-aligned shares.
class CopyPool {
 public:
  explicit CopyPool(int threads);
  ~CopyPool();
  CopyPool(const CopyPool&) = delete;
  CopyPool& operator=(const CopyPool&) = delete;
  void copy(void* dst, const void* src, size_t n);
  // parts = how many of the pool's threads share the list (0 = all of them).
  void copy_many(const CopyJob* jobs, size_t njobs, int parts = 0);
  int threads() const { return parts_; }

 private:
  void run(int id);
  void share(int id);
  int parts_ = 1;  // set before the workers start
  std::vector<std::thread> workers_;
  // A new list is published by bumping gen_ (release); workers spin on it for a while
  // after each share (the staging loop issues lists back to back), then sleep on cv_.
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<uint64_t> gen_{0};
  std::atomic<int> pending_{0};
  std::atomic<bool> stop_{false};
  const CopyJob* jobs_ = nullptr;
  size_t njobs_ = 0, total_ = 0;
  int active_ = 1;  // threads sharing the current list
  bool nt_ = true;  // streaming stores (SHELFI_NT_COPY=0: plain memcpy)
};

// A host range of a scatter/gather transfer.
struct HostPiece {
  uint8_t* p;
  size_t n;
};

class Stager {
 public:
  // slot_bytes: DMA granule; n_in / n_out: pinned slots per direction.
  Stager(size_t slot_bytes, int n_in, int n_out, int threads);
  ~Stager();
  Stager(const Stager&) = delete;
  Stager& operator=(const Stager&) = delete;

  // Enqueue host -> device of n bytes on `s`.  Returns once the data has been copied
  // into pinned slots (the source may then be reused); the DMAs run asynchronously.
  void h2d(void* dev, const void* host, size_t n, hipStream_t s);
  // Enqueue device -> host of n bytes on `s`.  `host` is written later, by poll() /
  // finish() (or when its slot is needed again); it must stay valid until finish().
  void d2h(void* host, const void* dev, size_t n, hipStream_t s);
  // Gather: the pieces, in order, land contiguously at `dev`.
  void h2dv(void* dev, const HostPiece* pieces, size_t np, hipStream_t s);
  // Scatter: contiguous device bytes at `dev` go to the pieces, in order (written
  // later, like d2h).
  void d2hv(const HostPiece* pieces, size_t np, const void* dev, hipStream_t s);
  // A call's first uploads ramp up: the first input slots are filled to a quarter and a half of a slot, so
  // the copy engine starts after a 4 MiB fill instead of a 16 MiB one (the fill runs ~2x the DMA rate, so
  // each slot is ready before the previous DMA ends).
  void begin() { ramp_ = 0; }
  // Drain every output slot whose DMA has completed (non-blocking).
  void poll();
  // Drain all outputs and wait for all inputs.  Must be called before the host
  // buffers are touched or released; rethrows the first error.
  void finish();
  // Abandon in-flight work after an error: wait for the DMAs, drop pending outputs.
  void abort() noexcept;

  size_t slot_bytes() const { return slot_bytes_; }
  int threads() const { return pool_.threads(); }
  bool trace() const { return trace_; }  // SHELFI_STAGE_TRACE=1

 private:
  struct Slot {
    uint8_t* host = nullptr;
    hipEvent_t ev = nullptr;
    bool used = false;             // an event has been recorded
    bool pending = false;          // output waiting to be drained (d2h slots)
    std::vector<CopyJob> out_jobs;  // where a pending output goes
  };
  bool drain_front(bool block);
  void wait_in_slot(Slot& sl);

  size_t slot_bytes_;
  std::vector<Slot> in_, out_;
  size_t in_next_ = 0, out_next_ = 0;
  std::deque<size_t> pending_;  // out slot indices in enqueue order
  CopyPool pool_;
  // SHELFI_STAGE_TRACE=1: seconds the calling thread spent filling input slots, waiting
  // for an input slot's DMA, and draining outputs (printed to stderr by finish())
  bool trace_ = false;
  double t_fill_ = 0, t_wait_ = 0, t_drain_ = 0;
  size_t b_in_ = 0;
  // Threads that fill an upload slot: fewer than the pool (pageable -> pinned copies
  // compete with the DMA engine reading pinned memory; 4 of 8 measured +8-16% H2D,
  // DESIGN.md §5.3).  Drains into fresh output pages keep the whole pool (page faults).
  int h2d_parts_ = 1;
  int ramp_ = 2;  // begin(): 0, then the first slots hold slot_bytes_ >> (2 - ramp_)
};

// Ask for transparent huge pages on the 2 MiB-aligned interior of a large output
// buffer that has not been touched yet (a new bytes object: 512x fewer first-touch
// faults and a cheaper munmap later).  numpy does the same for its large arrays.
void advise_huge(void* p, size_t n);

// Worker threads for a Stager: SHELFI_COPY_THREADS, else min(8, CPUs this process may use).
int default_copy_threads();
int default_h2d_copy_threads();  // SHELFI_H2D_COPY_THREADS, default 4

// Background scatter of device -> host chunks (round 5, the direct-upload aggregation): the caller
// DMAs a chunk into one of two pinned buffers (buffer(slot)), records an event after it and posts
// the pieces the chunk goes to; a worker thread waits for the event and copies the buffer into the
// pieces with its own CopyPool while the caller goes on uploading.  wait_slot() before a buffer is
// reused; finish() waits for every posted job and rethrows the worker's first error.
class AsyncDrain {
 public:
  explicit AsyncDrain(int threads);
  ~AsyncDrain();
  AsyncDrain(const AsyncDrain&) = delete;
  AsyncDrain& operator=(const AsyncDrain&) = delete;
  uint8_t* buffer(int slot, size_t bytes);  // pinned; grown (the slot must be idle)
  void wait_slot(int slot);
  void post(int slot, hipEvent_t ev, std::vector<HostPiece> pieces);
  // First-touch the pages of [p, p + n) on the worker (ahead of the drains into a fresh output, which
  // would otherwise take the page faults in the call's tail)
  void prefault(uint8_t* p, size_t n);
  void finish();

 private:
  void run();
  struct Job {
    int slot;  // -1: prefault the pieces
    hipEvent_t ev;
    std::vector<HostPiece> pieces;
  };
  int prefaults_ = 0;  // posted, not yet done
  CopyPool pool_;
  std::thread worker_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job> q_;
  bool stop_ = false;
  int busy_[2] = {0, 0};  // posted, not yet drained, per slot
  uint8_t* buf_[2] = {nullptr, nullptr};
  size_t cap_[2] = {0, 0};
  std::string err_;
};

// A second uploading thread (round 5): the pageable hipMemcpyAsync returns only once the runtime has moved
// the data, so two threads with a stream each keep two copies in flight -- one copy's setup overlaps the
// other's transfer.  post() queues a copy on `stream`; wait() returns when every posted copy has been
// issued and rethrows the first error.
class AsyncUpload {
 public:
  AsyncUpload();
  ~AsyncUpload();
  AsyncUpload(const AsyncUpload&) = delete;
  AsyncUpload& operator=(const AsyncUpload&) = delete;
  void post(void* dst, const void* src, size_t n, hipStream_t stream);
  void wait();

 private:
  void run();
  struct Job {
    void* dst;
    const void* src;
    size_t n;
    hipStream_t stream;
  };
  std::thread worker_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job> q_;
  int pending_ = 0;
  bool stop_ = false;
  std::string err_;
};

}  // namespace shelfi

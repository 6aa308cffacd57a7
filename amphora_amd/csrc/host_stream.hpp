// Host-memory streaming support for the host-pointer entry points:
// page-locked staging buffers and a small memcpy thread pool.
//
// Caller buffers (e.g. Java heap arrays pinned by JNI, numpy arrays) are
// normally pageable.  hipMemcpyAsync from pageable memory is staged by the
// runtime and does not overlap with kernels, so each batch is instead copied
// by CPU threads into a page-locked slot, DMA'd with hipMemcpyAsync (truly
// async), and the outputs come back the same way.  Buffers the caller has
// page-locked (amph_host_register / hipHostMalloc) skip the staging copy.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/amphora.h"

namespace amph {

struct PinnedBuf {
  void* p = nullptr;
  size_t cap = 0;
  // hipHostMallocDefault for DMA staging (only the copy engines touch it);
  // hipHostMallocCoherent for memory kernels read and write in place
  // (run_small's arena): fine-grained, so a kernel never sees a line its
  // device cached from an earlier call at the same address.
  unsigned flags = hipHostMallocDefault;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    release();
    hipError_t e = hipHostMalloc(&p, bytes, flags);
    if (e == hipSuccess) cap = bytes;
    else p = nullptr;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// One staging copy: memcpy(dst, src, bytes), or -- for an AMPH_F_HOST_IO
// array -- its read (io_write false: array[io_off ..] -> dst) or write
// (io_write true: src -> array[io_off ..]) callback.
struct CopyTask {
  void* dst;
  const void* src;
  size_t bytes;
  const amph_host_array* io = nullptr;
  size_t io_off = 0;
  bool io_write = false;
};

inline int run_copy(const CopyTask& c) {
  if (!c.io) {
    std::memcpy(c.dst, c.src, c.bytes);
    return 0;
  }
  return c.io_write ? c.io->write(c.io, c.io_off, c.bytes, c.src) : c.io->read(c.io, c.io_off, c.bytes, c.dst);
}

// Persistent pool: copy(tasks) splits every task into chunks of >= 4 MiB and
// runs them on the workers and the calling thread; returns when all are done,
// with 0 or the first nonzero callback status (the other chunks still run).
class CopyPool {
 public:
  explicit CopyPool(int threads) {
    for (int i = 0; i < threads; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  int threads() const { return (int)workers_.size() + 1; }

  int copy(const std::vector<CopyTask>& tasks) {
    std::vector<CopyTask> chunks;
    const size_t kChunk = (size_t)4 << 20;
    for (const auto& t : tasks)
      for (size_t off = 0; off < t.bytes; off += kChunk) {
        CopyTask c = t;
        c.dst = (char*)t.dst + off;
        c.src = (const char*)t.src + off;
        c.bytes = std::min(kChunk, t.bytes - off);
        c.io_off = t.io_off + off;
        chunks.push_back(c);
      }
    if (chunks.empty()) return 0;
    std::unique_lock<std::mutex> lk(m_);
    jobs_ = &chunks;
    next_ = 0;
    remaining_ = chunks.size();
    status_ = 0;
    ++gen_;
    lk.unlock();
    cv_.notify_all();
    drain();
    lk.lock();
    done_cv_.wait(lk, [&] { return remaining_ == 0; });
    jobs_ = nullptr;
    return status_;
  }

 private:
  void drain() {
    for (;;) {
      CopyTask c;
      {
        std::lock_guard<std::mutex> g(m_);
        if (!jobs_ || next_ >= jobs_->size()) return;
        c = (*jobs_)[next_++];
      }
      const int st = run_copy(c);
      std::lock_guard<std::mutex> g(m_);
      if (st && !status_) status_ = st;
      if (--remaining_ == 0) done_cv_.notify_all();
    }
  }
  void loop() {
    size_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      drain();
    }
  }
  std::vector<std::thread> workers_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  std::vector<CopyTask>* jobs_ = nullptr;
  size_t next_ = 0;
  size_t remaining_ = 0;
  size_t gen_ = 0;
  int status_ = 0;
  bool stop_ = false;
};

// One long-lived thread that owns a device for a multi-device context's
// sub-context: run_sharded posts each call's shard to it instead of starting
// a fresh std::thread per call (a fresh thread's first HIP call pays the
// runtime's per-thread device setup, ~76 us of hipSetDevice in
// profiles/r03_c1_rocprof_before_pool.txt, on every call).  Tasks run in
// post order; the destructor drains the queue and joins.
class DeviceWorker {
 public:
  DeviceWorker() : th_([this] { loop(); }) {}
  ~DeviceWorker() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  DeviceWorker(const DeviceWorker&) = delete;
  DeviceWorker& operator=(const DeviceWorker&) = delete;
  void post(std::function<void()> fn) {
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push_back(std::move(fn));
    }
    cv_.notify_one();
  }

 private:
  void loop() {
    for (;;) {
      std::function<void()> fn;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        fn = std::move(q_.front());
        q_.pop_front();
      }
      fn();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false;
  std::thread th_;  // last: starts once the members above exist
};

// Completion count for a fan-out over DeviceWorkers.
class Latch {
 public:
  explicit Latch(size_t n) : n_(n) {}
  void count_down() {
    std::lock_guard<std::mutex> g(m_);
    if (--n_ == 0) cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(m_);
    cv_.wait(lk, [&] { return n_ == 0; });
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  size_t n_;
};

inline bool is_pinned_host(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: clear the sticky error
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

}  // namespace amph

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
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace amph {

struct PinnedBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    release();
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
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

struct CopyTask {
  void* dst;
  const void* src;
  size_t bytes;
};

// Persistent pool: copy(tasks) splits every task into chunks of >= 4 MiB and
// runs them on the workers and the calling thread; returns when all are done.
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

  void copy(const std::vector<CopyTask>& tasks) {
    std::vector<CopyTask> chunks;
    const size_t kChunk = (size_t)4 << 20;
    for (const auto& t : tasks)
      for (size_t off = 0; off < t.bytes; off += kChunk)
        chunks.push_back({(char*)t.dst + off, (const char*)t.src + off, std::min(kChunk, t.bytes - off)});
    if (chunks.empty()) return;
    std::unique_lock<std::mutex> lk(m_);
    jobs_ = &chunks;
    next_ = 0;
    remaining_ = chunks.size();
    ++gen_;
    lk.unlock();
    cv_.notify_all();
    drain();
    lk.lock();
    done_cv_.wait(lk, [&] { return remaining_ == 0; });
    jobs_ = nullptr;
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
      std::memcpy(c.dst, c.src, c.bytes);
      std::lock_guard<std::mutex> g(m_);
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
  bool stop_ = false;
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

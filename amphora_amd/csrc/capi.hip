// C ABI of libamphora_hip (declared in include/amphora.h).
//
// Host-pointer calls stream the word arrays through the device in batches
// (ctx->batch_words, default 4 Mi words): per batch the inputs go HtoD on the
// copy-in stream, the kernel runs on the kernel stream, the outputs come back
// DtoH on the copy-out stream; three device-side slots let batch k+1's copies
// overlap batch k's kernel and batch k-1's copy out (run_batched).  Verify
// failures are reported per batch into a device array of first-fail words,
// read back once at the end.  Device-pointer calls (AMPH_F_DEVICE) launch
// straight onto the caller's stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <initializer_list>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <atomic>
#include <memory>
#include <thread>

#include "../../include/amphora.h"
#include "host_stream.hpp"
#include "kernels.hpp"

using amph::Fp;
using amph::W4;

namespace {

thread_local std::string g_last_error;
thread_local hipEvent_t g_ev_start = nullptr, g_ev_stop = nullptr;  // amph_time_next_launch

int fail(int status, const std::string& msg) {
  g_last_error = msg;
  return status;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(AMPH_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr)                                   \
  do {                                                  \
    hipError_t e_ = (expr);                             \
    if (e_ != hipSuccess) return hip_fail(e_, #expr);   \
  } while (0)

// The context's device for this thread's next HIP calls: hipSetDevice only
// when the thread's current device differs (hipGetDevice reads thread-local
// state; the set is what a thread's first HIP call pays for).
hipError_t use_device(int device) {
  int cur = -1;
  if (hipGetDevice(&cur) == hipSuccess && cur == device) return hipSuccess;
  return hipSetDevice(device);
}

typedef unsigned __int128 u128;

u128 ld128(const uint8_t* b) {
  uint64_t lo, hi;
  std::memcpy(&lo, b, 8);
  std::memcpy(&hi, b + 8, 8);
  return ((u128)hi << 64) | lo;
}

W4 w4_of(u128 x) {
  return W4{{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)(x >> 64), (uint32_t)(x >> 96)}};
}

u128 u128_of(const W4& w) {
  return ((u128)w.v[3] << 96) | ((u128)w.v[2] << 64) | ((u128)w.v[1] << 32) | w.v[0];
}

std::string dec(u128 x) {
  if (x == 0) return "0";
  char buf[48];
  int n = 0;
  while (x) {
    buf[n++] = (char)('0' + (int)(x % 10));
    x /= 10;
  }
  std::string s(buf, n);
  std::reverse(s.begin(), s.end());
  return s;
}

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) cap = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

}  // namespace

struct amph_ctx {
  int device = 0;
  Fp f{};
  u128 p = 0, r = 0, rinv = 0;
  std::mutex mu;
  size_t batch_words = (size_t)4 << 20;
  int grid_cap = 0;
  int block = 0;  // 0 = by size (block_for)
  // host-pointer path: kSlots batches in flight, one stream each
  static constexpr int kSlots = 3;
  struct Slot {
    DevBuf dev;
    amph::PinnedBuf hin, hout;
    hipEvent_t in_done = nullptr, k_done = nullptr, out_done = nullptr;
    bool busy = false;  // hout holds outputs not yet copied to the caller
    bool used = false;  // the slot has a batch in this call (its events are live)
    size_t base = 0, cnt = 0;
  };
  hipStream_t streams[kSlots] = {};  // host path: HtoD, kernels, DtoH
  Slot slots[kSlots];
  std::vector<amph_ctx*> sub;  // amph_ctx_create_multi: one context per device
  // a sub-context's own long-lived thread (run_sharded posts its shards here)
  std::unique_ptr<amph::DeviceWorker> worker;
  DevBuf ff;  // per-batch first-fail words (host path)
  DevBuf tail;  // small scratch for the partial last unit of codec calls
  DevBuf wire;  // host-mode staging of the wire-text calls (texts, secrets, outputs, verdicts)
  DevBuf xstage;  // host-mode staging of the exchange codec calls
  DevBuf xdev;    // device-mode scan scratch of the exchange codec calls
  hipEvent_t xdev_done = nullptr;  // the last device-mode exchange call's kernels
  // small host calls (run_small): one page-locked arena the kernels read and
  // write in place, and device verdict words kept at kNoFail between calls
  size_t small_bytes = (size_t)2 << 20;
  amph::PinnedBuf small;
  DevBuf small_ff;
  bool small_ff_dirty = true;
  std::unique_ptr<amph::CopyPool> pool;
  // party sessions' device buffers, kept after amph_party_free for the next
  // session: a server runs one session per request, and hipMalloc / hipFree of
  // its gigabytes cost tens of microseconds per buffer (hipFree synchronises
  // the device) -- best fit, at most kPartyPoolMax buffers, freed with the context
  std::vector<DevBuf> party_pool;
  size_t pool_cap_bytes = (size_t)32 << 30;  // AMPH_PARTY_POOL_BYTES
  std::atomic<uint64_t> launches{0};      // amph_ctx_stats
  std::atomic<uint64_t> worker_tasks{0};
};

namespace {

// ---- device memory ------------------------------------------------------------
// (c->mu held) the party-session buffers pooled for reuse are the only device
// memory a context keeps that nothing is using: every allocation of the
// context that runs out of memory frees them and tries once more, so the
// pool never causes the out-of-memory error it would then report.
size_t pool_bytes(const amph_ctx* c) {
  size_t t = 0;
  for (const DevBuf& b : c->party_pool) t += b.cap;
  return t;
}

void pool_reclaim(amph_ctx* c) {
  for (DevBuf& b : c->party_pool) b.release();
  c->party_pool.clear();
}

hipError_t dev_ensure(amph_ctx* c, DevBuf& b, size_t bytes) {
  hipError_t e = b.ensure(bytes);
  if (e == hipErrorOutOfMemory && !c->party_pool.empty()) {
    (void)hipGetLastError();
    pool_reclaim(c);
    e = b.ensure(bytes);
  }
  return e;
}

// ---- field setup (host) -----------------------------------------------------
u128 add_mod(u128 a, u128 b, u128 p) {  // a, b < p
  u128 s = a + b;
  if (s < a || s >= p) s -= p;
  return s;
}

int setup_field(amph_ctx* c, const uint8_t* p_le, const uint8_t* r_le, const uint8_t* rinv_le) {
  const u128 p = ld128(p_le), r = ld128(r_le), rinv = ld128(rinv_le);
  if (p < 3 || (p & 1) == 0) return fail(AMPH_E_PARAM, "prime must be odd and > 2");
  const u128 R = ((u128)0 - p) % p;  // 2^128 mod p
  if (r != R) return fail(AMPH_E_PARAM, "r must equal 2^128 mod prime (MP-SPDZ auxiliary modulus)");
  Fp f{};
  const W4 pw = w4_of(p);
  for (int i = 0; i < 4; ++i) f.p[i] = pw.v[i];
  uint32_t inv = f.p[0];  // Newton: inv = p^-1 mod 2^32
  for (int i = 0; i < 5; ++i) inv *= 2u - f.p[0] * inv;
  f.n0 = (uint32_t)(0u - inv);
  u128 x = R;  // R^2 mod p = R * 2^128 mod p by 128 doublings
  for (int i = 0; i < 128; ++i) x = add_mod(x, x, p);
  const W4 r2 = w4_of(x);
  for (int i = 0; i < 4; ++i) f.r2[i] = r2.v[i];
  f.big = (p >> 127) != 0;
  if (rinv >= p) return fail(AMPH_E_PARAM, "rInv must be reduced mod prime");
  // r * rInv == 1 (mod p): mont_mul(mont_mul(r, rInv), R^2) = r rInv
  const W4 t = amph::mont_mul(amph::mont_mul(w4_of(r), w4_of(rinv), f), r2, f);
  if (u128_of(t) != 1) return fail(AMPH_E_PARAM, "rInv must be the inverse of r mod prime");
  c->f = f;
  c->p = p;
  c->r = r;
  c->rinv = rinv;
  return AMPH_OK;
}

u128 mulmod_host(const amph_ctx* c, u128 a, u128 b) {  // a < p
  return u128_of(amph::mont_mul(amph::mont_mul(w4_of(a), w4_of(b), c->f), amph::r2_word(c->f), c->f));
}

// Workgroup size: 1024 threads (16 waves).  Measured through bench.py on
// MI355X (gpurun_out r01c sweep): 1024 beat 128/256/512 by 2-5 % at both
// 1 Mi words x 2 parties and 16 Mi words x 3 parties.  AMPH_BLOCK overrides.
int block_for(const amph_ctx* c, size_t words) {
  (void)words;
  return c->block > 0 ? c->block : 1024;
}

amph::LaunchCfg cfg(amph_ctx* c, hipStream_t s, size_t words) {
  c->launches.fetch_add(1, std::memory_order_relaxed);
  amph::LaunchCfg lc{s, c->grid_cap, block_for(c, words)};
  lc.ev_start = g_ev_start;  // consumed by this launch only
  lc.ev_stop = g_ev_stop;
  g_ev_start = g_ev_stop = nullptr;
  return lc;
}

// ---- host batching ------------------------------------------------------------
// A batched host call is described by its input and output arrays, each with
// a per-word byte size; the kernel launcher receives device pointers of one
// batch.
struct HostIn {
  const uint8_t* host;
  size_t bytes_per_word;
  size_t base = 0;                        // words into the array where this call starts
  const amph_host_array* io = nullptr;    // AMPH_F_HOST_IO: the callbacks (host unused)
};
struct HostOut {
  uint8_t* host;
  size_t bytes_per_word;
  size_t base = 0;
  const amph_host_array* io = nullptr;
};

// AMPH_F_HOST_IO for the calling thread's current ABI call: set by the entry
// point (HostIoScope), turned into HostIn/HostOut::io by run_batched before
// any work leaves this thread.
thread_local bool g_host_io = false;
struct HostIoScope {
  explicit HostIoScope(uint32_t flags) { g_host_io = (flags & AMPH_F_HOST_IO) != 0; }
  ~HostIoScope() { g_host_io = false; }
};

// the staging copy of `words` words from word `word` of input x into dst
amph::CopyTask copy_in(const HostIn& x, size_t word, size_t words, void* dst) {
  const size_t off = (x.base + word) * x.bytes_per_word, bytes = words * x.bytes_per_word;
  if (x.io) return amph::CopyTask{dst, nullptr, bytes, x.io, off, false};
  return amph::CopyTask{dst, x.host + off, bytes};
}
amph::CopyTask copy_out(const HostOut& x, size_t word, size_t words, const void* src) {
  const size_t off = (x.base + word) * x.bytes_per_word, bytes = words * x.bytes_per_word;
  if (x.io) return amph::CopyTask{nullptr, src, bytes, x.io, off, true};
  return amph::CopyTask{x.host + off, src, bytes};
}
int io_failed() { return fail(AMPH_E_PARAM, "a host array callback (AMPH_F_HOST_IO) failed"); }

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// kPageableRule -- the ordering rule every host<->device copy here follows:
//
//   hipMemcpyAsync is used ONLY with page-locked host memory (the batched
//   pipeline's slot buffers, or caller buffers is_pinned_host() reports as
//   registered).  Pageable host memory moves with a blocking hipMemcpy,
//   issued only once the context stream that produces / consumes the device
//   side has been synchronised.
//
// Why: HIP defines an async copy of pageable memory only as "performed
// synchronously" (hip_runtime_api.h, hipMemcpyAsync @note) -- a host-staged
// transfer, not the stream-ordered copy CUDA code assumes -- so its order
// against the kernels of a non-blocking stream is not a guarantee this
// library may build on.  Round 2 saw that order fail once in each direction,
// both times in a one-shot call on a non-blocking context stream:
//   * DtoH (1e4fc5f): a pageable verdict word on the stack, hipMemcpyAsync'd
//     after the kernel that writes it, held the value from before the kernel;
//   * HtoD (9513c3e): base64 text hipMemcpyAsync'd from pageable memory into
//     hipMallocAsync staging on the same stream was seen by the kernel with
//     its first 16-character unit (the head of the first copy) unwritten.
// tests/test_host_ordering.py checks the rule statically over this file and
// runs a fresh process's first wire-text calls on the GPU.
//
// Results of a one-shot host call: wait for the stream, then copy with
// blocking hipMemcpy.
struct ReadBack {
  void* dst;
  const void* src;
  size_t bytes;
};
hipError_t read_back(hipStream_t s, std::initializer_list<ReadBack> copies) {
  hipError_t e = hipStreamSynchronize(s);
  for (const ReadBack& r : copies)
    if (e == hipSuccess && r.bytes) e = hipMemcpy(r.dst, r.src, r.bytes, hipMemcpyDeviceToHost);
  return e;
}

int host_threads() {
  if (const char* t = std::getenv("AMPH_HOST_THREADS")) return std::max(1, std::atoi(t));
  const unsigned hw = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(8u, hw ? hw / 2 : 1u));
}

template <class Launch>
int run_sharded(amph_ctx* g, size_t words, const std::vector<HostIn>& ins,
                const std::vector<HostOut>& outs, bool with_ff, int64_t* first_fail,
                Launch& launch, size_t ff_scale);

// Batch size of a host call: at most ctx->batch_words, and small enough that
// the call has about 8 batches -- so copies in, kernels and copies out of
// consecutive batches overlap -- but not below 32 MiB of traffic per batch
// (each batch costs a few events and copy launches).  A 4 Mi-word call at 3
// parties used to be ONE batch, every stage back to back: pageable odo_pre
// 43.6 -> 25.7 ms, open_post 48.0 -> 32.8, mask_input 30.8 -> 22.5 with
// 512 Ki-word batches (tools/host_rate_probe.py, profiles/r03_host_batches.jsonl);
// C5's 32 Mi-word calls keep their 4 Mi-word batches.
size_t batch_for(const amph_ctx* c, size_t words, size_t bytes_per_word) {
  constexpr size_t kMinBatchBytes = (size_t)32 << 20;
  const size_t floor_words = std::max<size_t>(1, kMinBatchBytes / std::max<size_t>(1, bytes_per_word));
  const size_t eighth = (words + 7) / 8;
  return std::max<size_t>(1, std::min({words, c->batch_words, std::max(eighth, floor_words)}));
}

// Streams `words` through the device in batches of ctx->batch_words, one
// HIP stream per engine: streams[0] carries every HtoD copy in batch order,
// streams[1] the kernels, streams[2] every DtoH copy.  kSlots device slots
// (inputs + outputs of one batch each) rotate; events order the slot reuse
// on the GPU (batch b's HtoD waits for the kernel of batch b - kSlots, its
// kernel for its HtoD and for the DtoH of batch b - kSlots, its DtoH for its
// kernel), so the copy-in engine streams batch after batch at the link's
// rate while kernels and copies out overlap it (with one stream per slot the
// slots' copies shared the link, finished together, and the link idled while
// their kernels and copies out drained: 2-4 ms every third batch in the
// rocprofv3 memory-copy trace of a C5 step).  The CPU only
// waits to reuse a page-locked staging slot: pageable inputs are copied into
// one by CPU threads once its previous HtoD is done, pageable outputs out of
// one once its previous DtoH is done.  Page-locked caller buffers are DMA'd
// directly.  Verify failures land in one device word per batch; the smallest
// global index is reported.  A kernel reports its failure index in units of
// 1/ff_scale of a batch word (the base64 stream decode: a character offset,
// 16 characters per batch word), so batch b's base is b * bw * ff_scale.
template <class Launch>
int run_batched_impl(amph_ctx* c, size_t words, const std::vector<HostIn>& ins,
                     const std::vector<HostOut>& outs, bool with_ff, int64_t* first_fail,
                     Launch& launch, size_t ff_scale) {
  if (first_fail) *first_fail = -1;
  if (words == 0) return AMPH_OK;
  constexpr int S = amph_ctx::kSlots;
  static_assert(S >= 3, "one stream per engine");
  HIP_TRY(use_device(c->device));
  for (int s = 0; s < S; ++s) {
    if (!c->streams[s]) HIP_TRY(hipStreamCreateWithFlags(&c->streams[s], hipStreamNonBlocking));
    amph_ctx::Slot& sl = c->slots[s];
    for (hipEvent_t* e : {&sl.in_done, &sl.k_done, &sl.out_done})
      if (!*e) HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
    sl.busy = false;
    sl.used = false;
  }
  hipStream_t s_in = c->streams[0], s_k = c->streams[1], s_out = c->streams[2];
  if (!c->pool) c->pool.reset(new amph::CopyPool(host_threads() - 1));
  size_t bpw = 0;
  for (const HostIn& x : ins) bpw += x.bytes_per_word;
  for (const HostOut& x : outs) bpw += x.bytes_per_word;
  const size_t bw = batch_for(c, words, bpw);
  const size_t nb = (words + bw - 1) / bw;
  std::vector<char> in_pinned(ins.size()), out_pinned(outs.size());
  size_t dev_bytes = 0, hin_bytes = 0, hout_bytes = 0;
  for (size_t k = 0; k < ins.size(); ++k) {
    in_pinned[k] = !ins[k].io && amph::is_pinned_host(ins[k].host);
    dev_bytes += align256(bw * ins[k].bytes_per_word);
    if (!in_pinned[k]) hin_bytes += align256(bw * ins[k].bytes_per_word);
  }
  for (size_t k = 0; k < outs.size(); ++k) {
    out_pinned[k] = !outs[k].io && amph::is_pinned_host(outs[k].host);
    dev_bytes += align256(bw * outs[k].bytes_per_word);
    if (!out_pinned[k]) hout_bytes += align256(bw * outs[k].bytes_per_word);
  }
  for (int s = 0; s < S && (size_t)s < nb; ++s) {
    hipError_t e = dev_ensure(c, c->slots[s].dev, dev_bytes);
    if (e == hipSuccess) e = c->slots[s].hin.ensure(hin_bytes);
    if (e == hipSuccess) e = c->slots[s].hout.ensure(hout_bytes);
    if (e != hipSuccess) return fail(AMPH_E_NOMEM, std::string("batch buffers: ") + hipGetErrorString(e));
  }
  if (with_ff) {
    hipError_t e = dev_ensure(c, c->ff, nb * sizeof(unsigned long long));
    if (e != hipSuccess) return fail(AMPH_E_NOMEM, "first-fail words");
    HIP_TRY(hipMemsetAsync(c->ff.p, 0x7F, nb * sizeof(unsigned long long), s_k));
  }
  // copy a finished batch's pageable outputs from the slot's staging buffer
  auto drain_out = [&](amph_ctx::Slot& sl) -> int {
    if (!sl.busy) return AMPH_OK;
    HIP_TRY(hipEventSynchronize(sl.out_done));
    std::vector<amph::CopyTask> tasks;
    size_t off = 0;
    for (size_t k = 0; k < outs.size(); ++k) {
      if (out_pinned[k]) continue;
      tasks.push_back(copy_out(outs[k], sl.base, sl.cnt, (char*)sl.hout.p + off));
      off += align256(bw * outs[k].bytes_per_word);
    }
    const int cst = c->pool->copy(tasks);
    sl.busy = false;
    return cst ? io_failed() : AMPH_OK;
  };
  for (size_t b = 0; b < nb; ++b) {
    amph_ctx::Slot& sl = c->slots[b % S];
    const size_t base = b * bw, cnt = std::min(bw, words - base);
    // stage pageable inputs into the slot's page-locked buffer once the slot's
    // previous HtoD has read it
    std::vector<amph::CopyTask> tasks;
    std::vector<const void*> src(ins.size());
    size_t hoff = 0;
    for (size_t k = 0; k < ins.size(); ++k) {
      if (in_pinned[k]) {
        src[k] = ins[k].host + (ins[k].base + base) * ins[k].bytes_per_word;
      } else {
        void* d = (char*)sl.hin.p + hoff;
        tasks.push_back(copy_in(ins[k], base, cnt, d));
        src[k] = d;
        hoff += align256(bw * ins[k].bytes_per_word);
      }
    }
    if (!tasks.empty()) {
      if (sl.used) HIP_TRY(hipEventSynchronize(sl.in_done));
      if (c->pool->copy(tasks)) return io_failed();
    }
    uint8_t* cur = (uint8_t*)sl.dev.p;
    std::vector<const uint4*> din;
    std::vector<uint4*> dout;
    if (sl.used) HIP_TRY(hipStreamWaitEvent(s_in, sl.k_done, 0));  // inputs consumed
    for (size_t k = 0; k < ins.size(); ++k) {
      HIP_TRY(hipMemcpyAsync(cur, src[k], cnt * ins[k].bytes_per_word, hipMemcpyHostToDevice, s_in));
      din.push_back((const uint4*)cur);
      cur += align256(bw * ins[k].bytes_per_word);
    }
    HIP_TRY(hipEventRecord(sl.in_done, s_in));
    for (size_t k = 0; k < outs.size(); ++k) {
      dout.push_back((uint4*)cur);
      cur += align256(bw * outs[k].bytes_per_word);
    }
    HIP_TRY(hipStreamWaitEvent(s_k, sl.in_done, 0));
    if (sl.used) HIP_TRY(hipStreamWaitEvent(s_k, sl.out_done, 0));  // outputs copied out
    unsigned long long* ff = with_ff ? (unsigned long long*)c->ff.p + b : nullptr;
    hipError_t e = launch(din, dout, cnt, ff, cfg(c, s_k, cnt));
    if (e != hipSuccess) return hip_fail(e, "kernel launch");
    HIP_TRY(hipEventRecord(sl.k_done, s_k));
    // the slot's staging buffer still holds the previous batch's outputs
    if (int rc = drain_out(sl)) return rc;
    HIP_TRY(hipStreamWaitEvent(s_out, sl.k_done, 0));
    size_t ooff = 0;
    for (size_t k = 0; k < outs.size(); ++k) {
      void* dst = outs[k].host + (outs[k].base + base) * outs[k].bytes_per_word;
      if (!out_pinned[k]) {
        dst = (char*)sl.hout.p + ooff;
        ooff += align256(bw * outs[k].bytes_per_word);
      }
      HIP_TRY(hipMemcpyAsync(dst, dout[k], cnt * outs[k].bytes_per_word, hipMemcpyDeviceToHost, s_out));
    }
    HIP_TRY(hipEventRecord(sl.out_done, s_out));
    sl.busy = hout_bytes > 0;  // page-locked outputs need no copy-out (s_out is synced below)
    sl.used = true;
    sl.base = base;
    sl.cnt = cnt;
  }
  for (size_t b = nb > (size_t)S ? nb - S : 0; b < nb; ++b)
    if (int rc = drain_out(c->slots[b % S])) return rc;
  HIP_TRY(hipStreamSynchronize(s_out));  // page-locked outputs (no staging slot) landed too
  // a call with no outputs (amph_verify, the verify-only tail of
  // amph_mask_input) has nothing on s_out that waits for its kernels: wait
  // for them before the verdicts are read (the blocking copy below runs on
  // the null stream, which does not order with non-blocking streams)
  HIP_TRY(hipStreamSynchronize(s_k));
  if (with_ff) {
    std::vector<unsigned long long> h(nb);
    HIP_TRY(hipMemcpy(h.data(), c->ff.p, nb * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    for (size_t b = 0; b < nb; ++b) {
      if (h[b] != amph::kNoFail) {
        if (first_fail) *first_fail = (int64_t)(b * bw * ff_scale + h[b]);
        return AMPH_E_VERIFY;
      }
    }
  }
  return AMPH_OK;
}

// ---- small host calls ------------------------------------------------------------
// A host call whose inputs and outputs together fit c->small_bytes (default
// 2 MiB; AMPH_SMALL_BYTES, 0 = off) skips the batched pipeline: the inputs
// are memcpy'd into the context's page-locked arena, the kernel reads them
// and writes its outputs there in place (hipHostMalloc memory is mapped into
// the device's address space), its verdict words go from device memory to
// the arena by one 64-lane copy kernel, and the call makes ONE stream
// synchronisation -- no DMA round trips, events or staging threads.  At C1
// sizes (1 k words) each host call is then launch + PCIe latency, where the
// batched path paid three streams' worth of copies and synchronisations.
// Kernel stores to the arena are visible to the host once the stream has
// synchronised (end-of-kernel system-scope release); the CPU's memcpy into
// it completes before the launch is issued.
struct Arena {
  uint8_t* base = nullptr;
  size_t off = 0;
  uint8_t* take(size_t bytes) {
    uint8_t* p = base + off;
    off += align256(bytes ? bytes : 16);
    return p;
  }
};

int host_stream1(amph_ctx* c, hipStream_t* s) {
  if (!c->streams[1]) HIP_TRY(hipStreamCreateWithFlags(&c->streams[1], hipStreamNonBlocking));
  *s = c->streams[1];
  return AMPH_OK;
}

bool small_call(const amph_ctx* c, size_t bytes) { return c->small_bytes && bytes <= c->small_bytes; }

// `bytes` of arena (plus 256 for the verdict words at its head) and the
// device verdict words, reset if an earlier call left them unknown
int small_begin(amph_ctx* c, size_t bytes, hipStream_t s, Arena* a, unsigned long long** dff) {
  if (c->small.ensure(bytes + 256) != hipSuccess) return fail(AMPH_E_NOMEM, "small-call arena");
  if (dev_ensure(c, c->small_ff, 256) != hipSuccess) return fail(AMPH_E_NOMEM, "small-call verdict words");
  if (c->small_ff_dirty) {
    HIP_TRY(hipMemsetAsync(c->small_ff.p, 0x7F, 256, s));
    c->small_ff_dirty = false;
  }
  a->base = (uint8_t*)c->small.p;
  a->off = 256;
  *dff = (unsigned long long*)c->small_ff.p;
  return AMPH_OK;
}

// after the kernels: verdict words to the arena head, one synchronisation
int small_end(amph_ctx* c, hipStream_t s, int n_ff) {
  hipError_t e = amph::launch_take_words((unsigned long long*)c->small_ff.p, (unsigned long long*)c->small.p,
                                         n_ff, s);
  if (e != hipSuccess) {
    c->small_ff_dirty = true;
    (void)hipStreamSynchronize(s);
    return hip_fail(e, "verdict copy");
  }
  e = hipStreamSynchronize(s);
  if (e != hipSuccess) {
    c->small_ff_dirty = true;
    return hip_fail(e, "small-call synchronise");
  }
  return AMPH_OK;
}

int small_launch_failed(amph_ctx* c, hipStream_t s, hipError_t e, const char* what) {
  c->small_ff_dirty = true;
  (void)hipStreamSynchronize(s);
  return hip_fail(e, what);
}

template <class Launch>
int run_small(amph_ctx* c, size_t words, const std::vector<HostIn>& ins, const std::vector<HostOut>& outs,
              bool with_ff, int64_t* first_fail, Launch& launch, size_t bytes) {
  if (first_fail) *first_fail = -1;
  if (words == 0) return AMPH_OK;
  HIP_TRY(use_device(c->device));
  hipStream_t s;
  if (int st = host_stream1(c, &s)) return st;
  Arena a;
  unsigned long long* dff;
  if (int st = small_begin(c, bytes, s, &a, &dff)) return st;
  std::vector<const uint4*> din;
  std::vector<uint4*> dout;
  for (const HostIn& x : ins) {
    uint8_t* p = a.take(words * x.bytes_per_word);
    if (amph::run_copy(copy_in(x, 0, words, p))) return io_failed();
    din.push_back((const uint4*)p);
  }
  for (const HostOut& x : outs) dout.push_back((uint4*)a.take(words * x.bytes_per_word));
  hipError_t e = launch(din, dout, words, with_ff ? dff : nullptr, cfg(c, s, words));
  if (e != hipSuccess) return small_launch_failed(c, s, e, "kernel launch");
  if (int st = small_end(c, s, with_ff ? 1 : 0)) return st;
  for (size_t k = 0; k < outs.size(); ++k)
    if (amph::run_copy(copy_out(outs[k], 0, words, dout[k]))) return io_failed();
  const unsigned long long v = *(volatile unsigned long long*)c->small.p;
  if (with_ff && v != amph::kNoFail) {
    if (first_fail) *first_fail = (int64_t)v;
    return AMPH_E_VERIFY;
  }
  return AMPH_OK;
}

size_t call_bytes(size_t words, const std::vector<HostIn>& ins, const std::vector<HostOut>& outs) {
  size_t b = 0;
  for (const HostIn& x : ins) b += align256(words * x.bytes_per_word);
  for (const HostOut& x : outs) b += align256(words * x.bytes_per_word);
  return b;
}

// An error part-way through leaves earlier batches' copies in flight (into
// the caller's page-locked buffers, or the slots): wait for them before
// returning, so nothing writes caller memory after the call has returned.
template <class Launch>
int run_batched(amph_ctx* c, size_t words, const std::vector<HostIn>& ins,
                const std::vector<HostOut>& outs, bool with_ff, int64_t* first_fail,
                Launch&& launch, size_t ff_scale = 1) {
  if (g_host_io) {  // the entry point's AMPH_F_HOST_IO: the pointers are descriptors
    std::vector<HostIn> ins2(ins);
    std::vector<HostOut> outs2(outs);
    for (HostIn& x : ins2) {
      x.io = (const amph_host_array*)x.host;
      if (words && (!x.io || !x.io->read)) return fail(AMPH_E_PARAM, "host array without a read callback");
    }
    for (HostOut& x : outs2) {
      x.io = (const amph_host_array*)x.host;
      if (words && (!x.io || !x.io->write)) return fail(AMPH_E_PARAM, "host array without a write callback");
    }
    g_host_io = false;  // consumed: the nested call sees explicit descriptors
    const int st = run_batched(c, words, ins2, outs2, with_ff, first_fail, launch, ff_scale);
    g_host_io = true;
    return st;
  }
  if (!c->sub.empty()) return run_sharded(c, words, ins, outs, with_ff, first_fail, launch, ff_scale);
  const size_t bytes = call_bytes(words, ins, outs);
  if (small_call(c, bytes)) return run_small(c, words, ins, outs, with_ff, first_fail, launch, bytes);
  const int rc = run_batched_impl(c, words, ins, outs, with_ff, first_fail, launch, ff_scale);
  if (rc != AMPH_OK && rc != AMPH_E_VERIFY) {
    for (int s = 0; s < amph_ctx::kSlots; ++s) {
      if (c->streams[s]) (void)hipStreamSynchronize(c->streams[s]);
      c->slots[s].busy = false;
    }
  }
  return rc;
}

// Multi-device context: contiguous shards of ceil(words / ndev), one thread
// per device running that device's own batched pipeline; the first failing
// shard (in word order) gives the global first-fail index.
template <class Launch>
int run_sharded(amph_ctx* g, size_t words, const std::vector<HostIn>& ins,
                const std::vector<HostOut>& outs, bool with_ff, int64_t* first_fail,
                Launch& launch, size_t ff_scale) {
  if (first_fail) *first_fail = -1;
  g_ev_start = g_ev_stop = nullptr;  // per-launch timing is single-device only
  if (words == 0) return AMPH_OK;
  const size_t nd = g->sub.size(), per = (words + nd - 1) / nd;
  struct Res {
    int st = AMPH_OK;
    int64_t ff = -1;
    std::string err;
  };
  std::vector<Res> res(nd);
  size_t used = 0;
  while (used < nd && used * per < words) ++used;
  amph::Latch done(used);
  for (size_t d = 0; d < used; ++d) {
    const size_t start = d * per, cnt = std::min(per, words - start);
    std::vector<HostIn> in2(ins);
    for (auto& x : in2) x.base += start;
    std::vector<HostOut> out2(outs);
    for (auto& x : out2) x.base += start;
    amph_ctx* s = g->sub[d];
    s->worker->post([&, d, s, cnt, in2 = std::move(in2), out2 = std::move(out2)]() {
      try {
        std::lock_guard<std::mutex> lk(s->mu);
        res[d].st = run_batched(s, cnt, in2, out2, with_ff, &res[d].ff, launch, ff_scale);
      } catch (const std::exception& e) {
        res[d].st = fail(AMPH_E_NOMEM, e.what());
      }
      if (res[d].st != AMPH_OK) res[d].err = g_last_error;
      s->worker_tasks.fetch_add(1, std::memory_order_relaxed);
      done.count_down();
    });
  }
  done.wait();
  for (size_t d = 0; d < used; ++d)
    if (res[d].st != AMPH_OK && res[d].st != AMPH_E_VERIFY) return fail(res[d].st, res[d].err);
  for (size_t d = 0; d < used; ++d)
    if (res[d].st == AMPH_E_VERIFY) {
      if (first_fail) *first_fail = (int64_t)(d * per * ff_scale) + res[d].ff;
      return AMPH_E_VERIFY;
    }
  return AMPH_OK;
}

int check_ctx(amph_ctx* c) { return c ? AMPH_OK : fail(AMPH_E_PARAM, "null context"); }

// Entry of a call that accepts AMPH_F_HOST_IO / one that refuses it.
#define AMPH_HOST_IO_ENTRY(flags)                                                      \
  if (((flags) & AMPH_F_HOST_IO) && ((flags) & AMPH_F_DEVICE))                         \
    return fail(AMPH_E_PARAM, "AMPH_F_HOST_IO and AMPH_F_DEVICE exclude each other");  \
  HostIoScope host_io_scope_(flags)
#define AMPH_NO_HOST_IO(flags) \
  if ((flags) & AMPH_F_HOST_IO) return fail(AMPH_E_PARAM, "AMPH_F_HOST_IO is not accepted by this call")

// recombineObject's word count and ragged party arrays (client
// SecretShareUtil.java:75,87-88): W = party 0's length / 16, and party j's
// word i is Arrays.copyOfRange(share_j, 16 i, 16 i + 16) -- a longer array
// is cut, a word running past the end of a shorter one is zero-padded, and a
// word STARTING past the end (16 i > length) throws
// ArrayIndexOutOfBoundsException (AMPH_E_RANGE).  So only word W-1 can be
// padded: *ragged says some party ends inside it (16 (W-1) <= length < 16 W).
// Callers that cannot take a padded word pass ragged = nullptr and get
// AMPH_E_LEN for it.
int party_words(const size_t* lens, int n, size_t* words, bool* ragged) {
  const size_t w = lens[0] / AMPH_WORD_WIDTH;
  bool rg = false;
  for (int j = 1; j < n; ++j) {
    if (lens[j] >= AMPH_WORD_WIDTH * w) continue;
    if (lens[j] + AMPH_WORD_WIDTH < AMPH_WORD_WIDTH * w)
      return fail(AMPH_E_RANGE, "Arrays.copyOfRange: word " +
                                    std::to_string(lens[j] / AMPH_WORD_WIDTH + 1) +
                                    " starts past the end of party " + std::to_string(j) + "'s " +
                                    std::to_string(lens[j]) + "-byte share array (" +
                                    std::to_string(w) + " words from party 0)");
    rg = true;
  }
  if (rg && !ragged) return fail(AMPH_E_LEN, "The provided shares must be of the same length");
  if (ragged) *ragged = rg;
  *words = w;
  return AMPH_OK;
}

int odo_words(const amph_odo* odos, int n, size_t* words, bool* ragged = nullptr) {
  if (!odos || n < 1 || n > AMPH_MAX_PARTIES)
    return fail(AMPH_E_PARAM, "n_parties must be in [1, 16] with a non-null ODO array");
  size_t lens[AMPH_MAX_PARTIES];
  for (int j = 0; j < n; ++j) lens[j] = odos[j].nbytes;
  if (int st = party_words(lens, n, words, ragged)) return st;
  for (int j = 0; j < n; ++j)
    if (*words && odos[j].nbytes && (!odos[j].secret_shares || !odos[j].r_shares || !odos[j].v_shares ||
                   !odos[j].w_shares || !odos[j].u_shares))
      return fail(AMPH_E_PARAM, "null ODO field");
  return AMPH_OK;
}

const uint8_t* odo_field(const amph_odo& o, int k) {
  switch (k) {
    case 0: return o.secret_shares;
    case 1: return o.r_shares;
    case 2: return o.v_shares;
    case 3: return o.w_shares;
    default: return o.u_shares;
  }
}

// Device-pointer word arrays are read and written as 16-byte vectors
// (global_load/store_dwordx4), so every one must be 16-byte aligned.
int check_dev_words(std::initializer_list<const void*> ptrs) {
  for (const void* p : ptrs)
    if (p && ((uintptr_t)p & 15))
      return fail(AMPH_E_PARAM, "device word arrays must be 16-byte aligned");
  return AMPH_OK;
}

// 24-character base64 records move as 8-byte vectors
int check_dev_records(const void* p) {
  if (p && ((uintptr_t)p & 7))
    return fail(AMPH_E_PARAM, "device base64 record arrays must be 8-byte aligned");
  return AMPH_OK;
}

int check_dev_odos(const amph_odo* odos, int n) {
  for (int j = 0; j < n; ++j)
    for (int k = 0; k < 5; ++k)
      if (int st = check_dev_words({odo_field(odos[j], k)})) return st;
  return AMPH_OK;
}

// device-mode first-fail: reset to the sentinel on the caller's stream,
// unless the caller accumulates (AMPH_F_ACCUMULATE: min-combine into it)
int reset_ff_dev(int64_t* ff, uint32_t flags, hipStream_t s) {
  if (!ff) return fail(AMPH_E_PARAM, "first_fail is required");
  if ((uintptr_t)ff & 7) return fail(AMPH_E_PARAM, "first_fail must be 8-byte aligned");
  if (!(flags & AMPH_F_ACCUMULATE)) HIP_TRY(hipMemsetAsync(ff, 0x7F, sizeof(int64_t), s));
  return AMPH_OK;
}

// ---- the ragged last word (party_words) --------------------------------------
// A ragged call runs words [0, W-1) as usual (every party holds them in full)
// and word W-1 as a one-word call over zero-padded copies of each array's
// bytes [16 (W-1), length): what Arrays.copyOfRange hands fromGfp.

// Stage array i's bytes [off, min(len[i], off + 16)), zero-padded, into the
// 16-byte word dst + 16 i.  src: host pointers (flags 0), amph_host_array
// descriptors (AMPH_F_HOST_IO; read through their callback) or device
// pointers (AMPH_F_DEVICE: dst is device memory, the copies go on s).
int stage_tail(const uint8_t* const* src, const size_t* len, int m, size_t off, uint8_t* dst,
               uint32_t flags, hipStream_t s) {
  if (flags & AMPH_F_DEVICE) {
    HIP_TRY(hipMemsetAsync(dst, 0, 16 * (size_t)m, s));
    for (int i = 0; i < m; ++i) {
      const size_t nb = std::min<size_t>(16, len[i] - off);
      if (nb) HIP_TRY(hipMemcpyAsync(dst + 16 * i, src[i] + off, nb, hipMemcpyDeviceToDevice, s));
    }
    return AMPH_OK;
  }
  std::memset(dst, 0, 16 * (size_t)m);
  for (int i = 0; i < m; ++i) {
    const size_t nb = std::min<size_t>(16, len[i] - off);
    if (!nb) continue;
    if (flags & AMPH_F_HOST_IO) {
      const amph_host_array* a = (const amph_host_array*)src[i];
      if (a->read(a, off, nb, dst + 16 * i)) return fail(AMPH_E_PARAM, "a host-array read callback failed");
    } else {
      std::memcpy(dst + 16 * i, src[i] + off, nb);
    }
  }
  return AMPH_OK;
}

// one host word to / from an output / input argument (descriptor under AMPH_F_HOST_IO)
int put_word(uint8_t* dst, size_t off, const uint8_t* w, uint32_t flags) {
  if (flags & AMPH_F_HOST_IO) {
    const amph_host_array* a = (const amph_host_array*)dst;
    if (a->write(a, off, 16, w)) return fail(AMPH_E_PARAM, "a host-array write callback failed");
  } else {
    std::memcpy(dst + off, w, 16);
  }
  return AMPH_OK;
}

// Device scratch of one ragged call: the staged words and a verdict word.
struct TailScratch {
  uint8_t* p = nullptr;
  hipStream_t s = nullptr;
  ~TailScratch() {
    if (p) (void)hipFreeAsync(p, s);
  }
};


// The ODO calls over ragged parties: `masked` = false runs
// amph_recombine_verify, true amph_mask_input (n_secrets <= W).
int ragged_odo_call(amph_ctx* c, const amph_odo* odos, int n, size_t W, bool masked, const uint8_t* secrets,
                    size_t n_secrets, uint8_t* out, int64_t* first_fail, uint32_t flags, void* stream) {
  const size_t off = AMPH_WORD_WIDTH * (W - 1);
  const bool dev = flags & AMPH_F_DEVICE, io = flags & AMPH_F_HOST_IO;
  hipStream_t s = (hipStream_t)stream;
  amph_odo head[AMPH_MAX_PARTIES], tail[AMPH_MAX_PARTIES];
  const uint8_t* src[5 * AMPH_MAX_PARTIES];
  size_t len[5 * AMPH_MAX_PARTIES];
  for (int j = 0; j < n; ++j) {
    head[j] = odos[j];
    head[j].nbytes = off;
    for (int k = 0; k < 5; ++k) {
      src[k * n + j] = odo_field(odos[j], k);
      len[k * n + j] = odos[j].nbytes;
    }
  }
  // words [0, W-1): secrets below W-1 masked there, word W-1's secret (if
  // any) in the tail; the rest verify only, as amph_mask_input does
  const size_t hs = std::min(n_secrets, W - 1), ts = n_secrets == W ? 1 : 0;
  int64_t hf = -1;
  int64_t* hff = dev ? first_fail : &hf;
  const int st = masked ? amph_mask_input(c, head, n, secrets, hs, out, hff, flags, stream)
                        : amph_recombine_verify(c, head, n, out, hff, flags, stream);
  if (st != AMPH_OK && st != AMPH_E_VERIFY) return st;
  auto point = [&](uint8_t* base) {
    for (int j = 0; j < n; ++j) {
      tail[j] = amph_odo{base + 16 * (0 * n + j), base + 16 * (1 * n + j), base + 16 * (2 * n + j),
                         base + 16 * (3 * n + j), base + 16 * (4 * n + j), 16};
    }
  };
  if (dev) {
    HIP_TRY(use_device(c->device));
    TailScratch sc;
    sc.s = s;
    HIP_TRY(hipMallocAsync((void**)&sc.p, 16 * 5 * (size_t)n + 16, s));
    int64_t* tf = (int64_t*)(sc.p + 16 * 5 * n);
    if (int r = stage_tail(src, len, 5 * n, off, sc.p, flags, s)) return r;
    HIP_TRY(hipMemsetAsync(tf, 0x7F, sizeof(int64_t), s));
    point(sc.p);
    const uint32_t tfl = AMPH_F_DEVICE | AMPH_F_ACCUMULATE;
    const int t = masked ? amph_mask_input(c, tail, n, ts ? secrets + off : nullptr, ts,
                                           ts ? out + off : nullptr, tf, tfl, stream)
                         : amph_recombine_verify(c, tail, n, out + off, tf, tfl, stream);
    if (t != AMPH_OK) return t;
    hipError_t e = amph::launch_ff_merge((unsigned long long*)first_fail, (const unsigned long long*)tf, W - 1, s);
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_ff_merge");
  }
  uint8_t words[16 * 5 * AMPH_MAX_PARTIES], sec[16], res[16];
  if (int r = stage_tail(src, len, 5 * n, off, words, flags, nullptr)) return r;
  point(words);
  if (ts) {
    if (io) {
      const amph_host_array* a = (const amph_host_array*)secrets;
      if (a->read(a, off, 16, sec)) return fail(AMPH_E_PARAM, "a host-array read callback failed");
    } else {
      std::memcpy(sec, secrets + off, 16);
    }
  }
  int64_t tf = -1;
  const int t = masked ? amph_mask_input(c, tail, n, ts ? sec : nullptr, ts, ts ? res : nullptr, &tf, 0, nullptr)
                       : amph_recombine_verify(c, tail, n, res, &tf, 0, nullptr);
  if (t != AMPH_OK && t != AMPH_E_VERIFY) return t;
  if ((!masked || ts) && put_word(out, off, res, flags)) return AMPH_E_PARAM;
  const int64_t v = st == AMPH_E_VERIFY ? hf : (t == AMPH_E_VERIFY ? (int64_t)(W - 1) : -1);
  if (first_fail) *first_fail = v;
  return v >= 0 ? AMPH_E_VERIFY : AMPH_OK;
}

}  // namespace

// ============================================================================
extern "C" {

int amph_time_next_launch(void* start_event, void* stop_event) {
  g_ev_start = (hipEvent_t)start_event;
  g_ev_stop = (hipEvent_t)stop_event;
  return AMPH_OK;
}

int amph_timing_event_create(void** event) {
  if (!event) return fail(AMPH_E_PARAM, "null event");
  hipEvent_t e = nullptr;
  HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  *event = (void*)e;
  return AMPH_OK;
}

int amph_timing_event_destroy(void* event) {
  if (event) HIP_TRY(hipEventDestroy((hipEvent_t)event));
  return AMPH_OK;
}

int amph_timing_event_record(void* event, void* stream) {
  if (!event) return fail(AMPH_E_PARAM, "null event");
  HIP_TRY(hipEventRecord((hipEvent_t)event, (hipStream_t)stream));
  return AMPH_OK;
}

int amph_timing_event_elapsed_ms(void* start_event, void* stop_event, float* ms) {
  if (!start_event || !stop_event || !ms) return fail(AMPH_E_PARAM, "null event or result");
  HIP_TRY(hipEventSynchronize((hipEvent_t)stop_event));
  HIP_TRY(hipEventElapsedTime(ms, (hipEvent_t)start_event, (hipEvent_t)stop_event));
  return AMPH_OK;
}

const char* amph_version(void) { return "amphora_amd 0.1.0 (gfx950)"; }

const char* amph_last_error(void) { return g_last_error.c_str(); }

const char* amph_strerror(int status) {
  switch (status) {
    case AMPH_OK: return "ok";
    case AMPH_E_VERIFY: return "Verification of secret has failed";
    case AMPH_E_LEN: return "length invariant violated";
    case AMPH_E_PARAM: return "invalid argument";
    case AMPH_E_HIP: return "HIP runtime error";
    case AMPH_E_NOMEM: return "out of memory";
    case AMPH_E_RANGE: return "array index out of range";
    default: return "unknown status";
  }
}

int amph_ctx_create(const uint8_t p_le[16], const uint8_t r_le[16], const uint8_t rinv_le[16],
                    int device, amph_ctx** out) {
  if (!out || !p_le || !r_le || !rinv_le) return fail(AMPH_E_PARAM, "null argument");
  *out = nullptr;
  amph_ctx* c = new (std::nothrow) amph_ctx();
  if (!c) return fail(AMPH_E_NOMEM, "context");
  int st = setup_field(c, p_le, r_le, rinv_le);
  if (st != AMPH_OK) {
    delete c;
    return st;
  }
  c->device = device;
  c->small.flags = hipHostMallocCoherent;  // kernels read and write the arena in place
  if (const char* g = std::getenv("AMPH_GRID_CAP")) c->grid_cap = std::max(0, std::atoi(g));
  if (const char* sb = std::getenv("AMPH_SMALL_BYTES")) c->small_bytes = (size_t)std::strtoull(sb, nullptr, 10);
  if (const char* pb = std::getenv("AMPH_PARTY_POOL_BYTES")) c->pool_cap_bytes = (size_t)std::strtoull(pb, nullptr, 10);
  if (const char* b = std::getenv("AMPH_BLOCK")) {
    const int v = std::atoi(b);
    if (v >= 64 && v <= amph::kMaxBlock && v % 64 == 0) c->block = v;
  }
  *out = c;
  return AMPH_OK;
}

int amph_ctx_create_multi(const uint8_t p_le[16], const uint8_t r_le[16],
                          const uint8_t rinv_le[16], const int* devices, int ndev,
                          amph_ctx** out) {
  if (!out || !devices || ndev < 1) return fail(AMPH_E_PARAM, "devices must name at least one device");
  if (ndev == 1) return amph_ctx_create(p_le, r_le, rinv_le, devices[0], out);
  *out = nullptr;
  amph_ctx* g = nullptr;
  if (int st = amph_ctx_create(p_le, r_le, rinv_le, devices[0], &g)) return st;
  for (int d = 0; d < ndev; ++d) {
    amph_ctx* s = nullptr;
    if (int st = amph_ctx_create(p_le, r_le, rinv_le, devices[d], &s)) {
      amph_ctx_destroy(g);
      return st;
    }
    s->worker.reset(new (std::nothrow) amph::DeviceWorker());
    g->sub.push_back(s);
    if (!s->worker) {
      amph_ctx_destroy(g);
      return fail(AMPH_E_NOMEM, "device worker thread");
    }
  }
  *out = g;
  return AMPH_OK;
}

int amph_ctx_device_count(const amph_ctx* c) {
  return c ? (c->sub.empty() ? 1 : (int)c->sub.size()) : 0;
}

void amph_ctx_destroy(amph_ctx* c) {
  if (!c) return;
  c->worker.reset();  // drains its queue and joins: nothing of c runs after this
  for (amph_ctx* s : c->sub) amph_ctx_destroy(s);
  c->sub.clear();
  if (c->streams[0] || c->slots[0].dev.p || c->ff.p) {
    (void)use_device(c->device);
    for (int s = 0; s < amph_ctx::kSlots; ++s) {
      if (c->streams[s]) (void)hipStreamSynchronize(c->streams[s]);
      c->slots[s].dev.release();
      c->slots[s].hin.release();
      c->slots[s].hout.release();
      for (hipEvent_t e : {c->slots[s].in_done, c->slots[s].k_done, c->slots[s].out_done})
        if (e) (void)hipEventDestroy(e);
      if (c->streams[s]) (void)hipStreamDestroy(c->streams[s]);
    }
    c->ff.release();
    c->tail.release();
    c->wire.release();
    c->xstage.release();
  }
  if (c->small.p || c->small_ff.p) {
    (void)use_device(c->device);
    if (c->streams[1]) (void)hipStreamSynchronize(c->streams[1]);
    c->small.release();
    c->small_ff.release();
  }
  if (c->xdev_done) {
    (void)use_device(c->device);
    (void)hipEventSynchronize(c->xdev_done);
    (void)hipEventDestroy(c->xdev_done);
  }
  c->xdev.release();
  if (!c->party_pool.empty()) {
    (void)use_device(c->device);
    for (DevBuf& b : c->party_pool) b.release();
  }
  delete c;
}

int amph_ctx_device(const amph_ctx* c) { return c ? c->device : -1; }

int amph_ctx_stats(amph_ctx* c, amph_stats* out) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  if (!out) return fail(AMPH_E_PARAM, "null stats output");
  *out = amph_stats{};
  auto add = [&](amph_ctx* x) {
    std::lock_guard<std::mutex> g(x->mu);
    out->kernel_launches += x->launches.load(std::memory_order_relaxed);
    out->pool_buffers += x->party_pool.size();
    out->pool_bytes += pool_bytes(x);
    out->device_workers += x->worker ? 1 : 0;
    out->worker_tasks += x->worker_tasks.load(std::memory_order_relaxed);
  };
  add(c);
  for (amph_ctx* s : c->sub) add(s);
  return AMPH_OK;
}

int amph_ctx_set_batch_words(amph_ctx* c, size_t words) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  std::lock_guard<std::mutex> g(c->mu);
  if (words) c->batch_words = words;
  for (amph_ctx* s : c->sub) amph_ctx_set_batch_words(s, words);
  return AMPH_OK;
}

int amph_recombine_verify(amph_ctx* c, const amph_odo* odos, int n, uint8_t* out_secrets,
                          int64_t* first_fail, uint32_t flags, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_HOST_IO_ENTRY(flags);
  size_t W;
  bool ragged;
  if (int st = odo_words(odos, n, &W, &ragged)) return st;
  if (W && !out_secrets) return fail(AMPH_E_PARAM, "null output");
  if (ragged) {
    if (flags & AMPH_F_DEVICE)
      if (int st = check_dev_odos(odos, n)) return st;
    return ragged_odo_call(c, odos, n, W, false, nullptr, 0, out_secrets, first_fail, flags, stream);
  }
  if (flags & AMPH_F_DEVICE) {
    if (int st = check_dev_odos(odos, n)) return st;
    if (int st = check_dev_words({out_secrets})) return st;
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(use_device(c->device));
    if (int st = reset_ff_dev(first_fail, flags, s)) return st;
    amph::OdoSet set{};
    for (int k = 0; k < 5; ++k)
      for (int j = 0; j < n; ++j) set.f[k][j] = (const uint4*)odo_field(odos[j], k);
    hipError_t e = amph::launch_recombine_verify(set, n, W, (uint4*)out_secrets,
                                                 (unsigned long long*)first_fail, c->f, cfg(c, s, W));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_rv");
  }
  std::lock_guard<std::mutex> g(c->mu);
  std::vector<HostIn> ins;
  for (int k = 0; k < 5; ++k)
    for (int j = 0; j < n; ++j) ins.push_back({odo_field(odos[j], k), 16});
  return run_batched(c, W, ins, {{out_secrets, 16}}, true, first_fail,
                     [&](auto& din, auto& dout, size_t cnt, unsigned long long* ff,
                         const amph::LaunchCfg& lc) {
                       amph::OdoSet set{};
                       for (int k = 0; k < 5; ++k)
                         for (int j = 0; j < n; ++j) set.f[k][j] = din[k * n + j];
                       return amph::launch_recombine_verify(set, n, cnt, dout[0], ff, c->f, lc);
                     });
}

int amph_mask_input(amph_ctx* c, const amph_odo* odos, int n, const uint8_t* secrets,
                    size_t n_secrets, uint8_t* out_masked, int64_t* first_fail, uint32_t flags,
                    void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_HOST_IO_ENTRY(flags);
  size_t W;
  bool ragged;
  if (int st = odo_words(odos, n, &W, &ragged)) return st;
  if (n_secrets > W) {
    // The reference verifies every mask before it indexes past the last one
    // (DefaultAmphoraClient.java:153 before :160): a MAC failure outranks the
    // length error.  Verify all W words (n_secrets = 0), then report.  Device
    // mode waits for the verdict here -- an error path, so the stream sync
    // costs nothing a correct call pays.
    int st = amph_mask_input(c, odos, n, nullptr, 0, nullptr, first_fail, flags, stream);
    if (st != AMPH_OK) return st;
    if ((flags & AMPH_F_DEVICE) && first_fail) {
      HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
      int64_t h = 0;
      HIP_TRY(hipMemcpy(&h, first_fail, sizeof h, hipMemcpyDeviceToHost));  // kPageableRule
      if ((uint64_t)h != amph::kNoFail)
        return fail(AMPH_E_VERIFY, "input mask MAC check failed at word " + std::to_string(h));
    }
    return fail(AMPH_E_LEN, "more secret words than verified input masks");
  }
  if (n_secrets && (!secrets || !out_masked)) return fail(AMPH_E_PARAM, "null secrets/output");
  if (ragged) {
    if (flags & AMPH_F_DEVICE)
      if (int st = check_dev_odos(odos, n)) return st;
    return ragged_odo_call(c, odos, n, W, true, secrets, n_secrets, out_masked, first_fail, flags, stream);
  }
  if (flags & AMPH_F_DEVICE) {
    if (int st = check_dev_odos(odos, n)) return st;
    if (int st = check_dev_words({secrets, out_masked})) return st;
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(use_device(c->device));
    if (int st = reset_ff_dev(first_fail, flags, s)) return st;
    amph::OdoSet set{};
    for (int k = 0; k < 5; ++k)
      for (int j = 0; j < n; ++j) set.f[k][j] = (const uint4*)odo_field(odos[j], k);
    hipError_t e = amph::launch_mask_input(set, n, W, (const uint4*)secrets, n_secrets,
                                           (uint4*)out_masked, (unsigned long long*)first_fail,
                                           c->f, cfg(c, s, W));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_mask");
  }
  std::lock_guard<std::mutex> g(c->mu);
  std::vector<HostIn> ins;
  for (int k = 0; k < 5; ++k)
    for (int j = 0; j < n; ++j) ins.push_back({odo_field(odos[j], k), 16});
  ins.push_back({secrets, 16});
  int st = run_batched(c, n_secrets, ins, {{out_masked, 16}}, true, first_fail,
                       [&](auto& din, auto& dout, size_t cnt, unsigned long long* ff,
                           const amph::LaunchCfg& lc) {
                         amph::OdoSet set{};
                         for (int k = 0; k < 5; ++k)
                           for (int j = 0; j < n; ++j) set.f[k][j] = din[k * n + j];
                         return amph::launch_mask_input(set, n, cnt, din[5 * n], cnt, dout[0],
                                                        ff, c->f, lc);
                       });
  if (st != AMPH_OK || n_secrets == W) return st;
  // verify-only tail [n_secrets, W) (the Java loop reads inputMasks.get(i) for
  // i < secret.size() only, but verifyOutputDeliveryObjects checked them all)
  std::vector<HostIn> tins;
  for (int k = 0; k < 5; ++k)
    for (int j = 0; j < n; ++j) tins.push_back({odo_field(odos[j], k), 16, n_secrets});
  int64_t tf = -1;
  st = run_batched(c, W - n_secrets, tins, {}, true, &tf,
                   [&](auto& din, auto&, size_t cnt, unsigned long long* ff,
                       const amph::LaunchCfg& lc) {
                     amph::OdoSet set{};
                     for (int k = 0; k < 5; ++k)
                       for (int j = 0; j < n; ++j) set.f[k][j] = din[k * n + j];
                     return amph::launch_mask_input(set, n, cnt, nullptr, 0, nullptr, ff, c->f, lc);
                   });
  if (st == AMPH_E_VERIFY && first_fail) *first_fail = (int64_t)n_secrets + tf;
  return st;
}

int amph_recombine(amph_ctx* c, const uint8_t* const* shares, int n, size_t nbytes, uint8_t* out,
                   uint32_t flags, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_HOST_IO_ENTRY(flags);
  if (!shares || n < 1 || n > AMPH_MAX_PARTIES) return fail(AMPH_E_PARAM, "n_parties must be in [1, 16]");
  const size_t W = nbytes / AMPH_WORD_WIDTH;
  if (W && !out) return fail(AMPH_E_PARAM, "null output");
  for (int j = 0; j < n; ++j)
    if (W && !shares[j]) return fail(AMPH_E_PARAM, "null share array");
  if (flags & AMPH_F_DEVICE) {
    for (int j = 0; j < n; ++j)
      if (int st = check_dev_words({shares[j]})) return st;
    if (int st = check_dev_words({out})) return st;
    HIP_TRY(use_device(c->device));
    amph::ShareSet set{};
    for (int j = 0; j < n; ++j) set.s[j] = (const uint4*)shares[j];
    hipError_t e = amph::launch_recombine(set, n, W, (uint4*)out, c->f, cfg(c, (hipStream_t)stream, W));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_recombine");
  }
  std::lock_guard<std::mutex> g(c->mu);
  std::vector<HostIn> ins;
  for (int j = 0; j < n; ++j) ins.push_back({shares[j], 16});
  return run_batched(c, W, ins, {{out, 16}}, false, nullptr,
                     [&](auto& din, auto& dout, size_t cnt, unsigned long long*,
                         const amph::LaunchCfg& lc) {
                       amph::ShareSet set{};
                       for (int j = 0; j < n; ++j) set.s[j] = din[j];
                       return amph::launch_recombine(set, n, cnt, dout[0], c->f, lc);
                     });
}

int amph_recombine_object(amph_ctx* c, const uint8_t* const* shares, int n, const size_t* nbytes,
                          uint8_t* out, uint32_t flags, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_HOST_IO_ENTRY(flags);
  if (!shares || !nbytes || n < 1 || n > AMPH_MAX_PARTIES)
    return fail(AMPH_E_PARAM, "n_parties must be in [1, 16] with non-null share and length arrays");
  size_t W;
  bool ragged;
  if (int st = party_words(nbytes, n, &W, &ragged)) return st;
  if (!ragged) return amph_recombine(c, shares, n, AMPH_WORD_WIDTH * W, out, flags, stream);
  const size_t off = AMPH_WORD_WIDTH * (W - 1);
  if (!out) return fail(AMPH_E_PARAM, "null output");
  for (int j = 0; j < n; ++j)
    if (!shares[j] && nbytes[j]) return fail(AMPH_E_PARAM, "null share array");
  if (int st = amph_recombine(c, shares, n, off, out, flags, stream)) return st;
  const uint8_t* tail[AMPH_MAX_PARTIES];
  if (flags & AMPH_F_DEVICE) {
    for (int j = 0; j < n; ++j)
      if (int st = check_dev_words({shares[j]})) return st;
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(use_device(c->device));
    TailScratch sc;
    sc.s = s;
    HIP_TRY(hipMallocAsync((void**)&sc.p, 16 * (size_t)n, s));
    if (int st = stage_tail(shares, nbytes, n, off, sc.p, flags, s)) return st;
    for (int j = 0; j < n; ++j) tail[j] = sc.p + 16 * j;
    return amph_recombine(c, tail, n, 16, out + off, flags, stream);
  }
  uint8_t words[16 * AMPH_MAX_PARTIES], res[16];
  if (int st = stage_tail(shares, nbytes, n, off, words, flags, nullptr)) return st;
  for (int j = 0; j < n; ++j) tail[j] = words + 16 * j;
  if (int st = amph_recombine(c, tail, n, 16, res, 0, nullptr)) return st;
  return put_word(out, off, res, flags);
}

int amph_verify(amph_ctx* c, const uint8_t* y, const uint8_t* r, const uint8_t* u,
                const uint8_t* v, const uint8_t* w, size_t words, int64_t* first_fail,
                uint32_t flags, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_HOST_IO_ENTRY(flags);
  if (words && (!y || !r || !u || !v || !w)) return fail(AMPH_E_PARAM, "null input");
  if (flags & AMPH_F_DEVICE) {
    if (int st = check_dev_words({y, r, u, v, w})) return st;
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(use_device(c->device));
    if (int st = reset_ff_dev(first_fail, flags, s)) return st;
    hipError_t e = amph::launch_verify((const uint4*)y, (const uint4*)r, (const uint4*)u,
                                       (const uint4*)v, (const uint4*)w, words,
                                       (unsigned long long*)first_fail, c->f, cfg(c, s, words));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_verify");
  }
  std::lock_guard<std::mutex> g(c->mu);
  return run_batched(c, words, {{y, 16}, {r, 16}, {u, 16}, {v, 16}, {w, 16}}, {}, true,
                     first_fail,
                     [&](auto& din, auto&, size_t cnt, unsigned long long* ff,
                         const amph::LaunchCfg& lc) {
                       return amph::launch_verify(din[0], din[1], din[2], din[3], din[4], cnt, ff,
                                                  c->f, lc);
                     });
}

int amph_verify_message(amph_ctx* c, const uint8_t y[16], const uint8_t r[16], const uint8_t u[16],
                        const uint8_t v[16], const uint8_t w[16], char* buf, size_t cap) {
  if (check_ctx(c) || !y || !r || !u || !v || !w) return -AMPH_E_PARAM;
  const u128 Y = ld128(y) % c->p, R = ld128(r) % c->p, V = ld128(v) % c->p;
  const u128 Wv = ld128(w), Uv = ld128(u);
  const u128 aw = mulmod_host(c, Y, R), au = mulmod_host(c, V, R);
  const std::string m = "Verification of secret has failed:\n\t" + dec(Wv) + " = " + dec(ld128(y)) +
                        " * " + dec(ld128(r)) + "   &&   " + dec(Uv) + " = " + dec(ld128(v)) +
                        " * " + dec(ld128(r)) + "\n\t" + dec(Wv) + " = " + dec(aw) +
                        "   &&   " + dec(Uv) + " = " + dec(au);
  if (buf && cap) {
    const size_t k = std::min(cap - 1, m.size());
    std::memcpy(buf, m.data(), k);
    buf[k] = 0;
  }
  return (int)m.size();
}

int amph_convert_share(amph_ctx* c, const uint8_t* masked, const uint8_t* tuples, size_t words,
                       const uint8_t mac_key_le[16], int use_zero, uint8_t* out, uint32_t flags,
                       void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_HOST_IO_ENTRY(flags);
  if (!mac_key_le) return fail(AMPH_E_PARAM, "null mac key");
  if (words && (!masked || !tuples || !out)) return fail(AMPH_E_PARAM, "null buffer");
  // [alpha] = alpha R mod p, computed once per call on the host
  const W4 alpha = amph::mont_mul(w4_of(ld128(mac_key_le)), amph::r2_word(c->f), c->f);
  if (flags & AMPH_F_DEVICE) {
    if (int st = check_dev_words({masked, tuples, out})) return st;
    HIP_TRY(use_device(c->device));
    hipError_t e = amph::launch_convert_share((const uint4*)masked, (const uint4*)tuples, words,
                                              alpha, use_zero, (uint4*)out, c->f,
                                              cfg(c, (hipStream_t)stream, words));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_conv");
  }
  std::lock_guard<std::mutex> g(c->mu);
  return run_batched(c, words, {{masked, 16}, {tuples, 32}}, {{out, 32}}, false, nullptr,
                     [&](auto& din, auto& dout, size_t cnt, unsigned long long*,
                         const amph::LaunchCfg& lc) {
                       return amph::launch_convert_share(din[0], din[1], cnt, alpha, use_zero,
                                                         dout[0], c->f, lc);
                     });
}

int amph_odo_pre(amph_ctx* c, const uint8_t* share_data, size_t share_stride,
                 const uint8_t* masks, const uint8_t* triples, size_t words, uint8_t* oy,
                 uint8_t* orr, uint8_t* ov, uint8_t* omag, uint8_t* oneg, uint32_t flags,
                 void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_HOST_IO_ENTRY(flags);
  if (share_stride != 16 && share_stride != 32)
    return fail(AMPH_E_PARAM, "share_stride must be 16 or 32");
  if (words && (!share_data || !masks || !triples || !oy || !orr || !ov || !omag || !oneg))
    return fail(AMPH_E_PARAM, "null buffer");
  const int sw = (int)(share_stride / 16);
  if (flags & AMPH_F_DEVICE) {
    if (int st = check_dev_words({share_data, masks, triples, oy, orr, ov, omag})) return st;
    HIP_TRY(use_device(c->device));
    hipError_t e = amph::launch_odo_pre((const uint4*)share_data, sw, (const uint4*)masks,
                                        (const uint4*)triples, words, (uint4*)oy, (uint4*)orr,
                                        (uint4*)ov, (uint4*)omag, (uint32_t*)oneg, c->f,
                                        cfg(c, (hipStream_t)stream, words));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_odo_pre");
  }
  std::lock_guard<std::mutex> g(c->mu);
  return run_batched(c, words, {{share_data, share_stride}, {masks, 64}, {triples, 192}},
                     {{oy, 16}, {orr, 16}, {ov, 16}, {omag, 64}, {oneg, 4}}, false, nullptr,
                     [&](auto& din, auto& dout, size_t cnt, unsigned long long*,
                         const amph::LaunchCfg& lc) {
                       return amph::launch_odo_pre(din[0], sw, din[1], din[2], cnt, dout[0],
                                                   dout[1], dout[2], dout[3],
                                                   (uint32_t*)dout[4], c->f, lc);
                     });
}

int amph_open_diffs(amph_ctx* c, const uint8_t* const* mags, const uint8_t* const* negs, int n,
                    size_t n_pairs, uint8_t* out, uint32_t flags, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_HOST_IO_ENTRY(flags);
  if (!mags || !negs || n < 1 || n > AMPH_MAX_PARTIES) return fail(AMPH_E_PARAM, "n_parties must be in [1, 16]");
  if (n_pairs % 2) return fail(AMPH_E_LEN, "n_pairs must be 2 * words");
  const size_t W = n_pairs / 2;
  if (W && !out) return fail(AMPH_E_PARAM, "null output");
  for (int j = 0; j < n; ++j)
    if (W && (!mags[j] || !negs[j])) return fail(AMPH_E_PARAM, "null diff array");
  if (flags & AMPH_F_DEVICE) {
    for (int j = 0; j < n; ++j)
      if (int st = check_dev_words({mags[j]})) return st;
    if (int st = check_dev_words({out})) return st;
    HIP_TRY(use_device(c->device));
    amph::SignedSet set{};
    for (int j = 0; j < n; ++j) {
      set.mag[j] = (const uint4*)mags[j];
      set.neg[j] = (const uint32_t*)negs[j];
    }
    hipError_t e = amph::launch_open_diffs(set, n, W, (uint4*)out, c->f, cfg(c, (hipStream_t)stream, W));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_open");
  }
  std::lock_guard<std::mutex> g(c->mu);
  std::vector<HostIn> ins;
  for (int j = 0; j < n; ++j) ins.push_back({mags[j], 64});
  for (int j = 0; j < n; ++j) ins.push_back({negs[j], 4});
  return run_batched(c, W, ins, {{out, 64}}, false, nullptr,
                     [&](auto& din, auto& dout, size_t cnt, unsigned long long*,
                         const amph::LaunchCfg& lc) {
                       amph::SignedSet set{};
                       for (int j = 0; j < n; ++j) {
                         set.mag[j] = din[j];
                         set.neg[j] = (const uint32_t*)din[n + j];
                       }
                       return amph::launch_open_diffs(set, n, cnt, dout[0], c->f, lc);
                     });
}

int amph_odo_post(amph_ctx* c, const uint8_t* opened, const uint8_t* triples, size_t words,
                  int is_player0, uint8_t* ow, uint8_t* ou, uint32_t flags, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_HOST_IO_ENTRY(flags);
  if (words && (!opened || !triples || !ow || !ou)) return fail(AMPH_E_PARAM, "null buffer");
  if (flags & AMPH_F_DEVICE) {
    if (int st = check_dev_words({opened, triples, ow, ou})) return st;
    HIP_TRY(use_device(c->device));
    hipError_t e = amph::launch_odo_post((const uint4*)opened, (const uint4*)triples, words,
                                         is_player0, (uint4*)ow, (uint4*)ou, c->f,
                                         cfg(c, (hipStream_t)stream, words));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_odo_post");
  }
  std::lock_guard<std::mutex> g(c->mu);
  return run_batched(c, words, {{opened, 64}, {triples, 192}}, {{ow, 16}, {ou, 16}}, false,
                     nullptr,
                     [&](auto& din, auto& dout, size_t cnt, unsigned long long*,
                         const amph::LaunchCfg& lc) {
                       return amph::launch_odo_post(din[0], din[1], cnt, is_player0, dout[0],
                                                    dout[1], c->f, lc);
                     });
}

int amph_open_post(amph_ctx* c, const uint8_t* const* mags, const uint8_t* const* negs, int n,
                   const uint8_t* triples, size_t words, int is_player0, uint8_t* ow, uint8_t* ou,
                   uint32_t flags, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_HOST_IO_ENTRY(flags);
  if (!mags || !negs || n < 1 || n > AMPH_MAX_PARTIES) return fail(AMPH_E_PARAM, "n_parties must be in [1, 16]");
  if (words && (!triples || !ow || !ou)) return fail(AMPH_E_PARAM, "null buffer");
  for (int j = 0; j < n; ++j)
    if (words && (!mags[j] || !negs[j])) return fail(AMPH_E_PARAM, "null diff array");
  if (flags & AMPH_F_DEVICE) {
    for (int j = 0; j < n; ++j)
      if (int st = check_dev_words({mags[j]})) return st;
    if (int st = check_dev_words({triples, ow, ou})) return st;
    HIP_TRY(use_device(c->device));
    amph::SignedSet set{};
    for (int j = 0; j < n; ++j) {
      set.mag[j] = (const uint4*)mags[j];
      set.neg[j] = (const uint32_t*)negs[j];
    }
    hipError_t e = amph::launch_open_post(set, n, (const uint4*)triples, words, is_player0, (uint4*)ow,
                                          (uint4*)ou, c->f, cfg(c, (hipStream_t)stream, words));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_open_post");
  }
  std::lock_guard<std::mutex> g(c->mu);
  std::vector<HostIn> ins;
  for (int j = 0; j < n; ++j) ins.push_back({mags[j], 64});
  for (int j = 0; j < n; ++j) ins.push_back({negs[j], 4});
  ins.push_back({triples, 192});
  return run_batched(c, words, ins, {{ow, 16}, {ou, 16}}, false, nullptr,
                     [&](auto& din, auto& dout, size_t cnt, unsigned long long*,
                         const amph::LaunchCfg& lc) {
                       amph::SignedSet set{};
                       for (int j = 0; j < n; ++j) {
                         set.mag[j] = din[j];
                         set.neg[j] = (const uint32_t*)din[n + j];
                       }
                       return amph::launch_open_post(set, n, din[2 * n], cnt, is_player0, dout[0],
                                                     dout[1], c->f, lc);
                     });
}

int amph_to_gfp(amph_ctx* c, const uint8_t* in, size_t words, uint8_t* out, uint32_t flags,
                void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_HOST_IO_ENTRY(flags);
  if (words && (!in || !out)) return fail(AMPH_E_PARAM, "null buffer");
  if (flags & AMPH_F_DEVICE) {
    if (int st = check_dev_words({in, out})) return st;
    HIP_TRY(use_device(c->device));
    hipError_t e = amph::launch_to_gfp((const uint4*)in, words, (uint4*)out, c->f, cfg(c, (hipStream_t)stream, words));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_to_gfp");
  }
  std::lock_guard<std::mutex> g(c->mu);
  return run_batched(c, words, {{in, 16}}, {{out, 16}}, false, nullptr,
                     [&](auto& din, auto& dout, size_t cnt, unsigned long long*,
                         const amph::LaunchCfg& lc) {
                       return amph::launch_to_gfp(din[0], cnt, dout[0], c->f, lc);
                     });
}

int amph_from_gfp(amph_ctx* c, const uint8_t* in, size_t words, uint8_t* out, uint32_t flags,
                  void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_HOST_IO_ENTRY(flags);
  if (words && (!in || !out)) return fail(AMPH_E_PARAM, "null buffer");
  if (flags & AMPH_F_DEVICE) {
    if (int st = check_dev_words({in, out})) return st;
    HIP_TRY(use_device(c->device));
    hipError_t e = amph::launch_from_gfp((const uint4*)in, words, (uint4*)out, c->f, cfg(c, (hipStream_t)stream, words));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_from_gfp");
  }
  std::lock_guard<std::mutex> g(c->mu);
  return run_batched(c, words, {{in, 16}}, {{out, 16}}, false, nullptr,
                     [&](auto& din, auto& dout, size_t cnt, unsigned long long*,
                         const amph::LaunchCfg& lc) {
                       return amph::launch_from_gfp(din[0], cnt, dout[0], c->f, lc);
                     });
}

int amph_mask_words(amph_ctx* c, const uint8_t* secrets, const uint8_t* masks, size_t words,
                    uint8_t* out, uint32_t flags, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_HOST_IO_ENTRY(flags);
  if (words && (!secrets || !masks || !out)) return fail(AMPH_E_PARAM, "null buffer");
  if (flags & AMPH_F_DEVICE) {
    if (int st = check_dev_words({secrets, masks, out})) return st;
    HIP_TRY(use_device(c->device));
    hipError_t e = amph::launch_mask_words((const uint4*)secrets, (const uint4*)masks, words,
                                           (uint4*)out, c->f, cfg(c, (hipStream_t)stream, words));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_mask_words");
  }
  std::lock_guard<std::mutex> g(c->mu);
  return run_batched(c, words, {{secrets, 16}, {masks, 16}}, {{out, 16}}, false, nullptr,
                     [&](auto& din, auto& dout, size_t cnt, unsigned long long*,
                         const amph::LaunchCfg& lc) {
                       return amph::launch_mask_words(din[0], din[1], cnt, dout[0], c->f, lc);
                     });
}

int amph_mask_word_host(amph_ctx* c, const uint8_t secret[16], const uint8_t mask[16], uint8_t out[16]) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  if (!secret || !mask || !out) return fail(AMPH_E_PARAM, "null word");
  const u128 s = ld128(secret) % c->p, m = ld128(mask) % c->p;
  u128 d = s - m;  // mod 2^128; the true difference (s - m) mod p is < p < 2^128
  if (s < m) d += c->p;
  const W4 x = amph::mont_mul(w4_of(d), amph::r2_word(c->f), c->f);  // d R mod p, reduced
  for (int i = 0; i < 4; ++i) std::memcpy(out + 4 * i, &x.v[i], 4);
  return AMPH_OK;
}

// ---- base64 wire codec ---------------------------------------------------------
}  // extern "C"
namespace {
size_t b64_padding(const char* last2) {
  return (last2[1] == '=') + (last2[1] == '=' && last2[0] == '=');
}

// Host-path helper for the < 1-unit tail: copy in, run, copy out, synchronously.
template <class Launch>
int run_tail(amph_ctx* c, const void* in, size_t in_bytes, void* out, size_t out_bytes,
             bool with_bad, unsigned long long* bad_host, Launch&& launch) {
  HIP_TRY(use_device(c->device));
  hipError_t e = dev_ensure(c, c->tail, 512);
  if (e != hipSuccess) return fail(AMPH_E_NOMEM, "tail scratch");
  if (!c->streams[0]) HIP_TRY(hipStreamCreateWithFlags(&c->streams[0], hipStreamNonBlocking));
  hipStream_t s = c->streams[0];  // the context's own stream: no device-wide sync
  uint8_t* d = (uint8_t*)c->tail.p;
  // `in` is caller memory, pageable in general: a blocking copy after the
  // stream is idle (kPageableRule, above read_back)
  HIP_TRY(hipStreamSynchronize(s));
  HIP_TRY(hipMemcpy(d, in, in_bytes, hipMemcpyHostToDevice));
  if (with_bad) HIP_TRY(hipMemsetAsync(d + 448, 0x7F, 8, s));
  e = launch(d, d + 256, (unsigned long long*)(d + 448), cfg(c, s, 1));
  if (e != hipSuccess) return hip_fail(e, "codec tail");
  HIP_TRY(read_back(s, {{out, d + 256, out_bytes}, {bad_host, d + 448, with_bad ? (size_t)8 : 0}}));
  return AMPH_OK;
}
}  // namespace
extern "C" {

int amph_base64_encode(amph_ctx* c, const uint8_t* in, size_t nbytes, char* out, uint32_t flags,
                       void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_NO_HOST_IO(flags);
  if (nbytes && (!in || !out)) return fail(AMPH_E_PARAM, "null buffer");
  if (flags & AMPH_F_DEVICE) {
    HIP_TRY(use_device(c->device));
    hipError_t e = amph::launch_b64_encode(in, nbytes, out, cfg(c, (hipStream_t)stream, (nbytes + 11) / 12));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_b64_encode");
  }
  std::lock_guard<std::mutex> g(c->mu);
  const size_t units = nbytes / 12, rem = nbytes % 12;
  int st = run_batched(c, units, {{in, 12}}, {{(uint8_t*)out, 16}}, false, nullptr,
                       [&](auto& din, auto& dout, size_t cnt, unsigned long long*,
                           const amph::LaunchCfg& lc) {
                         return amph::launch_b64_encode((const uint8_t*)din[0], 12 * cnt,
                                                        (char*)dout[0], lc);
                       });
  if (st != AMPH_OK || rem == 0) return st;
  return run_tail(c, in + 12 * units, rem, out + 16 * units, 4 * ((rem + 2) / 3), false, nullptr,
                  [&](uint8_t* di, uint8_t* dout, unsigned long long*, const amph::LaunchCfg& lc) {
                    return amph::launch_b64_encode(di, rem, (char*)dout, lc);
                  });
}

int amph_base64_decode(amph_ctx* c, const char* in, size_t nchars, uint8_t* out,
                       size_t* out_bytes, int64_t* bad_index, uint32_t flags, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_NO_HOST_IO(flags);
  if (nchars % 4) return fail(AMPH_E_LEN, "base64 input length must be a multiple of 4");
  if (nchars && (!in || !out)) return fail(AMPH_E_PARAM, "null buffer");
  if (bad_index && !(flags & AMPH_F_DEVICE)) *bad_index = -1;
  if (nchars == 0) {
    if (out_bytes) *out_bytes = 0;
    return AMPH_OK;
  }
  char last2[2];
  if (flags & AMPH_F_DEVICE) {
    HIP_TRY(use_device(c->device));
    if (!bad_index) return fail(AMPH_E_PARAM, "bad_index is required");
    // out_bytes given: one 2-byte read-back decides the padding (the only
    // synchronous step); null: fully asynchronous, the kernel sizes it
    size_t ob = amph::kB64PadOnDevice;
    if (out_bytes) {
      HIP_TRY(read_back((hipStream_t)stream, {{last2, in + nchars - 2, 2}}));
      ob = 3 * nchars / 4 - b64_padding(last2);
      *out_bytes = ob;
    }
    if (int st = reset_ff_dev(bad_index, flags, (hipStream_t)stream)) return st;
    hipError_t e = amph::launch_b64_decode(in, nchars, out, ob, (unsigned long long*)bad_index,
                                           cfg(c, (hipStream_t)stream, (nchars + 15) / 16));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_b64_decode");
  }
  std::lock_guard<std::mutex> g(c->mu);
  std::memcpy(last2, in + nchars - 2, 2);
  const size_t ob = 3 * nchars / 4 - b64_padding(last2);
  if (out_bytes) *out_bytes = ob;
  // full 16-char units that contain no padding go through the batched path
  const size_t units = (nchars - 4) / 16, tail_chars = nchars - 16 * units;
  int64_t bad = -1;
  int st = run_batched(c, units, {{(const uint8_t*)in, 16}}, {{out, 12}}, true, &bad,
                       [&](auto& din, auto& dout, size_t cnt, unsigned long long* ff,
                           const amph::LaunchCfg& lc) {
                         return amph::launch_b64_decode((const char*)din[0], 16 * cnt,
                                                        (uint8_t*)dout[0], 12 * cnt, ff, lc,
                                                        false);  // batches never end the text
                       },
                       16);  // the kernel reports a character offset, 16 per unit
  if (st != AMPH_OK && st != AMPH_E_VERIFY) return st;
  unsigned long long tb = amph::kNoFail;
  const size_t tail_out = ob - 12 * units;
  int st2 = run_tail(c, in + 16 * units, tail_chars, out + 12 * units, tail_out, true, &tb,
                     [&](uint8_t* di, uint8_t* dout, unsigned long long* bb, const amph::LaunchCfg& lc) {
                       return amph::launch_b64_decode((const char*)di, tail_chars, dout, tail_out,
                                                      bb, lc);
                     });
  if (st2 != AMPH_OK) return st2;
  // the tail kernel saw the tail as the whole text, so its '=' rule is exact
  const int64_t first = st == AMPH_E_VERIFY ? bad : (tb != amph::kNoFail ? (int64_t)(16 * units + tb) : -1);
  if (first >= 0) {
    if (bad_index) *bad_index = first;
    return fail(AMPH_E_PARAM, "Illegal base64 character at index " + std::to_string(first));
  }
  return AMPH_OK;
}

int amph_base64_encode_words(amph_ctx* c, const uint8_t* words16, size_t words, char* out24,
                             uint32_t flags, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_NO_HOST_IO(flags);
  if (words && (!words16 || !out24)) return fail(AMPH_E_PARAM, "null buffer");
  if (flags & AMPH_F_DEVICE) {
    if (int st = check_dev_words({words16})) return st;
    if (int st = check_dev_records(out24)) return st;
    HIP_TRY(use_device(c->device));
    hipError_t e = amph::launch_b64_words((const uint4*)words16, words, out24, cfg(c, (hipStream_t)stream, words));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_b64_words");
  }
  std::lock_guard<std::mutex> g(c->mu);
  return run_batched(c, words, {{words16, 16}}, {{(uint8_t*)out24, 24}}, false, nullptr,
                     [&](auto& din, auto& dout, size_t cnt, unsigned long long*,
                         const amph::LaunchCfg& lc) {
                       return amph::launch_b64_words(din[0], cnt, (char*)dout[0], lc);
                     });
}

int amph_base64_decode_words(amph_ctx* c, const char* in24, size_t words, uint8_t* out16,
                             int64_t* bad_index, uint32_t flags, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_NO_HOST_IO(flags);
  if (words && (!in24 || !out16)) return fail(AMPH_E_PARAM, "null buffer");
  if (flags & AMPH_F_DEVICE) {
    if (int st = check_dev_words({out16})) return st;
    if (int st = check_dev_records(in24)) return st;
    hipStream_t s = (hipStream_t)stream;
    HIP_TRY(use_device(c->device));
    if (int st = reset_ff_dev(bad_index, flags, s)) return st;
    hipError_t e = amph::launch_b64_unwords(in24, words, (uint4*)out16, (unsigned long long*)bad_index,
                                            cfg(c, s, words));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_b64_unwords");
  }
  std::lock_guard<std::mutex> g(c->mu);
  int64_t bad = -1;
  int st = run_batched(c, words, {{(const uint8_t*)in24, 24}}, {{out16, 16}}, true, &bad,
                       [&](auto& din, auto& dout, size_t cnt, unsigned long long* ff,
                           const amph::LaunchCfg& lc) {
                         return amph::launch_b64_unwords((const char*)din[0], cnt, dout[0], ff, lc);
                       });
  if (bad_index) *bad_index = bad;
  if (st == AMPH_E_VERIFY)
    return fail(AMPH_E_PARAM, "Illegal base64 word record at index " + std::to_string(bad));
  return st;
}

// ---- Beaver open exchange codec ------------------------------------------------
size_t amph_exchange_max_chars(size_t npairs) { return amph::xenc_max_bytes(npairs); }

namespace {
// Host-pointer calls of the exchange codec: one shot on the context's first
// stream (the whole text is scanned at once, so there is no batching).
//
// Device-pointer calls take their scan scratch from one per-context buffer:
// under the context mutex each call makes its stream wait for the previous
// call's kernels (xdev_done) before reusing it, then records its own.  (The
// device's stream-ordered pool handed two contexts overlapping buffers in
// the host paths)
int dev_scratch(amph_ctx* c, size_t bytes, hipStream_t s, void** p) {
  if (!c->xdev_done) HIP_TRY(hipEventCreateWithFlags(&c->xdev_done, hipEventDisableTiming));
  else HIP_TRY(hipStreamWaitEvent(s, c->xdev_done, 0));
  if (c->xdev.cap < bytes) {
    HIP_TRY(hipEventSynchronize(c->xdev_done));  // the old buffer is idle before it is freed
    if (dev_ensure(c, c->xdev, bytes) != hipSuccess) return fail(AMPH_E_NOMEM, "exchange scratch");
  }
  *p = c->xdev.p;
  return AMPH_OK;
}

int host_stream0(amph_ctx* c, hipStream_t* s) {
  if (!c->streams[0]) HIP_TRY(hipStreamCreateWithFlags(&c->streams[0], hipStreamNonBlocking));
  *s = c->streams[0];
  return AMPH_OK;
}

// Host-mode buffers of the exchange codec calls: carved from one per-context
// device arena (grown with hipMalloc, held under the context mutex).  Two
// contexts on one device calling at the same time once got overlapping
// stream-ordered (hipMallocAsync) staging buffers: each party's exchange
// text came back empty or overwritten (tools/c1_native, two party threads).
struct XStage {
  uint8_t* base = nullptr;
  size_t off = 0;
  int stage(amph_ctx* c, const size_t* sizes, int n) {
    size_t total = 0;
    for (int i = 0; i < n; ++i) total += align256(sizes[i] ? sizes[i] : 16);
    hipError_t e = dev_ensure(c, c->xstage, total);
    if (e != hipSuccess) return fail(AMPH_E_NOMEM, "exchange staging");
    base = (uint8_t*)c->xstage.p;
    return AMPH_OK;
  }
  void* take(size_t bytes) {
    void* p = base + off;
    off += align256(bytes ? bytes : 16);
    return p;
  }
};
}  // namespace

int amph_exchange_encode(amph_ctx* c, const uint8_t* mag16, const uint8_t* neg, size_t npairs,
                         char* out, size_t out_cap, uint64_t* out_len, uint32_t flags,
                         void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_NO_HOST_IO(flags);
  if (!out || !out_len || (npairs && (!mag16 || !neg))) return fail(AMPH_E_PARAM, "null buffer");
  HIP_TRY(use_device(c->device));
  const size_t maxb = amph::xenc_max_bytes(npairs);
  if (flags & AMPH_F_DEVICE) {
    if (int st = check_dev_words({mag16})) return st;
    if (out_cap < maxb) return fail(AMPH_E_LEN, "output capacity below amph_exchange_max_chars(npairs)");
    hipStream_t s = (hipStream_t)stream;
    std::lock_guard<std::mutex> g(c->mu);
    void* scratch;
    if (int st = dev_scratch(c, amph::xenc_scratch_bytes(npairs), s, &scratch)) return st;
    hipError_t e = amph::launch_exchange_encode((const uint4*)mag16, neg, npairs, out,
                                                (unsigned long long*)out_len, scratch, cfg(c, s, npairs));
    if (e != hipSuccess) return hip_fail(e, "k_xenc");
    HIP_TRY(hipEventRecord(c->xdev_done, s));
    return AMPH_OK;
  }
  std::lock_guard<std::mutex> g(c->mu);
  if (npairs && small_call(c, align256(32 * npairs) + align256(2 * npairs) + align256(maxb))) {
    // small call: diffs in, text out through the page-locked arena, one sync
    hipStream_t s;
    if (int st = host_stream1(c, &s)) return st;
    Arena a;
    unsigned long long* dff;
    if (int st = small_begin(c, align256(32 * npairs) + align256(2 * npairs) + align256(maxb), s, &a, &dff))
      return st;
    XStage x;
    const size_t ssz[1] = {amph::xenc_scratch_bytes(npairs)};
    if (int st = x.stage(c, ssz, 1)) return st;
    uint8_t *hmag = a.take(32 * npairs), *hneg = a.take(2 * npairs), *htext = a.take(maxb);
    std::memcpy(hmag, mag16, 32 * npairs);
    std::memcpy(hneg, neg, 2 * npairs);
    unsigned long long* hlen = (unsigned long long*)c->small.p;  // the arena head
    hipError_t e = amph::launch_exchange_encode((const uint4*)hmag, hneg, npairs, (char*)htext, hlen,
                                                x.take(ssz[0]), cfg(c, s, npairs));
    if (e != hipSuccess) return small_launch_failed(c, s, e, "k_xenc");
    HIP_TRY(hipStreamSynchronize(s));
    const uint64_t len = *(volatile unsigned long long*)hlen;
    *out_len = len;
    if (len > out_cap) return fail(AMPH_E_LEN, "output capacity " + std::to_string(out_cap) +
                                                   " below the encoded length " + std::to_string(len));
    std::memcpy(out, htext, len);
    return AMPH_OK;
  }
  hipStream_t s;
  if (int st = host_stream0(c, &s)) return st;
  XStage x;
  const size_t sizes[5] = {32 * npairs, 2 * npairs, maxb, 8, amph::xenc_scratch_bytes(npairs)};
  if (int st = x.stage(c, sizes, 5)) return st;
  void *dmag = x.take(sizes[0]), *dneg = x.take(sizes[1]), *dout = x.take(sizes[2]), *dlen = x.take(sizes[3]),
       *scratch = x.take(sizes[4]);
  if (npairs) {
    HIP_TRY(hipMemcpy(dmag, mag16, 32 * npairs, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dneg, neg, 2 * npairs, hipMemcpyHostToDevice));
  }
  hipError_t e = amph::launch_exchange_encode((const uint4*)dmag, (const uint8_t*)dneg, npairs,
                                              (char*)dout, (unsigned long long*)dlen, scratch,
                                              cfg(c, s, npairs));
  if (e != hipSuccess) return hip_fail(e, "k_xenc");
  uint64_t len = 0;
  HIP_TRY(read_back(s, {{&len, dlen, 8}}));
  *out_len = len;
  if (len > out_cap) return fail(AMPH_E_LEN, "output capacity " + std::to_string(out_cap) +
                                                 " below the encoded length " + std::to_string(len));
  HIP_TRY(read_back(s, {{out, dout, len}}));
  return AMPH_OK;
}

int amph_exchange_decode(amph_ctx* c, const char* text, size_t len, size_t npairs, uint8_t* mag16,
                         uint8_t* neg, int64_t* bad_index, uint32_t flags, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_NO_HOST_IO(flags);
  if ((len && !text) || (npairs && (!mag16 || !neg))) return fail(AMPH_E_PARAM, "null buffer");
  HIP_TRY(use_device(c->device));
  if (flags & AMPH_F_DEVICE) {
    if (int st = check_dev_words({mag16})) return st;
    hipStream_t s = (hipStream_t)stream;
    if (int st = reset_ff_dev(bad_index, flags, s)) return st;
    std::lock_guard<std::mutex> g(c->mu);
    void* scratch;
    if (int st = dev_scratch(c, amph::xdec_scratch_bytes(len), s, &scratch)) return st;
    hipError_t e = amph::launch_exchange_decode(text, len, npairs, (uint4*)mag16, neg,
                                                (unsigned long long*)bad_index, scratch, cfg(c, s, len));
    if (e != hipSuccess) return hip_fail(e, "k_xdec");
    HIP_TRY(hipEventRecord(c->xdev_done, s));
    return AMPH_OK;
  }
  std::lock_guard<std::mutex> g(c->mu);
  const size_t sbytes = align256(len) + align256(32 * npairs) + align256(2 * npairs);
  if (len && small_call(c, sbytes)) {
    // small call: text in, diffs out through the page-locked arena, one sync
    hipStream_t s;
    if (int st = host_stream1(c, &s)) return st;
    Arena a;
    unsigned long long* dff;
    if (int st = small_begin(c, sbytes, s, &a, &dff)) return st;
    XStage x;
    const size_t ssz[1] = {amph::xdec_scratch_bytes(len)};
    if (int st = x.stage(c, ssz, 1)) return st;
    uint8_t *htext = a.take(len), *hmag = a.take(32 * npairs), *hneg = a.take(2 * npairs);
    std::memcpy(htext, text, len);
    hipError_t e = amph::launch_exchange_decode((const char*)htext, len, npairs, (uint4*)hmag, hneg, dff,
                                                x.take(ssz[0]), cfg(c, s, len));
    if (e != hipSuccess) return small_launch_failed(c, s, e, "k_xdec");
    if (int st = small_end(c, s, 1)) return st;
    const int64_t bad = (int64_t) * (volatile unsigned long long*)c->small.p;
    const bool ok = bad == (int64_t)AMPH_NO_FAILURE;
    if (bad_index) *bad_index = ok ? -1 : bad;
    if (!ok) {
      if ((size_t)bad == len)
        return fail(AMPH_E_LEN, "interimValues must hold exactly " + std::to_string(npairs) + " FactorPairs");
      return fail(AMPH_E_PARAM, "Malformed FactorPair JSON at offset " + std::to_string(bad));
    }
    std::memcpy(mag16, hmag, 32 * npairs);
    std::memcpy(neg, hneg, 2 * npairs);
    return AMPH_OK;
  }
  hipStream_t s;
  if (int st = host_stream0(c, &s)) return st;
  XStage x;
  const size_t sizes[5] = {len, 32 * npairs, 2 * npairs, 8, amph::xdec_scratch_bytes(len)};
  if (int st = x.stage(c, sizes, 5)) return st;
  void *dtext = x.take(sizes[0]), *dmag = x.take(sizes[1]), *dneg = x.take(sizes[2]), *dbad = x.take(sizes[3]),
       *scratch = x.take(sizes[4]);
  if (len) HIP_TRY(hipMemcpy(dtext, text, len, hipMemcpyHostToDevice));
  HIP_TRY(hipMemsetAsync(dbad, 0x7F, 8, s));
  hipError_t e = amph::launch_exchange_decode((const char*)dtext, len, npairs, (uint4*)dmag,
                                              (uint8_t*)dneg, (unsigned long long*)dbad, scratch,
                                              cfg(c, s, len));
  if (e != hipSuccess) return hip_fail(e, "k_xdec");
  int64_t bad = 0;
  HIP_TRY(read_back(s, {{&bad, dbad, 8}}));
  const bool ok = bad == (int64_t)AMPH_NO_FAILURE;
  if (bad_index) *bad_index = ok ? -1 : bad;
  if (!ok) {
    if ((size_t)bad == len)
      return fail(AMPH_E_LEN, "interimValues must hold exactly " + std::to_string(npairs) + " FactorPairs");
    return fail(AMPH_E_PARAM, "Malformed FactorPair JSON at offset " + std::to_string(bad));
  }
  HIP_TRY(read_back(s, {{mag16, dmag, 32 * npairs}, {neg, dneg, 2 * npairs}}));
  return AMPH_OK;
}

// ---- K_RV / K_MASK from the wire ----------------------------------------------
namespace {
const char* const kOdoFieldNames[5] = {"secretShares", "rShares", "vShares", "wShares", "uShares"};

const char* b64_field(const amph_odo_b64& o, int k) {
  switch (k) {
    case 0: return o.secret_shares;
    case 1: return o.r_shares;
    case 2: return o.v_shares;
    case 3: return o.w_shares;
    default: return o.u_shares;
  }
}

// Shared checks; *nchars / *pad for `words` 16-byte words.
int wire_check(const amph_odo_b64* odos, int n, size_t words, size_t* nchars, uint32_t* pad) {
  if (!odos || n < 1 || n > AMPH_MAX_PARTIES)
    return fail(AMPH_E_PARAM, "n_parties must be in [1, 16] with a non-null ODO array");
  const size_t nb = 16 * words;
  *nchars = 4 * ((nb + 2) / 3);
  *pad = (uint32_t)((3 - nb % 3) % 3);
  for (int j = 0; j < n; ++j) {
    if (odos[j].nchars != *nchars)
      return fail(AMPH_E_LEN, "party " + std::to_string(j) + ": base64 fields of " +
                                  std::to_string(odos[j].nchars) + " characters, expected " +
                                  std::to_string(*nchars) + " for " + std::to_string(words) + " words");
    for (int k = 0; k < 5 && words; ++k)
      if (!b64_field(odos[j], k)) return fail(AMPH_E_PARAM, "null ODO field text");
  }
  return AMPH_OK;
}

int wire_bad_message(int64_t bad, size_t nchars) {
  const size_t o = (size_t)bad / nchars, at = (size_t)bad % nchars;
  return fail(AMPH_E_PARAM, "Illegal base64 character at index " + std::to_string(at) + " of party " +
                                std::to_string(o / 5) + "'s " + kOdoFieldNames[o % 5]);
}

// Host mode, one launch per call (no batching).  Small calls (c->small_bytes)
// stage the texts in the page-locked arena, which the kernel reads in place,
// and make one stream synchronisation (run_small).  Larger ones copy each
// text with a blocking hipMemcpy into the context's device staging buffer
// (kPageableRule), run the kernel on the context's stream, and read the
// results back after it.  (A first version staged through stream-ordered
// hipMallocAsync memory with pageable hipMemcpyAsync; in a fresh process its
// first call intermittently saw the first text unit unwritten.)
struct WireHost {
  amph::TextSet tx{};
  uint8_t* base = nullptr;
  size_t off = 0;
  bool small = false;
  unsigned long long* fl = nullptr;  // first-fail, bad character
  uint8_t* take(size_t bytes) {
    uint8_t* p = base + off;
    off += align256(bytes ? bytes : 16);
    return p;
  }
  static size_t bytes_for(int n, size_t nchars, size_t extra) {
    return 5 * n * align256(nchars ? nchars : 16) + extra + 256;
  }
  int stage(amph_ctx* c, const amph_odo_b64* odos, int n, size_t nchars, size_t extra, hipStream_t s) {
    const size_t bytes = bytes_for(n, nchars, extra);
    small = small_call(c, bytes);
    if (small) {
      Arena a;
      if (int st = small_begin(c, bytes, s, &a, &fl)) return st;
      base = a.base;
      off = a.off;
    } else {
      hipError_t e = dev_ensure(c, c->wire, bytes);
      if (e != hipSuccess) return fail(AMPH_E_NOMEM, "wire staging");
      base = (uint8_t*)c->wire.p;
    }
    for (int j = 0; j < n; ++j)
      for (int k = 0; k < 5; ++k) {
        uint8_t* d = take(nchars);
        if (nchars) HIP_TRY(put(d, b64_field(odos[j], k), nchars));
        tx.t[k][j] = (const char*)d;
      }
    if (!small) {
      fl = (unsigned long long*)take(16);
      HIP_TRY(hipMemsetAsync(fl, 0x7F, 16, s));
    }
    return AMPH_OK;
  }
  hipError_t put(void* dst, const void* src, size_t bytes) {
    if (small) {
      std::memcpy(dst, src, bytes);
      return hipSuccess;
    }
    return hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice);
  }
  // after the launch: the two verdict words and the outputs to the caller
  int finish(amph_ctx* c, hipStream_t s, int64_t v[2], std::initializer_list<ReadBack> outs) {
    if (small) {
      if (int st = small_end(c, s, 2)) return st;
      std::memcpy(v, c->small.p, 16);
      for (const ReadBack& r : outs)
        if (r.bytes) std::memcpy(r.dst, r.src, r.bytes);
      return AMPH_OK;
    }
    HIP_TRY(read_back(s, {{v, fl, 16}}));
    for (const ReadBack& r : outs)
      if (r.bytes) HIP_TRY(hipMemcpy(r.dst, r.src, r.bytes, hipMemcpyDeviceToHost));
    return AMPH_OK;
  }
  int launch_failed(amph_ctx* c, hipStream_t s, hipError_t e, const char* what) {
    return small ? small_launch_failed(c, s, e, what) : hip_fail(e, what);
  }
};
}  // namespace

int amph_recombine_verify_b64(amph_ctx* c, const amph_odo_b64* odos, int n, size_t words,
                              uint8_t* out_secrets, int64_t* first_fail, int64_t* bad_char,
                              uint32_t flags, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_NO_HOST_IO(flags);
  size_t nchars;
  uint32_t pad;
  if (int st = wire_check(odos, n, words, &nchars, &pad)) return st;
  if (words && !out_secrets) return fail(AMPH_E_PARAM, "null output");
  HIP_TRY(use_device(c->device));
  if (flags & AMPH_F_DEVICE) {
    amph::TextSet tx{};
    for (int j = 0; j < n; ++j)
      for (int k = 0; k < 5; ++k) {
        tx.t[k][j] = b64_field(odos[j], k);
        if (int st = check_dev_words({tx.t[k][j]})) return st;
      }
    if (int st = check_dev_words({out_secrets})) return st;
    hipStream_t s = (hipStream_t)stream;
    if (int st = reset_ff_dev(first_fail, flags, s)) return st;
    if (int st = reset_ff_dev(bad_char, flags, s)) return st;
    hipError_t e = amph::launch_rv_b64(tx, n, words, nchars, pad, (uint4*)out_secrets,
                                       (unsigned long long*)first_fail, (unsigned long long*)bad_char,
                                       c->f, cfg(c, s, words));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_rv_b64");
  }
  if (first_fail) *first_fail = -1;
  if (bad_char) *bad_char = -1;
  if (words == 0) return AMPH_OK;
  std::lock_guard<std::mutex> g(c->mu);
  hipStream_t s;
  if (int st = host_stream0(c, &s)) return st;
  WireHost h;
  if (int st = h.stage(c, odos, n, nchars, align256(16 * words) + 256, s)) return st;
  uint8_t* dout = h.take(16 * words);
  hipError_t e = amph::launch_rv_b64(h.tx, n, words, nchars, pad, (uint4*)dout, h.fl, h.fl + 1, c->f,
                                     cfg(c, s, words));
  if (e != hipSuccess) return h.launch_failed(c, s, e, "k_rv_b64");
  int64_t v[2];
  if (int st = h.finish(c, s, v, {{out_secrets, dout, 16 * words}})) return st;
  if (v[1] != (int64_t)AMPH_NO_FAILURE) {
    if (bad_char) *bad_char = v[1];
    return wire_bad_message(v[1], nchars);
  }
  if (v[0] != (int64_t)AMPH_NO_FAILURE) {
    if (first_fail) *first_fail = v[0];
    return AMPH_E_VERIFY;
  }
  return AMPH_OK;
}

int amph_mask_input_b64(amph_ctx* c, const amph_odo_b64* odos, int n, size_t words,
                        const uint8_t* secrets, size_t n_secrets, uint8_t* out16, char* out24,
                        int64_t* first_fail, int64_t* bad_char, uint32_t flags, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  AMPH_NO_HOST_IO(flags);
  size_t nchars;
  uint32_t pad;
  if (int st = wire_check(odos, n, words, &nchars, &pad)) return st;
  if (n_secrets > words) {
    // as amph_mask_input: the texts decode and every mask verifies before the
    // length error (DefaultAmphoraClient.java:153 before :160)
    int st = amph_mask_input_b64(c, odos, n, words, nullptr, 0, nullptr, nullptr, first_fail, bad_char,
                                 flags, stream);
    if (st != AMPH_OK) return st;
    if (flags & AMPH_F_DEVICE) {
      HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
      int64_t v[2] = {(int64_t)AMPH_NO_FAILURE, (int64_t)AMPH_NO_FAILURE};
      if (first_fail) HIP_TRY(hipMemcpy(&v[0], first_fail, 8, hipMemcpyDeviceToHost));  // kPageableRule
      if (bad_char) HIP_TRY(hipMemcpy(&v[1], bad_char, 8, hipMemcpyDeviceToHost));
      if (v[1] != (int64_t)AMPH_NO_FAILURE) return wire_bad_message(v[1], nchars);
      if (v[0] != (int64_t)AMPH_NO_FAILURE)
        return fail(AMPH_E_VERIFY, "input mask MAC check failed at word " + std::to_string(v[0]));
    }
    return fail(AMPH_E_LEN, "more secret words than verified input masks");
  }
  if (n_secrets && !secrets) return fail(AMPH_E_PARAM, "null secrets");
  HIP_TRY(use_device(c->device));
  if (flags & AMPH_F_DEVICE) {
    amph::TextSet tx{};
    for (int j = 0; j < n; ++j)
      for (int k = 0; k < 5; ++k) {
        tx.t[k][j] = b64_field(odos[j], k);
        if (int st = check_dev_words({tx.t[k][j]})) return st;
      }
    if (int st = check_dev_words({secrets, out16, out24})) return st;
    hipStream_t s = (hipStream_t)stream;
    if (int st = reset_ff_dev(first_fail, flags, s)) return st;
    if (int st = reset_ff_dev(bad_char, flags, s)) return st;
    hipError_t e = amph::launch_mask_b64(tx, n, words, nchars, pad, (const uint4*)secrets, n_secrets,
                                         (uint4*)out16, out24, (unsigned long long*)first_fail,
                                         (unsigned long long*)bad_char, c->f, cfg(c, s, words));
    return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_mask_b64");
  }
  if (first_fail) *first_fail = -1;
  if (bad_char) *bad_char = -1;
  if (words == 0) return AMPH_OK;
  std::lock_guard<std::mutex> g(c->mu);
  hipStream_t s;
  if (int st = host_stream0(c, &s)) return st;
  WireHost h;
  const size_t extra = 3 * align256(16 * n_secrets) + align256(24 * n_secrets) + 1024;
  if (int st = h.stage(c, odos, n, nchars, extra, s)) return st;
  uint8_t* dsec = h.take(16 * n_secrets);
  uint8_t* d16 = h.take(16 * n_secrets);
  uint8_t* d24 = h.take(24 * n_secrets);
  if (n_secrets) HIP_TRY(h.put(dsec, secrets, 16 * n_secrets));
  hipError_t e = amph::launch_mask_b64(h.tx, n, words, nchars, pad, (const uint4*)dsec, n_secrets,
                                       out16 ? (uint4*)d16 : nullptr, out24 ? (char*)d24 : nullptr,
                                       h.fl, h.fl + 1, c->f, cfg(c, s, words));
  if (e != hipSuccess) return h.launch_failed(c, s, e, "k_mask_b64");
  int64_t v[2];
  if (int st = h.finish(c, s, v, {{out16, d16, out16 ? 16 * n_secrets : 0},
                                  {out24, d24, out24 ? 24 * n_secrets : 0}}))
    return st;
  if (v[1] != (int64_t)AMPH_NO_FAILURE) {
    if (bad_char) *bad_char = v[1];
    return wire_bad_message(v[1], nchars);
  }
  if (v[0] != (int64_t)AMPH_NO_FAILURE) {
    if (first_fail) *first_fail = v[0];
    return AMPH_E_VERIFY;
  }
  return AMPH_OK;
}

int amph_host_register(amph_ctx* c, void* ptr, size_t bytes) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  if (!ptr || !bytes) return fail(AMPH_E_PARAM, "null or empty range");
  HIP_TRY(use_device(c->device));
  HIP_TRY(hipHostRegister(ptr, bytes, hipHostRegisterPortable));
  return AMPH_OK;
}

int amph_host_unregister(amph_ctx* c, void* ptr) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  if (!ptr) return fail(AMPH_E_PARAM, "null pointer");
  HIP_TRY(use_device(c->device));
  HIP_TRY(hipHostUnregister(ptr));
  return AMPH_OK;
}

int amph_synth_odos(amph_ctx* c, uint64_t seed, int n, size_t words, uint8_t* const* out_fields,
                    uint8_t* out_plain_y, int64_t fault_index, int noncanon_permille,
                    void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  if (!out_fields || n < 1 || n > AMPH_MAX_PARTIES) return fail(AMPH_E_PARAM, "n_parties must be in [1, 16]");
  amph::OutSet set{};
  for (int k = 0; k < 5; ++k)
    for (int j = 0; j < n; ++j) {
      if (words && !out_fields[k * n + j]) return fail(AMPH_E_PARAM, "null output field");
      set.f[k][j] = (uint4*)out_fields[k * n + j];
    }
  HIP_TRY(use_device(c->device));
  hipError_t e = amph::launch_synth_odos(set, n, words, seed, (uint4*)out_plain_y, fault_index,
                                         noncanon_permille, c->f, cfg(c, (hipStream_t)stream, words));
  return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_synth");
}

int amph_stream_probe(amph_ctx* c, const amph_odo* odos, int n, const uint8_t* secrets, size_t words,
                      uint8_t* out, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  size_t W;
  if (int st = odo_words(odos, n, &W)) return st;
  if (words > W) return fail(AMPH_E_LEN, "more words than the ODO arrays hold");
  if (words && (!secrets || !out)) return fail(AMPH_E_PARAM, "null secrets/output");
  if (int st = check_dev_odos(odos, n)) return st;
  if (int st = check_dev_words({secrets, out})) return st;
  HIP_TRY(use_device(c->device));
  amph::OdoSet set{};
  for (int k = 0; k < 5; ++k)
    for (int j = 0; j < n; ++j) set.f[k][j] = (const uint4*)odo_field(odos[j], k);
  hipError_t e = amph::launch_stream_probe(set, n, words, (const uint4*)secrets, (uint4*)out,
                                           cfg(c, (hipStream_t)stream, words));
  return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_stream_probe");
}

int amph_synth_words(amph_ctx* c, uint64_t seed, size_t count, uint8_t* out, void* stream) {
  if (check_ctx(c)) return AMPH_E_PARAM;
  if (count && !out) return fail(AMPH_E_PARAM, "null output");
  HIP_TRY(use_device(c->device));
  hipError_t e = amph::launch_synth_words((uint4*)out, count, seed, c->f, cfg(c, (hipStream_t)stream, count));
  return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_synth_words");
}

}  // extern "C"

// ---- one party's Output Delivery, device-resident between steps ----------------
// (include/amphora.h, "one party's Output Delivery with device-resident state")
// Device memory: one allocation carved into the triples (host mode), the five
// ODO fields, this party's diffs, its text and the encoder's scratch; the share
// data and masks live in a second one released once begin has run; each
// partner's diffs (the exchange decode's span form, amph::XSpans) and its
// decode scratch in one allocation per slot, sized by its text; partner texts
// and the base64 output staged in a fourth (host mode).  Host mode: every copy
// is a blocking hipMemcpy issued with the context's stream idle
// (kPageableRule), so caller buffers may be pageable or page-locked.  Device
// mode (amph_party_*_dev): nothing is copied; the caller's buffers are used in
// place and every launch goes on the caller's stream.
struct amph_party {
  amph_ctx* c = nullptr;
  size_t W = 0;
  int n = 0;
  bool dev = false;               // device mode
  hipStream_t dstream = nullptr;  // device mode: the stream of the latest call
  DevBuf mem, tmp, io;
  const uint4* triples = nullptr;
  uint4* f5[5] = {};  // y, r, v, w, u
  char* b64[5] = {};  // the five fields as base64 text (finish_b64)
  uint4* mag[AMPH_MAX_PARTIES] = {};
  uint8_t* neg[AMPH_MAX_PARTIES] = {};
  DevBuf pbuf[AMPH_MAX_PARTIES];
  amph::XSpans xs[AMPH_MAX_PARTIES] = {};
  char* text = nullptr;
  unsigned long long* text_len_dev = nullptr;
  void* enc_scratch = nullptr;
  uint64_t* enc_lens = nullptr;  // K_ODO_PRE's exchange text lengths, scanned by the encode
  uint64_t text_len = 0;
  uint32_t have = 0;  // bit j: party j's diffs are on the device (bit 0 after begin)
  const unsigned long long* bad_dev[AMPH_MAX_PARTIES] = {};  // device mode: partner verdict words
  // device mode: the session's own copies of the partner verdicts, and per
  // slot an event after the partner call's work (finish may use another stream)
  DevBuf verdicts;
  hipEvent_t partner_ev[AMPH_MAX_PARTIES] = {};
  bool finished = false;
  ~amph_party() {
    mem.release();
    tmp.release();
    io.release();
    verdicts.release();
    for (DevBuf& b : pbuf) b.release();
    for (hipEvent_t& e : partner_ev)
      if (e) (void)hipEventDestroy(e);
  }
};

namespace {
size_t b64_chars(size_t nbytes) { return 4 * ((nbytes + 2) / 3); }

constexpr size_t kPartyPoolMax = 16;

// (c->mu held) hand a session buffer back to the context's pool: at most
// kPartyPoolMax buffers and c->pool_cap_bytes bytes, the smallest dropped first
void pool_put(amph_ctx* c, DevBuf& b) {
  if (!b.p) return;
  c->party_pool.push_back(b);
  b.p = nullptr;
  b.cap = 0;
  while (!c->party_pool.empty() &&
         (c->party_pool.size() > kPartyPoolMax || pool_bytes(c) > c->pool_cap_bytes)) {
    size_t m = 0;
    for (size_t i = 1; i < c->party_pool.size(); ++i)
      if (c->party_pool[i].cap < c->party_pool[m].cap) m = i;
    c->party_pool[m].release();
    c->party_pool.erase(c->party_pool.begin() + (long)m);
  }
}

// (c->mu held) b holds at least `bytes`: kept, or the best-fitting pooled
// buffer, or a new allocation (after freeing the pool if memory ran out)
hipError_t pool_ensure(amph_ctx* c, DevBuf& b, size_t bytes) {
  if (bytes <= b.cap) return hipSuccess;
  pool_put(c, b);
  long best = -1;
  for (size_t i = 0; i < c->party_pool.size(); ++i)
    if (c->party_pool[i].cap >= bytes && (best < 0 || c->party_pool[i].cap < c->party_pool[(size_t)best].cap))
      best = (long)i;
  if (best >= 0) {
    b = c->party_pool[(size_t)best];
    c->party_pool.erase(c->party_pool.begin() + best);
    return hipSuccess;
  }
  return dev_ensure(c, b, bytes);
}

int party_check(amph_party* p) {
  if (!p || !p->c) return fail(AMPH_E_PARAM, "null party session");
  if (p->finished) return fail(AMPH_E_PARAM, "the party session is already finished");
  return AMPH_OK;
}

int party_args(amph_ctx* c, size_t share_stride, int n_parties, size_t words, const void* share_data,
               const void* masks, const void* triples, amph_party** out) {
  if (!out) return fail(AMPH_E_PARAM, "null session output");
  *out = nullptr;
  if (check_ctx(c)) return AMPH_E_PARAM;
  if (share_stride != 16 && share_stride != 32) return fail(AMPH_E_PARAM, "share_stride must be 16 or 32");
  if (n_parties < 1 || n_parties > AMPH_MAX_PARTIES) return fail(AMPH_E_PARAM, "n_parties must be in [1, 16]");
  if (words && (!share_data || !masks || !triples)) return fail(AMPH_E_PARAM, "null buffer");
  return AMPH_OK;
}

// the session's device memory; yrv[k] non-null: field k lives in the caller's
// device buffer (device mode), else in the session's
int party_alloc(amph_party* p, bool copy_triples, uint8_t* const yrv[3]) {
  const size_t W = p->W, P = 2 * W, nc = b64_chars(16 * W);
  const size_t nl = (P + amph::kXLenPairs - 1) / amph::kXLenPairs;
  const size_t sz[] = {copy_triples ? 192 * W : 0, 16 * W, 16 * W, 16 * W, 16 * W, 16 * W,
                       amph::xenc_max_bytes(P), 8, amph::xenc_lens_scratch_bytes(P), 64 * W, 4 * W, nc, nc, nc, nc, nc,
                       8 * (nl + 1)};
  size_t total = 0;
  for (size_t b : sz) total += align256(b ? b : 16);
  if (pool_ensure(p->c, p->mem, total) != hipSuccess) return fail(AMPH_E_NOMEM, "party session device memory");
  uint8_t* cur = (uint8_t*)p->mem.p;
  auto take = [&](size_t b) {
    uint8_t* q = cur;
    cur += align256(b ? b : 16);
    return q;
  };
  p->triples = (const uint4*)take(sz[0]);
  for (int k = 0; k < 5; ++k) {
    uint4* own = (uint4*)take(sz[1 + k]);
    p->f5[k] = k < 3 && yrv[k] ? (uint4*)yrv[k] : own;
  }
  p->text = (char*)take(sz[6]);
  p->text_len_dev = (unsigned long long*)take(sz[7]);
  p->enc_scratch = take(sz[8]);
  p->mag[0] = (uint4*)take(sz[9]);
  p->neg[0] = take(sz[10]);
  for (int k = 0; k < 5; ++k) p->b64[k] = (char*)take(sz[11 + k]);
  p->enc_lens = (uint64_t*)take(sz[16]);
  return AMPH_OK;
}

// k_odo_pre (y, r, v + this party's diffs and their exchange text lengths)
// and the exchange encode of the diffs
int party_pre(amph_party* p, const uint8_t* dshare, size_t share_stride, const uint8_t* dmasks, hipStream_t s) {
  amph_ctx* c = p->c;
  const size_t W = p->W, P = 2 * W;
  hipError_t e = amph::launch_odo_pre((const uint4*)dshare, (int)(share_stride / 16), (const uint4*)dmasks,
                                      p->triples, W, p->f5[0], p->f5[1], p->f5[2], p->mag[0], (uint32_t*)p->neg[0],
                                      c->f, cfg(c, s, W), p->enc_lens);
  if (e != hipSuccess) return hip_fail(e, "k_odo_pre");
  e = amph::launch_exchange_encode_lens(p->mag[0], p->neg[0], P, p->enc_lens, p->text, p->text_len_dev,
                                        p->enc_scratch, cfg(c, s, P));
  return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_xenc");
}

int party_slot_check(amph_party* p, int slot, const char* text, size_t len) {
  if (int st = party_check(p)) return st;
  if (slot < 1 || slot >= p->n)
    return fail(AMPH_E_PARAM, "partner slot must be in [1, " + std::to_string(p->n - 1) + "]");
  if (p->have >> slot & 1u) return fail(AMPH_E_PARAM, "partner slot " + std::to_string(slot) + " already holds a text");
  if (len && !text) return fail(AMPH_E_PARAM, "null text");
  return AMPH_OK;
}

// a partner's text (device memory) decoded into the slot's span form; bad:
// the device word the decode reports into (reset by its first kernel)
int party_decode(amph_party* p, int slot, const char* dtext, size_t len, unsigned long long* bad, hipStream_t s) {
  const size_t P = 2 * p->W;
  const size_t nb = amph::xspan_spans(len), slots = amph::xspan_slots(len, P);
  const size_t xsz[5] = {16 * slots, slots, 8 * (nb + 1), 16 * amph::xspan_map_words(P),
                         amph::xdec_spans_scratch_bytes(len)};
  size_t xtotal = 0;
  for (size_t b : xsz) xtotal += align256(b);
  if (pool_ensure(p->c, p->pbuf[slot], xtotal) != hipSuccess)
    return fail(AMPH_E_NOMEM, "party session partner diffs");
  uint8_t* xp = (uint8_t*)p->pbuf[slot].p;
  amph::XSpans& xs = p->xs[slot];
  xs.mag = (uint4*)xp;
  xs.neg = xp + align256(xsz[0]);
  xs.base = (uint64_t*)(xs.neg + align256(xsz[1]));
  xs.map = (uint4*)((uint8_t*)xs.base + align256(xsz[2]));
  void* scratch = (uint8_t*)xs.map + align256(xsz[3]);
  xs.nb = nb;
  p->mag[slot] = xs.mag;
  p->neg[slot] = xs.neg;
  hipError_t e = amph::launch_exchange_decode_spans(dtext, len, P, xs, bad, scratch, cfg(p->c, s, len));
  return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_xdec");
}

int decode_status(int64_t bad, size_t len, size_t P, int64_t* bad_index) {
  if (bad == (int64_t)AMPH_NO_FAILURE) return AMPH_OK;
  if (bad_index) *bad_index = bad;
  if ((size_t)bad == len)
    return fail(AMPH_E_LEN, "interimValues must hold exactly " + std::to_string(P) + " FactorPairs");
  return fail(AMPH_E_PARAM, "Malformed FactorPair JSON at offset " + std::to_string(bad));
}

int party_all_in(amph_party* p) {
  const uint32_t all = p->n >= 32 ? ~0u : ((1u << p->n) - 1u);
  if ((p->have & all) == all) return AMPH_OK;
  int j = 1;
  while (j < p->n && (p->have >> j & 1u)) ++j;
  return fail(AMPH_E_PARAM, "partner slot " + std::to_string(j) + "'s interimValues text is missing");
}

// the summed diffs -> w, u on the device (every partner's text must be in)
int party_open_post(amph_party* p, int is_player0, hipStream_t s) {
  if (int st = party_all_in(p)) return st;
  amph::SignedSet set{};
  for (int j = 0; j < p->n; ++j) {
    set.mag[j] = p->mag[j];
    set.neg[j] = (const uint32_t*)p->neg[j];
    if (j > 0) {
      set.sbase[j] = p->xs[j].base;
      set.smap[j] = p->xs[j].map;
      set.snb[j] = p->xs[j].nb;
    }
  }
  hipError_t e = amph::launch_open_post(set, p->n, p->triples, p->W, is_player0, p->f5[3], p->f5[4], p->c->f,
                                        cfg(p->c, s, p->W));
  return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_open_post");
}

// the five fields as base64 text in the session's memory (one launch)
int party_b64(amph_party* p, hipStream_t s) {
  const size_t nb = 16 * p->W;
  const uint8_t* const in[5] = {(const uint8_t*)p->f5[0], (const uint8_t*)p->f5[1], (const uint8_t*)p->f5[2],
                                (const uint8_t*)p->f5[3], (const uint8_t*)p->f5[4]};
  hipError_t e = amph::launch_b64_encode_multi(in, p->b64, 5, nb, cfg(p->c, s, (nb + 11) / 12));
  return e == hipSuccess ? AMPH_OK : hip_fail(e, "k_b64_encode_multi");
}

int party_mode(amph_party* p, bool dev) {
  if (p->dev != dev)
    return fail(AMPH_E_PARAM, dev ? "a host-mode party session takes the host calls"
                                  : "a device-mode party session takes the *_dev calls");
  return AMPH_OK;
}
}  // namespace

extern "C" {

int amph_party_begin(amph_ctx* c, const uint8_t* share_data, size_t share_stride, const uint8_t* masks,
                     const uint8_t* triples, size_t words, int n_parties, uint8_t* oy, uint8_t* orr,
                     uint8_t* ov, amph_party** out) {
  if (int st = party_args(c, share_stride, n_parties, words, share_data, masks, triples, out)) return st;
  if (!c->sub.empty()) c = c->sub[0];  // a multi-device context runs sessions on its first device
  HIP_TRY(use_device(c->device));
  std::lock_guard<std::mutex> g(c->mu);
  std::unique_ptr<amph_party> p(new amph_party);
  p->c = c;
  p->W = words;
  p->n = n_parties;
  const size_t W = words;
  uint8_t* const none[3] = {nullptr, nullptr, nullptr};
  if (int st = party_alloc(p.get(), true, none)) return st;
  if (pool_ensure(c, p->tmp, align256(share_stride * W + 16) + align256(64 * W + 16)) != hipSuccess)
    return fail(AMPH_E_NOMEM, "party session staging");
  uint8_t* dshare = (uint8_t*)p->tmp.p;
  uint8_t* dmasks = dshare + align256(share_stride * W + 16);
  hipStream_t s;
  if (int st = host_stream0(c, &s)) return st;
  HIP_TRY(hipStreamSynchronize(s));
  if (W) {
    HIP_TRY(hipMemcpy(dshare, share_data, share_stride * W, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dmasks, masks, 64 * W, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy((void*)p->triples, triples, 192 * W, hipMemcpyHostToDevice));
  }
  if (int st = party_pre(p.get(), dshare, share_stride, dmasks, s)) return st;
  uint64_t len = 0;
  HIP_TRY(read_back(s, {{&len, p->text_len_dev, 8}, {oy, p->f5[0], oy ? 16 * W : 0},
                        {orr, p->f5[1], orr ? 16 * W : 0}, {ov, p->f5[2], ov ? 16 * W : 0}}));
  p->text_len = len;
  p->have = 1u;
  pool_put(c, p->tmp);
  *out = p.release();
  return AMPH_OK;
}

size_t amph_party_words(const amph_party* p) { return p ? p->W : 0; }

uint64_t amph_party_text_len(const amph_party* p) { return p && !p->dev ? p->text_len : 0; }

int amph_party_text(amph_party* p, char* out, size_t out_cap) {
  if (!p || !p->c) return fail(AMPH_E_PARAM, "null party session");
  if (int st = party_mode(p, false)) return st;
  if (!out && p->text_len) return fail(AMPH_E_PARAM, "null output");
  if (out_cap < p->text_len)
    return fail(AMPH_E_LEN, "output capacity " + std::to_string(out_cap) + " below the text length " +
                                std::to_string(p->text_len));
  amph_ctx* c = p->c;
  HIP_TRY(use_device(c->device));
  std::lock_guard<std::mutex> g(c->mu);
  hipStream_t s;
  if (int st = host_stream0(c, &s)) return st;
  HIP_TRY(read_back(s, {{out, p->text, p->text_len}}));
  return AMPH_OK;
}

int amph_party_partner(amph_party* p, int slot, const char* text, size_t len, int64_t* bad_index) {
  if (bad_index) *bad_index = -1;
  if (int st = party_slot_check(p, slot, text, len)) return st;
  if (int st = party_mode(p, false)) return st;
  amph_ctx* c = p->c;
  HIP_TRY(use_device(c->device));
  std::lock_guard<std::mutex> g(c->mu);
  if (pool_ensure(c, p->io, align256(len + 16) + 256) != hipSuccess)
    return fail(AMPH_E_NOMEM, "party session text staging");
  uint8_t* dtext = (uint8_t*)p->io.p;
  unsigned long long* dbad = (unsigned long long*)(dtext + align256(len + 16));
  hipStream_t s;
  if (int st = host_stream0(c, &s)) return st;
  HIP_TRY(hipStreamSynchronize(s));
  if (len) HIP_TRY(hipMemcpy(dtext, text, len, hipMemcpyHostToDevice));
  if (int st = party_decode(p, slot, (const char*)dtext, len, dbad, s)) return st;
  int64_t bad = 0;
  HIP_TRY(read_back(s, {{&bad, dbad, 8}}));
  if (int st = decode_status(bad, len, 2 * p->W, bad_index)) return st;
  p->have |= 1u << slot;
  return AMPH_OK;
}

int amph_party_finish(amph_party* p, int is_player0, uint8_t* ow, uint8_t* ou) {
  if (int st = party_check(p)) return st;
  if (int st = party_mode(p, false)) return st;
  if (p->W && (!ow || !ou)) return fail(AMPH_E_PARAM, "null output");
  amph_ctx* c = p->c;
  HIP_TRY(use_device(c->device));
  std::lock_guard<std::mutex> g(c->mu);
  hipStream_t s;
  if (int st = host_stream0(c, &s)) return st;
  if (int st = party_open_post(p, is_player0, s)) return st;
  HIP_TRY(read_back(s, {{ow, p->f5[3], 16 * p->W}, {ou, p->f5[4], 16 * p->W}}));
  p->finished = true;
  return AMPH_OK;
}

int amph_party_finish_b64(amph_party* p, int is_player0, char* const fields_b64[5]) {
  if (int st = party_check(p)) return st;
  if (int st = party_mode(p, false)) return st;
  if (!fields_b64) return fail(AMPH_E_PARAM, "null field array");
  for (int k = 0; k < 5; ++k)
    if (p->W && !fields_b64[k]) return fail(AMPH_E_PARAM, "null field text");
  amph_ctx* c = p->c;
  HIP_TRY(use_device(c->device));
  std::lock_guard<std::mutex> g(c->mu);
  const size_t nc = b64_chars(16 * p->W);
  hipStream_t s;
  if (int st = host_stream0(c, &s)) return st;
  if (int st = party_open_post(p, is_player0, s)) return st;
  if (int st = party_b64(p, s)) return st;
  char** d = p->b64;
  HIP_TRY(read_back(s, {{fields_b64[0], d[0], nc}, {fields_b64[1], d[1], nc}, {fields_b64[2], d[2], nc},
                        {fields_b64[3], d[3], nc}, {fields_b64[4], d[4], nc}}));
  p->finished = true;
  return AMPH_OK;
}

// ---- device mode ------------------------------------------------------------------
int amph_party_begin_dev(amph_ctx* c, const uint8_t* share_data, size_t share_stride, const uint8_t* masks,
                         const uint8_t* triples, size_t words, int n_parties, uint8_t* oy, uint8_t* orr,
                         uint8_t* ov, void* stream, amph_party** out) {
  if (int st = party_args(c, share_stride, n_parties, words, share_data, masks, triples, out)) return st;
  if (!c->sub.empty()) return fail(AMPH_E_PARAM, "device-mode sessions need a single-device context");
  if (int st = check_dev_words({share_data, masks, triples, oy, orr, ov})) return st;
  HIP_TRY(use_device(c->device));
  std::lock_guard<std::mutex> g(c->mu);
  std::unique_ptr<amph_party> p(new amph_party);
  p->c = c;
  p->W = words;
  p->n = n_parties;
  p->dev = true;
  p->dstream = (hipStream_t)stream;
  uint8_t* const yrv[3] = {oy, orr, ov};
  if (int st = party_alloc(p.get(), false, yrv)) return st;
  p->triples = (const uint4*)triples;
  if (int st = party_pre(p.get(), share_data, share_stride, masks, p->dstream)) return st;
  p->have = 1u;
  *out = p.release();
  return AMPH_OK;
}

int amph_party_text_dev(amph_party* p, const char** text, const uint64_t** len) {
  if (!p || !p->c) return fail(AMPH_E_PARAM, "null party session");
  if (int st = party_mode(p, true)) return st;
  if (!text || !len) return fail(AMPH_E_PARAM, "null output");
  *text = p->text;
  *len = (const uint64_t*)p->text_len_dev;
  return AMPH_OK;
}

int amph_party_partner_dev(amph_party* p, int slot, const char* text, size_t len, int64_t* bad_index,
                           void* stream) {
  if (int st = party_slot_check(p, slot, text, len)) return st;
  if (int st = party_mode(p, true)) return st;
  if (!bad_index || ((uintptr_t)bad_index & 7)) return fail(AMPH_E_PARAM, "bad_index must be an 8-byte aligned device word");
  amph_ctx* c = p->c;
  HIP_TRY(use_device(c->device));
  std::lock_guard<std::mutex> g(c->mu);
  p->dstream = (hipStream_t)stream;
  if (dev_ensure(c, p->verdicts, sizeof(unsigned long long) * AMPH_MAX_PARTIES) != hipSuccess)
    return fail(AMPH_E_NOMEM, "partner verdict words");
  if (!p->partner_ev[slot]) HIP_TRY(hipEventCreateWithFlags(&p->partner_ev[slot], hipEventDisableTiming));
  if (int st = party_decode(p, slot, text, len, (unsigned long long*)bad_index, p->dstream)) return st;
  // the session's copy of the verdict: the caller's word may be reused once
  // the stream has passed this call
  unsigned long long* mine = (unsigned long long*)p->verdicts.p + slot;
  HIP_TRY(hipMemcpyAsync(mine, bad_index, sizeof(unsigned long long), hipMemcpyDeviceToDevice, p->dstream));
  HIP_TRY(hipEventRecord(p->partner_ev[slot], p->dstream));
  p->have |= 1u << slot;
  p->bad_dev[slot] = mine;
  return AMPH_OK;
}

int amph_party_reset_partner(amph_party* p, int slot) {
  if (int st = party_check(p)) return st;
  if (slot < 1 || slot >= p->n)
    return fail(AMPH_E_PARAM, "partner slot must be in [1, " + std::to_string(p->n - 1) + "]");
  std::lock_guard<std::mutex> g(p->c->mu);
  p->have &= ~(1u << slot);
  p->bad_dev[slot] = nullptr;
  return AMPH_OK;
}

int amph_party_finish_b64_dev(amph_party* p, int is_player0, const char* fields_b64[5], void* stream) {
  if (int st = party_check(p)) return st;
  if (int st = party_mode(p, true)) return st;
  if (!fields_b64) return fail(AMPH_E_PARAM, "null field array");
  amph_ctx* c = p->c;
  HIP_TRY(use_device(c->device));
  std::lock_guard<std::mutex> g(c->mu);
  p->dstream = (hipStream_t)stream;
  // every accepted partner call's decode and verdict copy, whatever its stream
  for (int j = 1; j < p->n; ++j)
    if (p->bad_dev[j] && p->partner_ev[j]) HIP_TRY(hipStreamWaitEvent(p->dstream, p->partner_ev[j], 0));
  if (int st = party_open_post(p, is_player0, p->dstream)) return st;
  if (int st = party_b64(p, p->dstream)) return st;
  amph::PoisonB64 pz{};
  for (int j = 1; j < p->n; ++j)
    if (p->bad_dev[j]) pz.bad[pz.n_bad++] = p->bad_dev[j];
  for (int k = 0; k < 5; ++k) pz.field[k] = p->b64[k];
  pz.chars = b64_chars(16 * p->W);
  if (hipError_t e = amph::launch_poison_b64(pz, p->dstream)) return hip_fail(e, "k_poison_b64");
  for (int k = 0; k < 5; ++k) fields_b64[k] = p->b64[k];
  p->finished = true;
  return AMPH_OK;
}

void amph_party_free(amph_party* p) {
  if (!p) return;
  if (p->c) {
    (void)use_device(p->c->device);
    std::lock_guard<std::mutex> g(p->c->mu);
    if (p->dev) (void)hipStreamSynchronize(p->dstream);
    else if (p->c->streams[0]) (void)hipStreamSynchronize(p->c->streams[0]);
    // the buffers go back to the context for the next session
    for (DevBuf* b : {&p->mem, &p->tmp, &p->io}) pool_put(p->c, *b);
    for (DevBuf& b : p->pbuf) pool_put(p->c, b);
  }
  delete p;
}

}  // extern "C"

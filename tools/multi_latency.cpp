// Per-call latency of host-pointer calls on a multi-device context
// (amph_ctx_create_multi), for VERDICT r3 item 3: run_sharded's per-call
// std::thread fan-out vs the sub-contexts' long-lived DeviceWorkers.
//
//   multi_latency LIB.so WORDS CALLS DEV[,DEV...]
//
// dlopen()s the given build of libamphora_hip (so two builds can be timed in
// one process run each), creates one context over the listed devices (one GPU
// named three times on a one-GPU box), makes CALLS host calls of
// amph_recombine_verify on WORDS words x 2 parties (honest ODOs are not
// needed: the call does all its work whatever the verdict) and prints one
// JSON line with the median / p10 / p90 per-call microseconds.
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "amphora.h"

typedef int (*create_multi_t)(const uint8_t*, const uint8_t*, const uint8_t*, const int*, int, amph_ctx**);
typedef void (*destroy_t)(amph_ctx*);
typedef int (*rv_t)(amph_ctx*, const amph_odo*, int, uint8_t*, int64_t*, uint32_t, void*);

static void le16(const char* hex_be, uint8_t out[16]) {  // big-endian hex -> LE16
  for (int i = 0; i < 16; ++i) {
    unsigned v;
    std::sscanf(hex_be + 2 * (15 - i), "%2x", &v);
    out[i] = (uint8_t)v;
  }
}

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: %s LIB.so WORDS CALLS DEV[,DEV...]\n", argv[0]);
    return 2;
  }
  void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    std::fprintf(stderr, "dlopen: %s\n", dlerror());
    return 2;
  }
  auto create = (create_multi_t)dlsym(h, "amph_ctx_create_multi");
  auto destroy = (destroy_t)dlsym(h, "amph_ctx_destroy");
  auto rv = (rv_t)dlsym(h, "amph_recombine_verify");
  const size_t W = std::strtoull(argv[2], nullptr, 10);
  const int calls = std::atoi(argv[3]);
  std::vector<int> devs;
  for (const char* p = argv[4]; *p;) {
    devs.push_back(std::atoi(p));
    while (*p && *p != ',') ++p;
    if (*p == ',') ++p;
  }
  uint8_t p[16], r[16], ri[16];
  le16("958907458f2136861bd7554a24340001", p);
  // r = 2^128 mod p, rInv = r^-1 mod p (the reference's test field)
  le16("6a76f8ba70dec979e428aab5dbcbffff", r);
  le16("64b363aaebadc239c970b543e5633b46", ri);
  amph_ctx* ctx = nullptr;
  if (int st = create(p, r, ri, devs.data(), (int)devs.size(), &ctx)) {
    std::fprintf(stderr, "create: %d\n", st);
    return 1;
  }
  const int n = 2;
  std::mt19937_64 rng(7);
  std::vector<std::vector<uint8_t>> fields(5 * n, std::vector<uint8_t>(16 * W));
  for (auto& f : fields)
    for (auto& b : f) b = (uint8_t)(rng() & 0x7f);  // < 2^127 < p: canonical words
  amph_odo odos[n];
  for (int j = 0; j < n; ++j)
    odos[j] = amph_odo{fields[0 * n + j].data(), fields[1 * n + j].data(), fields[2 * n + j].data(),
                       fields[3 * n + j].data(), fields[4 * n + j].data(), 16 * W};
  std::vector<uint8_t> out(16 * W);
  std::vector<double> us;
  for (int i = 0; i < calls + 10; ++i) {
    int64_t ff = -1;
    auto t0 = std::chrono::steady_clock::now();
    int st = rv(ctx, odos, n, out.data(), &ff, 0, nullptr);
    auto t1 = std::chrono::steady_clock::now();
    if (st != AMPH_OK && st != AMPH_E_VERIFY) {
      std::fprintf(stderr, "call %d: status %d\n", i, st);
      return 1;
    }
    if (i >= 10) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  destroy(ctx);
  std::sort(us.begin(), us.end());
  auto q = [&](double f) { return us[std::min(us.size() - 1, (size_t)(f * us.size()))]; };
  std::printf("{\"lib\": \"%s\", \"words\": %zu, \"devices\": \"%s\", \"calls\": %d, "
              "\"us_median\": %.1f, \"us_p10\": %.1f, \"us_p90\": %.1f}\n",
              argv[1], W, argv[4], calls, q(0.5), q(0.1), q(0.9));
  return 0;
}

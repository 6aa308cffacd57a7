// A/B (tool): the base64 codec's bulk launches as a server runs them back to
// back -- 31 launches per span, median of 5 spans -- built from CODEC_SRC so
// two builds of codec.hip alternate on one box: launch_b64_encode and
// launch_b64_decode over a 256 MiB byte stream (16 Mi words), launch_b64_words
// (16 Mi words -> 24-character records).  FNV hashes of the outputs compare
// the builds.
#ifndef CODEC_SRC
#define CODEC_SRC "../../amphora_amd/csrc/codec.hip"
#endif
#include "../../amphora_amd/csrc/kernels.hip"
#include CODEC_SRC
#include <algorithm>
#include <cstdio>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static uint64_t fnv(const std::vector<uint8_t>& v) {
  uint64_t h = 1469598103934665603ull;
  for (uint8_t b : v) h = (h ^ b) * 1099511628211ull;
  return h;
}

int main(int argc, char** argv) {
  constexpr int L = 31;
  const size_t W = (size_t)(argc > 1 ? atoi(argv[1]) : 16) << 20;
  const size_t nb = 16 * W, nc = 4 * ((nb + 2) / 3);
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  for (int i = 0; i < 4; ++i) f.p[i] = p[i];
  f.big = 1;
  uint4 *words, *back;
  char *text, *rec;
  unsigned long long* bad;
  CK(hipMalloc(&words, nb));
  CK(hipMalloc(&back, nb));
  CK(hipMalloc(&text, nc + 256));
  CK(hipMalloc(&rec, 24 * W));
  CK(hipMalloc(&bad, 8));
  CK(hipMemset(bad, 0x7f, 8));
  LaunchCfg c{0, 0, 256};
  CK(launch_synth_words(words, W, 91, f, c));
  CK(launch_b64_encode((const uint8_t*)words, nb, text, c));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<float> t[3];
  for (int r = 0; r < 6; ++r) for (int v = 0; v < 3; ++v) {
    CK(hipEventRecord(e0, 0));
    for (int l = 0; l < L; ++l) {
      if (v == 0) CK(launch_b64_encode((const uint8_t*)words, nb, text, c));
      else if (v == 1) CK(launch_b64_decode(text, nc, (uint8_t*)back, nb, bad, c, true));
      else CK(launch_b64_words(words, W, rec, c));
    }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 1) t[v].push_back(ms * 1e3f / L);
  }
  std::vector<uint8_t> a(nc), b(nb), d(24 * W), src(nb);
  CK(hipMemcpy(a.data(), text, nc, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), back, nb, hipMemcpyDeviceToHost));
  CK(hipMemcpy(src.data(), words, nb, hipMemcpyDeviceToHost));
  CK(hipMemcpy(d.data(), rec, 24 * W, hipMemcpyDeviceToHost));
  unsigned long long hb;
  CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
  printf("%s: text %016llx round trip %s rec %016llx bad %llx\n", CODEC_SRC, (unsigned long long)fnv(a),
         b == src ? "identical" : "DIFFERS", (unsigned long long)fnv(d), hb);
  const char* names[3] = {"b64 encode", "b64 decode", "b64 words"};
  const double bytes[3] = {(double)nb + nc, (double)nb + nc, (double)nb + 24.0 * W};
  for (int v = 0; v < 3; ++v) {
    std::sort(t[v].begin(), t[v].end());
    const double med = t[v][t[v].size() / 2];
    printf("  %-11s median %8.2f us per launch, min %8.2f, %5.2f TB/s\n", names[v], med, t[v][0],
           bytes[v] / (med * 1e-6) / 1e12);
  }
  return 0;
}

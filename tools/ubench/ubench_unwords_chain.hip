// A/B (tool): the service's upload chain as it runs -- the MaskedInput
// records decoded to words (launch_b64_unwords), then K_CONV reads them
// (launch_convert_share) -- 31 chained pairs per span, median of 5 spans,
// 16 Mi words, built from CODEC_SRC so two store policies of k_b64_unwords
// alternate on one box.  Hashes of the shares compare the builds.
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

int main(int argc, char** argv) {
  constexpr int L = 31;
  const size_t W = (size_t)(argc > 1 ? atoi(argv[1]) : 16) << 20;
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = p[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu;
  f.big = 1;
  uint4 *words, *masked, *tuples, *share;
  char* rec;
  unsigned long long* bad;
  CK(hipMalloc(&words, 16 * W)); CK(hipMalloc(&masked, 16 * W)); CK(hipMalloc(&tuples, 32 * W));
  CK(hipMalloc(&share, 32 * W)); CK(hipMalloc(&rec, 24 * W)); CK(hipMalloc(&bad, 8));
  CK(hipMemset(bad, 0x7f, 8));
  LaunchCfg c{0, 0, 256};
  CK(launch_synth_words(words, W, 5, f, c));
  CK(launch_synth_words(tuples, 2 * W, 6, f, c));
  CK(launch_b64_words(words, W, rec, c));
  CK(hipDeviceSynchronize());
  W4 alpha{};
  alpha.v[0] = 12345u;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<float> t;
  for (int r = 0; r < 6; ++r) {
    CK(hipEventRecord(e0, 0));
    for (int l = 0; l < L; ++l) {
      CK(launch_b64_unwords(rec, W, masked, bad, c));
      CK(launch_convert_share(masked, tuples, W, alpha, 0, share, f, c));
    }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 1) t.push_back(ms * 1e3f / L);
  }
  std::vector<uint8_t> a(32 * W);
  CK(hipMemcpy(a.data(), share, 32 * W, hipMemcpyDeviceToHost));
  uint64_t h = 1469598103934665603ull;
  for (uint8_t b : a) h = (h ^ b) * 1099511628211ull;
  std::sort(t.begin(), t.end());
  printf("%s: share %016llx  unwords + k_conv median %8.2f us per pair, min %8.2f\n", CODEC_SRC,
         (unsigned long long)h, t[t.size() / 2], t[0]);
  return 0;
}

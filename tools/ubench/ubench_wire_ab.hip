// Fused wire kernels A/B (tool): k_mask_b64 / k_rv_b64 at W words x NP
// parties from base64 text made on the GPU, built against the csrc directory
// WSRC (a variant copy of amphora_amd/csrc), R back-to-back launches of each
// after 3 warm-up ones.  Prints a checksum of every output, so two builds can
// be compared for identical results, and per-kernel event medians; the
// sustained figure is rocprofv3's average over the same launches.
#ifndef WSRC
#define WSRC ../../amphora_amd/csrc
#endif
#define AMPH_STR2(x) #x
#define AMPH_STR(x) AMPH_STR2(x)
#include AMPH_STR(WSRC/kernels.hip)
#include AMPH_STR(WSRC/wire.hip)
#include AMPH_STR(WSRC/codec.hip)
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static Fp test_fp() {
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = p[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu;
  f.big = 1;
  return f;
}

static unsigned long long fnv(const std::vector<uint8_t>& v) {
  unsigned long long h = 1469598103934665603ull;
  for (uint8_t b : v) h = (h ^ b) * 1099511628211ull;
  return h;
}

int main(int argc, char** argv) {
  constexpr int NP = 3, BS = 256;
  const int R = argc > 1 ? atoi(argv[1]) : 30;
  const size_t W = (size_t)(argc > 2 ? atoi(argv[2]) : 4) << 20;
  const Fp f = test_fp();
  const size_t nb = 16 * W, nc = 4 * ((nb + 2) / 3), stride = (nc + 255) & ~(size_t)255;
  const uint32_t pad = (uint32_t)((3 - nb % 3) % 3);
  uint4 *raw, *y;
  char *text, *rec;
  unsigned long long* fl;
  CK(hipMalloc(&raw, (5 * NP + 1) * nb));
  CK(hipMalloc(&text, 5 * NP * stride));
  CK(hipMalloc(&y, nb));
  CK(hipMalloc(&rec, 24 * W));
  CK(hipMalloc(&fl, 4 * 8));
  CK(hipMemset(fl, 0x7f, 4 * 8));
  OutSet os{};
  for (int k = 0; k < 5; ++k) for (int j = 0; j < NP; ++j) os.f[k][j] = raw + (k * NP + j) * W;
  LaunchCfg c{0, 0, 256};
  CK(launch_synth_odos(os, NP, W, 77, nullptr, -1, 0, f, c));
  CK(launch_synth_words(raw + 5 * NP * W, W, 78, f, c));
  TextSet tx{};
  for (int k = 0; k < 5; ++k) for (int j = 0; j < NP; ++j) {
    char* t = text + (k * NP + j) * stride;
    CK(launch_b64_encode((const uint8_t*)os.f[k][j], nb, t, c));
    tx.t[k][j] = t;
  }
  CK(hipDeviceSynchronize());
  const dim3 g((unsigned)((W + Wire<BS>::words - 1) / Wire<BS>::words));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<float> tm, tr;
  for (int which = 0; which < 2; ++which)
    for (int r = 0; r < R + 3; ++r) {
      CK(hipEventRecord(e0, 0));
      if (which == 0)
        hipLaunchKernelGGL((k_mask_b64<NP, true, BS>), g, dim3(BS), 0, 0, tx, NP, W, nc, pad,
                           (const uint4*)(raw + 5 * NP * W), W, (uint4*)nullptr, rec, fl, fl + 1, f);
      else
        hipLaunchKernelGGL((k_rv_b64<NP, true, BS>), g, dim3(BS), 0, 0, tx, NP, W, nc, pad, y, fl + 2, fl + 3, f);
      CK(hipGetLastError());
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) (which == 0 ? tm : tr).push_back(ms);
    }
  std::vector<uint8_t> a(nb), b(24 * W);
  CK(hipMemcpy(a.data(), y, nb, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), rec, 24 * W, hipMemcpyDeviceToHost));
  unsigned long long h[4];
  CK(hipMemcpy(h, fl, 32, hipMemcpyDeviceToHost));
  std::sort(tm.begin(), tm.end());
  std::sort(tr.begin(), tr.end());
  double sm = 0, sr = 0;
  for (float x : tm) sm += x;
  for (float x : tr) sr += x;
  printf("{\"W\": %zu, \"parties\": %d, \"reps\": %d, \"y_fnv\": \"%016llx\", \"rec_fnv\": \"%016llx\", "
         "\"flags\": [\"%llx\", \"%llx\", \"%llx\", \"%llx\"], "
         "\"k_mask_b64_us\": {\"median\": %.1f, \"mean\": %.1f, \"min\": %.1f}, "
         "\"k_rv_b64_us\": {\"median\": %.1f, \"mean\": %.1f, \"min\": %.1f}}\n",
         W, NP, R, fnv(a), fnv(b), h[0], h[1], h[2], h[3], tm[tm.size() / 2] * 1e3, sm / tm.size() * 1e3,
         tm[0] * 1e3, tr[tr.size() / 2] * 1e3, sr / tr.size() * 1e3, tr[0] * 1e3);
  return 0;
}

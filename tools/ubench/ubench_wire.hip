// Sweep (tool): workgroup size of the fused wire kernels k_rv_b64 / k_mask_b64
// (kernels.hip) at 1 Mi words x 2 parties and 4 Mi x 3, outputs compared
// across sizes; the texts are made on the GPU with the product base64 encoder.
#include "../../amphora_amd/csrc/kernels.hip"
#include "../../amphora_amd/csrc/wire.hip"
#include <algorithm>
#include <cstdio>
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

template <int NP, int BS>
void run_rv(const TextSet& tx, size_t W, size_t nc, uint32_t pad, uint4* out, unsigned long long* fl, Fp f) {
  hipLaunchKernelGGL((k_rv_b64<NP, true, BS>), dim3((unsigned)((W + Wire<BS>::words - 1) / Wire<BS>::words)),
                     dim3(BS), 0, 0, tx, NP, W, nc, pad, out, fl, fl + 1, f);
}
static int g_mask_out = 0;  // argv[2]: 0 = records (24 B), 1 = raw words (16 B), 2 = no output (verify only)
template <int NP, int BS>
void run_mask(const TextSet& tx, size_t W, size_t nc, uint32_t pad, const uint4* sec, char* rec,
              unsigned long long* fl, Fp f) {
  uint4* o16 = g_mask_out == 1 ? (uint4*)rec : nullptr;
  char* o24 = g_mask_out == 0 ? rec : nullptr;
  hipLaunchKernelGGL((k_mask_b64<NP, true, BS>), dim3((unsigned)((W + Wire<BS>::words - 1) / Wire<BS>::words)),
                     dim3(BS), 0, 0, tx, NP, W, nc, pad, sec, W, o16, o24, fl, fl + 1, f);
}

template <int NP>
void sweep(size_t W, int R, Fp f) {
  const size_t nb = 16 * W, nc = 4 * ((nb + 2) / 3), stride = (nc + 255) & ~(size_t)255;
  const uint32_t pad = (uint32_t)((3 - nb % 3) % 3);
  uint4 *raw, *out[3];
  char *text, *rec[3];
  unsigned long long* fl;
  CK(hipMalloc(&raw, (5 * NP + 1) * nb));
  CK(hipMalloc(&text, 5 * NP * stride));
  for (int v = 0; v < 3; ++v) { CK(hipMalloc(&out[v], nb)); CK(hipMalloc(&rec[v], 24 * W)); }
  CK(hipMalloc(&fl, 16 * 8));
  CK(hipMemset(fl, 0x7f, 16 * 8));
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
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<float> t[6];
  for (int r = 0; r < R + 3; ++r) for (int v = 0; v < 6; ++v) {
    CK(hipEventRecord(e0, 0));
    switch (v) {
      case 0: run_rv<NP, 256>(tx, W, nc, pad, out[0], fl, f); break;
      case 1: run_rv<NP, 512>(tx, W, nc, pad, out[1], fl + 2, f); break;
      case 2: run_rv<NP, 1024>(tx, W, nc, pad, out[2], fl + 4, f); break;
      case 3: run_mask<NP, 256>(tx, W, nc, pad, raw + 5 * NP * W, rec[0], fl + 6, f); break;
      case 4: run_mask<NP, 512>(tx, W, nc, pad, raw + 5 * NP * W, rec[1], fl + 8, f); break;
      case 5: run_mask<NP, 1024>(tx, W, nc, pad, raw + 5 * NP * W, rec[2], fl + 10, f); break;
    }
    CK(hipGetLastError());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 3) t[v].push_back(ms);
  }
  std::vector<uint8_t> a(nb), b(nb), ra(24 * W), rb(24 * W);
  bool same = true;
  CK(hipMemcpy(a.data(), out[2], nb, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ra.data(), rec[2], 24 * W, hipMemcpyDeviceToHost));
  for (int v = 0; v < 2; ++v) {
    CK(hipMemcpy(b.data(), out[v], nb, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rb.data(), rec[v], 24 * W, hipMemcpyDeviceToHost));
    same = same && a == b && ra == rb;
  }
  unsigned long long h[16];
  CK(hipMemcpy(h, fl, 16 * 8, hipMemcpyDeviceToHost));
  printf("N=%d W=%zu outputs %s, flags %llx %llx\n", NP, W, same ? "identical" : "DIFFER", h[4], h[5]);
  const char* names[6] = {"k_rv_b64 BS=256", "k_rv_b64 BS=512", "k_rv_b64 BS=1024",
                          "k_mask_b64 BS=256", "k_mask_b64 BS=512", "k_mask_b64 BS=1024"};
  for (int v = 0; v < 6; ++v) {
    std::sort(t[v].begin(), t[v].end());
    const double med = t[v][t[v].size() / 2];
    const double bytes = v < 3 ? (5.0 * NP * nc + nb) : (5.0 * NP * nc + nb + 24.0 * W);
    printf("  %-20s median %8.2f us  min %8.2f us  %7.1f GB/s  %6.2f G words/s\n", names[v], med * 1e3,
           t[v][0] * 1e3, bytes / (med * 1e-3) / 1e9, W / (med * 1e-3) / 1e9);
  }
  CK(hipFree(raw)); CK(hipFree(text)); CK(hipFree(fl));
  for (int v = 0; v < 3; ++v) { CK(hipFree(out[v])); CK(hipFree(rec[v])); }
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 20;
  g_mask_out = argc > 2 ? atoi(argv[2]) : 0;
  Fp f = test_fp();
  sweep<2>((size_t)1 << 20, R, f);
  sweep<2>((size_t)1 << 24, R, f);
  sweep<3>((size_t)1 << 22, R, f);
  return 0;
}

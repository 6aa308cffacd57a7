// N=3 K_MASK / K_RV occupancy A/B (tool): default vs waves-per-EU hints.
#include "../../amphora_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <vector>
using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
namespace amph { namespace {
template <int WPE>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(WPE, 8)))
void k_mask_o(OdoSet odo, size_t words, const uint4* secrets, uint4* out, unsigned long long* ff, Fp f) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= words) return;
  const uint4 s = ld(secrets + i);
  W4 a[5];
  recombine5<3, true>(odo, 3, i, f, a);
  const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
  st(out + i, mod_sub(mont_mul(w4(s), r2_word(f), f), a[0], f));
  report_fail(!ok, i, ff);
}
template <int WPE>
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(WPE, 8)))
void k_rv_o(OdoSet odo, size_t words, uint4* out, unsigned long long* ff, Fp f) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= words) return;
  W4 a[5];
  recombine5<3, true>(odo, 3, i, f, a);
  const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
  st(out + i, redc(a[0], f));
  report_fail(!ok, i, ff);
}
}}
__global__ void k_init(uint4* buf, size_t W, int n, Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < W; i += stride) {
    auto hr = [&](uint64_t x) {
      x = x * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
      uint64_t a = (x ^ (x >> 29)) * 0x94D049BB133111EBull, b = (x * 0xBF58476D1CE4E5B9ull) ^ (x >> 31);
      return canon<true>(W4{{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)}}, f);
    };
    W4 v[5];
    for (int k = 0; k < 3; ++k) v[k] = hr(i * 64 + k);
    v[3] = mont_mul(v[0], v[1], f);
    v[4] = mont_mul(v[2], v[1], f);
    for (int k = 0; k < 5; ++k) {
      W4 rest = v[k];
      for (int j = 0; j < n - 1; ++j) {
        const W4 s0 = hr(i * 64 + 8 + k * 8 + j);
        buf[(size_t)(k * n + j) * W + i] = u4(s0);
        rest = mod_sub(rest, s0, f);
      }
      buf[(size_t)(k * n + n - 1) * W + i] = u4(rest);
    }
    buf[(size_t)5 * n * W + i] = u4(hr(i * 64 + 60));
  }
}
int main() {
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = p[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu; f.big = 1;
  const int n = 3;
  for (size_t W : {(size_t)1 << 20, (size_t)1 << 24}) {
    uint4* buf;
    CK(hipMalloc(&buf, (size_t)(5 * n + 2) * W * 16));
    hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, buf, W, n, f);
    CK(hipDeviceSynchronize());
    OdoSet odo{};
    for (int k = 0; k < 5; ++k) for (int j = 0; j < n; ++j) odo.f[k][j] = buf + (size_t)(k * n + j) * W;
    const uint4* sec = buf + (size_t)5 * n * W;
    uint4* out = buf + (size_t)(5 * n + 1) * W;
    unsigned long long* ff; CK(hipMalloc(&ff, 64)); CK(hipMemset(ff, 0x7f, 64));
    const char* names[] = {"mask_prod", "mask_w5", "mask_w6", "mask_w8", "mask_prod512", "rv_prod", "rv_w6", "rv_w8"};
    std::vector<std::vector<float>> t(8);
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const unsigned g = (unsigned)((W + 1023) / 1024);
    for (int r = 0; r < 23; ++r) for (int v = 0; v < 8; ++v) {
      CK(hipEventRecord(e0, 0));
      switch (v) {
        case 0: launch_mask_input(odo, n, W, sec, W, out, ff, f, LaunchCfg{0, 0, 1024}); break;
        case 1: hipLaunchKernelGGL(k_mask_o<5>, dim3(g), dim3(1024), 0, 0, odo, W, sec, out, ff, f); break;
        case 2: hipLaunchKernelGGL(k_mask_o<6>, dim3(g), dim3(1024), 0, 0, odo, W, sec, out, ff, f); break;
        case 3: hipLaunchKernelGGL(k_mask_o<8>, dim3(g), dim3(1024), 0, 0, odo, W, sec, out, ff, f); break;
        case 4: launch_mask_input(odo, n, W, sec, W, out, ff, f, LaunchCfg{0, 0, 512}); break;
        case 5: launch_recombine_verify(odo, n, W, out, ff, f, LaunchCfg{0, 0, 1024}); break;
        case 6: hipLaunchKernelGGL(k_rv_o<6>, dim3(g), dim3(1024), 0, 0, odo, W, out, ff, f); break;
        case 7: hipLaunchKernelGGL(k_rv_o<8>, dim3(g), dim3(1024), 0, 0, odo, W, out, ff, f); break;
      }
      CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) t[v].push_back(ms);
    }
    unsigned long long h; CK(hipMemcpy(&h, ff, 8, hipMemcpyDeviceToHost));
    printf("N=3 W=%zu ff=%llx\n", W, h);
    for (int v = 0; v < 8; ++v) {
      std::sort(t[v].begin(), t[v].end());
      const double bytes = (v >= 5 ? 256.0 : 272.0) * W, med = t[v][10];
      printf("  %-12s median %9.2f us  %7.1f GB/s\n", names[v], med * 1e3, bytes / (med * 1e-3) / 1e9);
    }
    CK(hipFree(buf)); CK(hipFree(ff));
  }
}

// A/B (tool): output stores of K_MASK / K_RV plain (product) vs nontemporal
// (global_store_dwordx4 nt), at 1 Mi and 16 Mi words, 2 parties.
#include "../../amphora_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace amph { namespace {
__device__ __forceinline__ void st_nt(uint4* p, const W4& v) {
  u32x4 x = {v.v[0], v.v[1], v.v[2], v.v[3]};
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p));
}
template <int NP>
__global__ __launch_bounds__(1024) void k_mask_nt(OdoSet odo, size_t words, const uint4* secrets,
                                                 uint4* out, unsigned long long* ff, Fp f) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= words) return;
  const W4 r2 = r2_word(f);
  const uint4 s = ld(secrets + i);
  W4 a[5];
  recombine5<NP, true>(odo, NP, i, f, a);
  const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
  st_nt(out + i, mod_sub(mont_mul(w4(s), r2, f), a[0], f));
  report_fail(!ok, i, ff);
}
template <int NP>
__global__ __launch_bounds__(1024) void k_rv_nt(OdoSet odo, size_t words, uint4* y,
                                               unsigned long long* ff, Fp f) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= words) return;
  W4 a[5];
  recombine5<NP, true>(odo, NP, i, f, a);
  const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
  st_nt(y + i, redc(a[0], f));
  report_fail(!ok, i, ff);
}
}}  // namespace amph::(anon)

static Fp test_fp() {
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = p[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu;
  f.big = 1;
  return f;
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 50;
  Fp f = test_fp();
  const int n = 2;
  for (size_t W : {(size_t)1 << 20, (size_t)1 << 24}) {
    uint4 *mb, *sb, *sec, *o1, *o2;
    unsigned long long* ff;
    CK(hipMalloc(&mb, 5 * n * W * 16)); CK(hipMalloc(&sb, 5 * n * W * 16)); CK(hipMalloc(&sec, W * 16));
    CK(hipMalloc(&o1, W * 16)); CK(hipMalloc(&o2, W * 16)); CK(hipMalloc(&ff, 16));
    OutSet om{}, os{};
    OdoSet mo{}, so{};
    for (int k = 0; k < 5; ++k) for (int j = 0; j < n; ++j) {
      om.f[k][j] = mb + (size_t)(k * n + j) * W; mo.f[k][j] = om.f[k][j];
      os.f[k][j] = sb + (size_t)(k * n + j) * W; so.f[k][j] = os.f[k][j];
    }
    LaunchCfg c{0, 0, 1024};
    CK(launch_synth_odos(om, n, W, 1, nullptr, -1, 0, f, c));
    CK(launch_synth_odos(os, n, W, 2, nullptr, -1, 0, f, c));
    CK(launch_synth_words(sec, W, 3, f, c));
    CK(hipMemset(ff, 0x7F, 16));
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const unsigned g = (unsigned)((W + 1023) / 1024);
    const char* names[] = {"mask_plain", "mask_nt", "rv_plain", "rv_nt", "step_plain", "step_nt"};
    std::vector<float> t[6];
    for (int r = 0; r < R + 3; ++r) for (int v = 0; v < 6; ++v) {
      CK(hipEventRecord(e0, 0));
      if (v == 0 || v == 4) CK(launch_mask_input(mo, n, W, sec, W, o1, ff, f, c));
      if (v == 1 || v == 5) hipLaunchKernelGGL((k_mask_nt<2>), dim3(g), dim3(1024), 0, 0, mo, W, sec, o2, ff, f);
      if (v == 2 || v == 4) CK(launch_recombine_verify(so, n, W, o1, ff + 1, f, c));
      if (v == 3 || v == 5) hipLaunchKernelGGL((k_rv_nt<2>), dim3(g), dim3(1024), 0, 0, so, W, o2, ff + 1, f);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) t[v].push_back(ms);
      if (r == 0 && (v == 1 || v == 3)) {
        std::vector<uint4> a(W), b(W);
        CK(hipMemcpy(a.data(), o1, W * 16, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), o2, W * 16, hipMemcpyDeviceToHost));
        printf("  %s matches: %d\n", names[v], !memcmp(a.data(), b.data(), W * 16));
      }
    }
    printf("W=%zu\n", W);
    const double bytes[6] = {192, 192, 176, 176, 368, 368};
    for (int v = 0; v < 6; ++v) {
      std::sort(t[v].begin(), t[v].end());
      const double med = t[v][t[v].size() / 2];
      printf("  %-11s median %8.2f us  %7.1f GB/s\n", names[v], med * 1e3, bytes[v] * W / (med * 1e-3) / 1e9);
    }
    CK(hipFree(mb)); CK(hipFree(sb)); CK(hipFree(sec)); CK(hipFree(o1)); CK(hipFree(o2)); CK(hipFree(ff));
  }
  return 0;
}

// K_CONV mapping A/B (tool): word per lane (product) vs two lanes per word
// (lane 2i: value' = value + [m]; lane 2i+1: mac' = mac + [alpha][m]), fully coalesced.
#include "../../amphora_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>
using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
namespace amph { namespace {
__global__ __launch_bounds__(1024) void k_conv2(const uint4* masked, const uint4* tuples, size_t n2,
                                               W4 alpha, int use_zero, uint4* out, Fp f) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n2) return;
  const uint4 tr = ld(tuples + t), mr = ld(masked + (t >> 1));
  const W4 m = canon<true>(w4(mr), f), x = canon<true>(w4(tr), f);
  W4 z;
  if (t & 1) z = mod_add(x, mont_mul(m, alpha, f), f);
  else z = use_zero ? x : mod_add(x, m, f);
  st(out + t, z);
}
}}
__global__ void k_fill(uint4* b, size_t n, Fp f) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull + 77, y = (x ^ (x >> 31)) * 0xBF58476D1CE4E5B9ull;
    b[i] = u4(canon<true>(W4{{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 33)}}, f));
  }
}
int main() {
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = p[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu; f.big = 1;
  for (size_t W : {(size_t)1 << 20, (size_t)1 << 24}) {
    uint4 *m, *t, *o1, *o2;
    CK(hipMalloc(&m, W * 16)); CK(hipMalloc(&t, 2 * W * 16)); CK(hipMalloc(&o1, 2 * W * 16)); CK(hipMalloc(&o2, 2 * W * 16));
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, m, W, f);
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, t, 2 * W, f);
    W4 alpha{{123, 456, 789, 0x1000}};
    LaunchCfg c{0, 0, 1024};
    std::vector<float> ta, tb;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int r = 0; r < 23; ++r) for (int v = 0; v < 2; ++v) {
      CK(hipEventRecord(e0, 0));
      if (v == 0) launch_convert_share(m, t, W, alpha, 0, o1, f, c);
      else hipLaunchKernelGGL(k_conv2, dim3((2 * W + 1023) / 1024), dim3(1024), 0, 0, m, t, 2 * W, alpha, 0, o2, f);
      CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) (v ? tb : ta).push_back(ms);
    }
    std::vector<uint4> a(2 * W), b(2 * W);
    CK(hipMemcpy(a.data(), o1, 2 * W * 16, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), o2, 2 * W * 16, hipMemcpyDeviceToHost));
    std::sort(ta.begin(), ta.end()); std::sort(tb.begin(), tb.end());
    printf("W=%zu same=%d prod %.2f us %.1f GB/s | two-lane %.2f us %.1f GB/s\n", W, memcmp(a.data(), b.data(), 2 * W * 16) == 0,
           ta[10] * 1e3, 80.0 * W / (ta[10] * 1e-3) / 1e9, tb[10] * 1e3, 80.0 * W / (tb[10] * 1e-3) / 1e9);
  }
}

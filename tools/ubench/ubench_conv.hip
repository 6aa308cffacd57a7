// K_CONV mapping A/B (tool): word per lane (product) vs two lanes per word
// (lane 2i: value' = value + [m]; lane 2i+1: mac' = mac + [alpha][m]), fully
// coalesced, vs word per lane with the workgroup's input-mask tuples and
// output shares moved through LDS as coalesced 16-B runs (stage_tuples).
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
template <int BS>
__global__ __launch_bounds__(BS) void k_conv3(const uint4* masked, const uint4* tuples, size_t words,
                                             W4 alpha, int use_zero, uint4* out, Fp f) {
  __shared__ uint4 buf[3 * BS];
  const size_t i0 = (size_t)blockIdx.x * BS, i = i0 + threadIdx.x;
  const size_t nblk = min((size_t)BS, words - i0);
  stage_tuples<2, BS>(buf, tuples + 2 * i0, nblk);
  uint4 mr = make_uint4(0, 0, 0, 0);
  if (i < words) mr = ld(masked + i);
  __syncthreads();
  if (i < words) {
    const W4 m = canon<true>(w4(mr), f);
    const W4 val = canon<true>(w4(buf[3 * threadIdx.x]), f), mac = canon<true>(w4(buf[3 * threadIdx.x + 1]), f);
    buf[3 * threadIdx.x] = u4(use_zero ? val : mod_add(val, m, f));
    buf[3 * threadIdx.x + 1] = u4(mod_add(mac, mont_mul(m, alpha, f), f));
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const size_t q = (size_t)r * BS + threadIdx.x;
    if (q < 2 * nblk) out[2 * i0 + q] = buf[(q >> 1) * 3 + (q & 1)];
  }
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
    uint4 *m, *t, *o1, *o2, *o3;
    CK(hipMalloc(&m, W * 16)); CK(hipMalloc(&t, 2 * W * 16)); CK(hipMalloc(&o1, 2 * W * 16)); CK(hipMalloc(&o2, 2 * W * 16));
    CK(hipMalloc(&o3, 2 * W * 16));
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, m, W, f);
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, t, 2 * W, f);
    W4 alpha{{123, 456, 789, 0x1000}};
    LaunchCfg c{0, 0, 1024};
    std::vector<float> ta, tb, tc, td;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int r = 0; r < 23; ++r) for (int v = 0; v < 4; ++v) {
      CK(hipEventRecord(e0, 0));
      if (v == 0) launch_convert_share(m, t, W, alpha, 0, o1, f, c);
      else if (v == 1) hipLaunchKernelGGL(k_conv2, dim3((2 * W + 1023) / 1024), dim3(1024), 0, 0, m, t, 2 * W, alpha, 0, o2, f);
      else if (v == 2) hipLaunchKernelGGL(k_conv3<256>, dim3((W + 255) / 256), dim3(256), 0, 0, m, t, W, alpha, 0, o3, f);
      else hipLaunchKernelGGL(k_conv3<512>, dim3((W + 511) / 512), dim3(512), 0, 0, m, t, W, alpha, 0, o3, f);
      CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) (v == 0 ? ta : v == 1 ? tb : v == 2 ? tc : td).push_back(ms);
    }
    std::vector<uint4> a(2 * W), b(2 * W), d(2 * W);
    CK(hipMemcpy(a.data(), o1, 2 * W * 16, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), o2, 2 * W * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(d.data(), o3, 2 * W * 16, hipMemcpyDeviceToHost));
    for (auto* v : {&ta, &tb, &tc, &td}) std::sort(v->begin(), v->end());
    printf("W=%zu same=%d/%d prod %.2f us %.1f GB/s | two-lane %.2f us %.1f GB/s | lds256 %.2f us %.1f GB/s | lds512 %.2f us %.1f GB/s\n", W,
           memcmp(a.data(), b.data(), 2 * W * 16) == 0, memcmp(a.data(), d.data(), 2 * W * 16) == 0,
           ta[10] * 1e3, 80.0 * W / (ta[10] * 1e-3) / 1e9, tb[10] * 1e3, 80.0 * W / (tb[10] * 1e-3) / 1e9,
           tc[10] * 1e3, 80.0 * W / (tc[10] * 1e-3) / 1e9, td[10] * 1e3, 80.0 * W / (td[10] * 1e-3) / 1e9);
  }
}

// Montgomery product variants (tool): mont_mul_ps (product scanning, the
// mad's carry-out through inline asm) against mont_mul_cios (the compiler's
// lowering of CIOS) -- bit-exact over 64 Mi random and edge operand pairs,
// then the throughput of dependent chains of each.
#include "../../amphora_amd/csrc/field.hpp"
#include <cstdio>
#include <vector>
#include <algorithm>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void k_check(size_t n, Fp f, unsigned long long* bad) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint64_t x0 = mix(4 * i), x1 = mix(4 * i + 1), x2 = mix(4 * i + 2), x3 = mix(4 * i + 3);
    W4 a{{(uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1, (uint32_t)(x1 >> 32)}};
    W4 b{{(uint32_t)x2, (uint32_t)(x2 >> 32), (uint32_t)x3, (uint32_t)(x3 >> 32)}};
    // edge operands on a share of the lanes: all-ones a, p - 1, 0, 1
    const int e = (int)(i % 16);
    if (e == 1) a = W4{{~0u, ~0u, ~0u, ~0u}};
    if (e == 2) b = W4{{f.p[0] - 1, f.p[1], f.p[2], f.p[3]}};
    if (e == 3) a = W4{{0, 0, 0, 0}};
    if (e == 4) b = W4{{1, 0, 0, 0}};
    if (e == 5) { a = W4{{~0u, ~0u, ~0u, ~0u}}; b = W4{{f.p[0] - 1, f.p[1], f.p[2], f.p[3]}}; }
    b = reduce_once(b, 0, f);  // b < p
    const W4 u = mont_mul_ps(a, b, f), v = mont_mul_cios(a, b, f);
    if (!eq(u, v)) atomicAdd(bad, 1ull);
  }
}

template <int V>
__global__ __launch_bounds__(256) void k_chain(uint4* io, int iters, Fp f) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  W4 a = w4(io[i]), b = reduce_once(w4(io[i + 1]), 0, f);
  for (int t = 0; t < iters; ++t) {
    a = V ? mont_mul_ps(a, b, f) : mont_mul_cios(a, b, f);
    b = V ? mont_mul_ps(b, a, f) : mont_mul_cios(b, a, f);
  }
  io[i] = u4(a);
}

int main() {
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = p[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu;
  f.big = 1;
  unsigned long long* bad;
  CK(hipMalloc(&bad, 8));
  CK(hipMemset(bad, 0, 8));
  hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, 0, (size_t)1 << 26, f, bad);
  unsigned long long hb;
  CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
  printf("mismatches over 64 Mi products: %llu\n", hb);
  const size_t n = (size_t)256 * 1024 * 4;
  uint4* io;
  CK(hipMalloc(&io, (n + 1) * 16));
  CK(hipMemset(io, 0x35, (n + 1) * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int v = 0; v < 2; ++v) {
    std::vector<float> t;
    for (int r = 0; r < 8; ++r) {
      CK(hipEventRecord(e0, 0));
      if (v) hipLaunchKernelGGL(k_chain<1>, dim3(n / 256), dim3(256), 0, 0, io, 64, f);
      else hipLaunchKernelGGL(k_chain<0>, dim3(n / 256), dim3(256), 0, 0, io, 64, f);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double prods = (double)n * 128;
    printf("%-14s median %8.3f ms  %7.2f G mont_mul/s\n", v ? "mont_mul_ps" : "mont_mul_cios", t[t.size() / 2],
           prods / (t[t.size() / 2] * 1e-3) / 1e9);
  }
  return 0;
}

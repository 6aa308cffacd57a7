// Words per thread at C2 (1 Mi words, 2 parties): does giving each thread
// WPT words (loads of all of them issued before any arithmetic, word w at
// i + w * grid) and a grid that fits the chip in one round beat the product's
// one word per thread over two rounds of workgroups?  Also the pure-memory
// version of the same access pattern (11 streams in, 1 out, no math) for each
// shape (tool, not product).
#include "../../amphora_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace amph { namespace {
template <int NP, int WPT, int BS>
__global__ __launch_bounds__(BS) void k_mask_w(OdoSet odo, size_t words, const uint4* secrets,
                                               uint4* out, unsigned long long* ff, Fp f) {
  const size_t G = (size_t)gridDim.x * BS;
  const size_t i0 = (size_t)blockIdx.x * BS + threadIdx.x;
  uint4 s[WPT];
  uint4 raw[WPT][5][NP];
#pragma unroll
  for (int w = 0; w < WPT; ++w) {
    const size_t i = i0 + w * G;
    s[w] = ld(secrets + i);
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int j = 0; j < NP; ++j) raw[w][k][j] = ld(odo.f[k][j] + i);
  }
  __builtin_amdgcn_sched_barrier(0);  // keep every load ahead of the arithmetic
  const W4 r2 = r2_word(f);
#pragma unroll
  for (int w = 0; w < WPT; ++w) {
    const size_t i = i0 + w * G;
    W4 a[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      a[k] = canon<true>(w4(raw[w][k][0]), f);
#pragma unroll
      for (int j = 1; j < NP; ++j) a[k] = mod_add(a[k], canon<true>(w4(raw[w][k][j]), f), f);
    }
    const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
    st(out + i, mod_sub(mont_mul(w4(s[w]), r2, f), a[0], f));
    report_fail(!ok, i, ff);
  }
}

// same loads and store, XOR instead of field arithmetic
template <int NP, int WPT, int BS>
__global__ __launch_bounds__(BS) void k_mem_w(OdoSet odo, size_t words, const uint4* secrets,
                                              uint4* out) {
  const size_t G = (size_t)gridDim.x * BS;
  const size_t i0 = (size_t)blockIdx.x * BS + threadIdx.x;
  uint4 acc[WPT];
#pragma unroll
  for (int w = 0; w < WPT; ++w) {
    const size_t i = i0 + w * G;
    acc[w] = ld(secrets + i);
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const uint4 v = ld(odo.f[k][j] + i);
        acc[w].x ^= v.x; acc[w].y ^= v.y; acc[w].z ^= v.z; acc[w].w ^= v.w;
      }
  }
#pragma unroll
  for (int w = 0; w < WPT; ++w) out[i0 + w * G] = acc[w];
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

__global__ void k_fill(uint4* buf, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    buf[i] = make_uint4((uint32_t)i * 2654435761u, (uint32_t)(i >> 7) ^ 0x5bd1e995u, (uint32_t)i, 0x12345u);
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 40;
  Fp f = test_fp();
  constexpr int n = 2;
  for (size_t W : {(size_t)1 << 20, (size_t)1 << 22, (size_t)1 << 24}) {
    uint4* buf;
    CK(hipMalloc(&buf, (size_t)(5 * n + 2) * W * 16));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, buf, (size_t)(5 * n + 2) * W);
    CK(hipDeviceSynchronize());
    OdoSet odo{};
    for (int k = 0; k < 5; ++k) for (int j = 0; j < n; ++j) odo.f[k][j] = buf + (size_t)(k * n + j) * W;
    const uint4* sec = buf + (size_t)5 * n * W;
    uint4* out = buf + (size_t)(5 * n + 1) * W;
    unsigned long long* ff;
    CK(hipMalloc(&ff, 64));
    const char* names[] = {"prod_mask", "mask_w1_b1024", "mask_w2_b1024", "mask_w2_b512",
                           "mask_w4_b256", "mem_w1_b1024", "mem_w2_b1024", "mem_w4_b1024",
                           "mem_w2_b512"};
    constexpr int NV = 9;
    std::vector<std::vector<float>> t(NV);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int r = 0; r < R + 3; ++r) for (int v = 0; v < NV; ++v) {
      LaunchCfg c{0, 0, 1024};
      CK(hipEventRecord(e0, 0));
      switch (v) {
        case 0: launch_mask_input(odo, n, W, sec, W, out, ff, f, c); break;
        case 1: hipLaunchKernelGGL((k_mask_w<2, 1, 1024>), dim3(W / 1024), dim3(1024), 0, 0, odo, W, sec, out, ff, f); break;
        case 2: hipLaunchKernelGGL((k_mask_w<2, 2, 1024>), dim3(W / 2048), dim3(1024), 0, 0, odo, W, sec, out, ff, f); break;
        case 3: hipLaunchKernelGGL((k_mask_w<2, 2, 512>), dim3(W / 1024), dim3(512), 0, 0, odo, W, sec, out, ff, f); break;
        case 4: hipLaunchKernelGGL((k_mask_w<2, 4, 256>), dim3(W / 1024), dim3(256), 0, 0, odo, W, sec, out, ff, f); break;
        case 5: hipLaunchKernelGGL((k_mem_w<2, 1, 1024>), dim3(W / 1024), dim3(1024), 0, 0, odo, W, sec, out); break;
        case 6: hipLaunchKernelGGL((k_mem_w<2, 2, 1024>), dim3(W / 2048), dim3(1024), 0, 0, odo, W, sec, out); break;
        case 7: hipLaunchKernelGGL((k_mem_w<2, 4, 1024>), dim3(W / 4096), dim3(1024), 0, 0, odo, W, sec, out); break;
        case 8: hipLaunchKernelGGL((k_mem_w<2, 2, 512>), dim3(W / 1024), dim3(512), 0, 0, odo, W, sec, out); break;
      }
      CK(hipGetLastError());
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) t[v].push_back(ms);
    }
    printf("N=%d W=%zu\n", n, W);
    for (int v = 0; v < NV; ++v) {
      std::sort(t[v].begin(), t[v].end());
      const double bytes = (80.0 * n + 32) * W;
      printf("  %-15s median %9.2f us  min %9.2f us  %7.1f GB/s\n", names[v], t[v][t[v].size() / 2] * 1e3,
             t[v][0] * 1e3, bytes / (t[v][t[v].size() / 2] * 1e-3) / 1e9);
    }
    CK(hipFree(buf)); CK(hipFree(ff));
  }
  return 0;
}

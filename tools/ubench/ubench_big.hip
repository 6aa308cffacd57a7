// Why is the K_MASK access pattern (11 x 16-B streams in, 1 out) slower at
// 64 Mi words (5.6 TB/s) than at 16 Mi (6.06 TB/s)?  Pure-memory kernel
// (XOR of the streams, no field arithmetic), one word per thread, 1024-thread
// groups, timed four ways (tool, not product):
//   one       one launch over all W words
//   slices    W / 16 Mi launches of 16 Mi words each, back to back
//   sep       the 12 arrays as separate hipMalloc allocations (one launch)
//   sep_sl    separate allocations, 16 Mi-word slices
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
struct Streams { const uint4* in[11]; uint4* out; };

__device__ __forceinline__ uint4 ld(const uint4* p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

__global__ __launch_bounds__(1024) void k_mem(Streams s, size_t base, size_t words) {
  const size_t i = base + (size_t)blockIdx.x * 1024 + threadIdx.x;
  if (i >= base + words) return;
  uint4 v[11];
#pragma unroll
  for (int k = 0; k < 11; ++k) v[k] = ld(s.in[k] + i);
  uint4 a = v[0];
#pragma unroll
  for (int k = 1; k < 11; ++k) { a.x ^= v[k].x; a.y ^= v[k].y; a.z ^= v[k].z; a.w ^= v[k].w; }
  s.out[i] = a;
}

__global__ void k_fill(uint4* buf, size_t n, uint32_t salt) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    buf[i] = make_uint4((uint32_t)i * 2654435761u, salt, (uint32_t)i, 0x12345u);
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 10;
  const size_t SL = (size_t)1 << 24;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (size_t W : {(size_t)1 << 24, (size_t)1 << 25, (size_t)1 << 26}) {
    Streams one{}, sep{};
    uint4* big;
    CK(hipMalloc(&big, 12 * W * 16));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, big, 12 * W, 1u);
    for (int k = 0; k < 11; ++k) one.in[k] = big + k * W;
    one.out = big + 11 * W;
    std::vector<uint4*> parts(12);
    for (int k = 0; k < 12; ++k) {
      CK(hipMalloc(&parts[k], W * 16));
      hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, parts[k], W, (uint32_t)k);
    }
    for (int k = 0; k < 11; ++k) sep.in[k] = parts[k];
    sep.out = parts[11];
    CK(hipDeviceSynchronize());
    const char* names[] = {"one", "slices", "sep", "sep_sl"};
    std::vector<std::vector<float>> t(4);
    for (int r = 0; r < R + 2; ++r) for (int v = 0; v < 4; ++v) {
      const Streams& s = (v < 2) ? one : sep;
      const bool sliced = (v & 1) != 0;
      CK(hipEventRecord(e0, 0));
      if (!sliced) {
        hipLaunchKernelGGL(k_mem, dim3((unsigned)(W / 1024)), dim3(1024), 0, 0, s, (size_t)0, W);
      } else {
        for (size_t b = 0; b < W; b += SL)
          hipLaunchKernelGGL(k_mem, dim3((unsigned)(SL / 1024)), dim3(1024), 0, 0, s, b, SL);
      }
      CK(hipGetLastError());
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 2) t[v].push_back(ms);
    }
    printf("W=%zu Mi words (12 arrays x %zu MiB)\n", W >> 20, W * 16 >> 20);
    for (int v = 0; v < 4; ++v) {
      std::sort(t[v].begin(), t[v].end());
      const double bytes = 12.0 * 16 * W;
      printf("  %-7s median %9.2f us  min %9.2f us  %7.1f GB/s\n", names[v], t[v][t[v].size() / 2] * 1e3,
             t[v][0] * 1e3, bytes / (t[v][t[v].size() / 2] * 1e-3) / 1e9);
    }
    CK(hipFree(big));
    for (auto p : parts) CK(hipFree(p));
  }
  return 0;
}

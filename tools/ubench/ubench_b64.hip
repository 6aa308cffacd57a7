// A/B (tool): base64 stream kernels, product (per-lane 12-byte units: three
// dword accesses at a 12-byte lane stride) vs workgroup-staged through LDS
// (fully coalesced 16-byte loads/stores of the block's contiguous run).
#include "../../amphora_amd/csrc/codec.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace amph { namespace {
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldnt(const uint4* p) {
  const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
template <int BS>
__global__ __launch_bounds__(BS) void k_enc_lds(const uint8_t* in, size_t nbytes, char* out) {
  __shared__ uint32_t lds[3 * BS];
  const size_t u0 = (size_t)blockIdx.x * BS;       // first unit of the block
  const size_t t = u0 + threadIdx.x;
  const uint4* src = reinterpret_cast<const uint4*>(in + 12 * u0);
  // full blocks only (the launcher gives the ragged tail to the product kernel)
  for (int q = threadIdx.x; q < 3 * BS / 4; q += BS) {
    const uint4 v = ldnt(src + q);
    lds[4 * q] = v.x; lds[4 * q + 1] = v.y; lds[4 * q + 2] = v.z; lds[4 * q + 3] = v.w;
  }
  __syncthreads();
  uint8_t b[12];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const uint32_t x = lds[3 * threadIdx.x + q];
    b[4 * q] = x & 0xFF; b[4 * q + 1] = (x >> 8) & 0xFF; b[4 * q + 2] = (x >> 16) & 0xFF; b[4 * q + 3] = x >> 24;
  }
  uint32_t g[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) g[q] = enc_group(b[3 * q], b[3 * q + 1], b[3 * q + 2]);
  *reinterpret_cast<uint4*>(out + 16 * t) = make_uint4(g[0], g[1], g[2], g[3]);
}

template <int BS>
__global__ __launch_bounds__(BS) void k_dec_lds(const char* in, uint8_t* out, unsigned long long* bad) {
  __shared__ uint32_t lds[3 * BS];
  const size_t u0 = (size_t)blockIdx.x * BS, t = u0 + threadIdx.x;
  const uint4 v = ldnt(reinterpret_cast<const uint4*>(in) + t);
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t firstbad = 0xFFFFFFFFu, o[3] = {0, 0, 0};
  uint8_t ob[12];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t d[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      d[k] = dec6((w[q] >> (8 * k)) & 0xFF);
      if (d[k] == 0xFFu && firstbad == 0xFFFFFFFFu) firstbad = 4 * q + k;
    }
    const uint32_t gg = (d[0] << 18) | (d[1] << 12) | (d[2] << 6) | d[3];
    ob[3 * q] = (gg >> 16) & 0xFF; ob[3 * q + 1] = (gg >> 8) & 0xFF; ob[3 * q + 2] = gg & 0xFF;
  }
#pragma unroll
  for (int q = 0; q < 3; ++q)
    o[q] = ob[4 * q] | (ob[4 * q + 1] << 8) | (ob[4 * q + 2] << 16) | ((uint32_t)ob[4 * q + 3] << 24);
  if (firstbad != 0xFFFFFFFFu) atomicMin(bad, (unsigned long long)(16 * t + firstbad));
#pragma unroll
  for (int q = 0; q < 3; ++q) lds[3 * threadIdx.x + q] = o[q];
  __syncthreads();
  uint4* dst = reinterpret_cast<uint4*>(out + 12 * u0);
  for (int q = threadIdx.x; q < 3 * BS / 4; q += BS)
    dst[q] = make_uint4(lds[4 * q], lds[4 * q + 1], lds[4 * q + 2], lds[4 * q + 3]);
}
}}  // namespace amph::(anon)

__global__ void k_fill(uint8_t* b, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b[i] = (uint8_t)((i * 0x9E3779B97F4A7C15ull) >> 56);
}

int main() {
  const size_t n = (size_t)3 << 28;  // 768 MiB
  const size_t units = n / 12, nch = 16 * units;
  uint8_t *in, *dec1, *dec2;
  char *e1, *e2;
  unsigned long long* bad;
  CK(hipMalloc(&in, n)); CK(hipMalloc(&dec1, n)); CK(hipMalloc(&dec2, n));
  CK(hipMalloc(&e1, nch)); CK(hipMalloc(&e2, nch)); CK(hipMalloc(&bad, 8));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, in, n);
  CK(hipMemset(bad, 0x7F, 8));
  CK(hipDeviceSynchronize());
  LaunchCfg c{0, 0, 1024};
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto timeit = [&](auto fn) {
    std::vector<float> t;
    for (int r = 0; r < 13; ++r) {
      CK(hipEventRecord(a, 0)); fn(); CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b)); if (r >= 3) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  };
  const double bytes = (double)n + nch;
  float t0 = timeit([&] { CK(launch_b64_encode(in, n, e1, c)); });
  float t1 = timeit([&] { hipLaunchKernelGGL((k_enc_lds<256>), dim3(units / 256), dim3(256), 0, 0, in, n, e2); });
  float t2 = timeit([&] { hipLaunchKernelGGL((k_enc_lds<1024>), dim3(units / 1024), dim3(1024), 0, 0, in, n, e2); });
  std::vector<char> h1(nch), h2(nch);
  CK(hipMemcpy(h1.data(), e1, nch, hipMemcpyDeviceToHost)); CK(hipMemcpy(h2.data(), e2, nch, hipMemcpyDeviceToHost));
  printf("encode product %.3f ms %.0f GB/s | lds256 %.3f ms %.0f GB/s | lds1024 %.3f ms %.0f GB/s | equal %d\n",
         t0, bytes / t0 / 1e6, t1, bytes / t1 / 1e6, t2, bytes / t2 / 1e6, !memcmp(h1.data(), h2.data(), nch));
  float d0 = timeit([&] { CK(launch_b64_decode(e1, nch, dec1, n, bad, c)); });
  float d1 = timeit([&] { hipLaunchKernelGGL((k_dec_lds<256>), dim3(units / 256), dim3(256), 0, 0, e1, dec2, bad); });
  float d2 = timeit([&] { hipLaunchKernelGGL((k_dec_lds<1024>), dim3(units / 1024), dim3(1024), 0, 0, e1, dec2, bad); });
  std::vector<uint8_t> g1(n), g2(n), g0(n);
  CK(hipMemcpy(g1.data(), dec1, n, hipMemcpyDeviceToHost)); CK(hipMemcpy(g2.data(), dec2, n, hipMemcpyDeviceToHost));
  CK(hipMemcpy(g0.data(), in, n, hipMemcpyDeviceToHost));
  unsigned long long hb; CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
  printf("decode product %.3f ms %.0f GB/s | lds256 %.3f ms %.0f GB/s | lds1024 %.3f ms %.0f GB/s | equal %d roundtrip %d bad %llx\n",
         d0, bytes / d0 / 1e6, d1, bytes / d1 / 1e6, d2, bytes / d2 / 1e6, !memcmp(g1.data(), g2.data(), n),
         !memcmp(g0.data(), g1.data(), n), hb);
  return 0;
}

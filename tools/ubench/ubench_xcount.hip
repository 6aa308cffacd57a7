// Exchange decode count pass (tool): the round-2 first count kernel (128
// lanes x 64 lane-contiguous bytes per 8 KiB span, one workgroup per span,
// "old") against one-wave-per-span variants (lane-interleaved 16-B loads, no
// barrier; the product's k_xdec_count is "wave x4"), on the same 8 Mi-pair
// text as ubench_xdec2.  Every variant's per-span counts are compared.
#include "../../amphora_amd/csrc/exchange.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace amph { namespace {
// one wave per 8 KiB span: 64 lanes x 128 bytes (eight 16-B loads in flight
// per lane), WPB waves per workgroup, no LDS, no barrier
template <int WPB>
__global__ __launch_bounds__(64 * WPB) void k_count_wave(Text t, uint64_t* bsum, size_t nb) {
  const size_t span = (size_t)blockIdx.x * WPB + (threadIdx.x >> 6);
  if (span >= nb) return;
  const size_t base = span * kDecSpan + (size_t)(threadIdx.x & 63) * 16;
  uint4 c[8];
  if (span * kDecSpan >= t.mis && (span + 1) * kDecSpan <= t.L) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(t.al + base + 1024 * k));
      c[k] = make_uint4(v.x, v.y, v.z, v.w);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = t.chunk((long long)(base + 1024 * k));
  }
  uint32_t cnt = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k)
    cnt += __popc(swar_colon(c[k].x)) + __popc(swar_colon(c[k].y)) + __popc(swar_colon(c[k].z)) +
           __popc(swar_colon(c[k].w));
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if ((threadIdx.x & 63) == 0) bsum[span] = cnt;
}

// the old layout: 128 lanes x 64 lane-contiguous bytes per span, one workgroup per span
__global__ __launch_bounds__(128) void k_count_old(Text t, uint64_t* bsum) {
  __shared__ uint32_t wsum[2];
  const size_t base = (size_t)blockIdx.x * kDecSpan + (size_t)threadIdx.x * 64;
  uint4 c[4];
  if (base >= t.mis && base + 64 <= t.L) {
    const u32x4* p = reinterpret_cast<const u32x4*>(t.al + base);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32x4 v = __builtin_nontemporal_load(p + k);
      c[k] = make_uint4(v.x, v.y, v.z, v.w);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = t.chunk((long long)base + 16 * k);
  }
  uint32_t cnt = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    cnt += __popc(swar_colon(c[k].x)) + __popc(swar_colon(c[k].y)) + __popc(swar_colon(c[k].z)) +
           __popc(swar_colon(c[k].w));
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if (__lane_id() == 0) wsum[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) bsum[blockIdx.x] = wsum[0] + wsum[1];
}

// the old layout (128 lanes x 64 B, lane-contiguous 64 B) but the two
// waves of a span reduce through one LDS atomic instead of a barrier
__global__ __launch_bounds__(256) void k_count_lane64(Text t, uint64_t* bsum, size_t nb) {
  const size_t span = (size_t)blockIdx.x * 2 + (threadIdx.x >> 7);
  if (span >= nb) return;
  const size_t base = span * kDecSpan + (size_t)(threadIdx.x & 127) * 64;
  uint4 c[4];
  if (span * kDecSpan >= t.mis && (span + 1) * kDecSpan <= t.L) {
    const u32x4* p = reinterpret_cast<const u32x4*>(t.al + base);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32x4 v = __builtin_nontemporal_load(p + k);
      c[k] = make_uint4(v.x, v.y, v.z, v.w);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) c[k] = t.chunk((long long)base + 16 * k);
  }
  uint32_t cnt = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    cnt += __popc(swar_colon(c[k].x)) + __popc(swar_colon(c[k].y)) + __popc(swar_colon(c[k].z)) +
           __popc(swar_colon(c[k].w));
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  __shared__ uint32_t wsum[4];
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if ((threadIdx.x & 127) == 0) bsum[span] = wsum[threadIdx.x >> 6] + wsum[(threadIdx.x >> 6) + 1];
}
}}  // namespace amph::(anon)

__global__ void k_fill(uint4* mag, uint8_t* neg, size_t nvals) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvals; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull + 12345, a = (x ^ (x >> 29)) * 0xBF58476D1CE4E5B9ull;
    uint64_t b = (a ^ (a >> 31)) * 0x94D049BB133111EBull;
    const int sh = (int)(i % 7) * 17;
    mag[i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> (33 + sh % 31)) >> (i % 7 == 3 ? 31 : 0));
    if (i % 11 == 5) mag[i] = make_uint4((uint32_t)(a % 1000), 0, 0, 0);
    neg[i] = (uint8_t)((b >> 40) & 1);
  }
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 20;
  const size_t npairs = (size_t)8 << 20, nvals = 2 * npairs;
  uint4* mag;
  uint8_t* neg;
  char* text;
  unsigned long long* len;
  CK(hipMalloc(&mag, nvals * 16));
  CK(hipMalloc(&neg, nvals));
  const size_t cap = xenc_max_bytes(npairs);
  CK(hipMalloc(&text, cap + 64));
  CK(hipMalloc(&len, 8));
  void* s1;
  CK(hipMalloc(&s1, xenc_scratch_bytes(npairs)));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, mag, neg, nvals);
  LaunchCfg c{0, 0, 256};
  CK(launch_exchange_encode(mag, neg, npairs, text, len, s1, c));
  unsigned long long L;
  CK(hipMemcpy(&L, len, 8, hipMemcpyDeviceToHost));
  const Text t{reinterpret_cast<const uint8_t*>(text), 0, L};
  const size_t nb = blocks_of(L, kDecSpan);
  printf("text %llu bytes, %zu spans\n", L, nb);
  uint64_t *b0, *b1;
  CK(hipMalloc(&b0, 8 * nb)); CK(hipMalloc(&b1, 8 * nb));
  std::vector<uint64_t> ref(nb), got(nb);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch, uint64_t* out) {
    std::vector<float> ts;
    for (int r = 0; r < R + 3; ++r) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    CK(hipMemcpy(got.data(), out, 8 * nb, hipMemcpyDeviceToHost));
    const bool same = out == b0 || got == ref;
    printf("  %-12s median %7.1f us  min %7.1f us  %5.2f TB/s  %s\n", name, ts[ts.size() / 2] * 1e3,
           ts[0] * 1e3, L / (ts[ts.size() / 2] * 1e-3) / 1e12, same ? "counts match" : "COUNTS DIFFER");
  };
  run("old", [&] { hipLaunchKernelGGL(k_count_old, dim3((unsigned)nb), dim3(128), 0, 0, t, b0); }, b0);
  CK(hipMemcpy(ref.data(), b0, 8 * nb, hipMemcpyDeviceToHost));
  run("product", [&] { hipLaunchKernelGGL(k_xdec_count, dim3((unsigned)blocks_of(nb, kCntWaves)), dim3(64 * kCntWaves), 0, 0, t, b1, nb); }, b1);
  run("wave x1", [&] { hipLaunchKernelGGL(k_count_wave<1>, dim3((unsigned)nb), dim3(64), 0, 0, t, b1, nb); }, b1);
  run("wave x4", [&] { hipLaunchKernelGGL(k_count_wave<4>, dim3((unsigned)blocks_of(nb, 4)), dim3(256), 0, 0, t, b1, nb); }, b1);
  run("wave x16", [&] { hipLaunchKernelGGL(k_count_wave<16>, dim3((unsigned)blocks_of(nb, 16)), dim3(1024), 0, 0, t, b1, nb); }, b1);
  run("lane64 x2", [&] { hipLaunchKernelGGL(k_count_lane64, dim3((unsigned)blocks_of(nb, 2)), dim3(256), 0, 0, t, b1, nb); }, b1);
  run("old", [&] { hipLaunchKernelGGL(k_count_old, dim3((unsigned)nb), dim3(128), 0, 0, t, b0); }, b0);
  return 0;
}

// Exchange encode length pass (tool): the product's k_xenc_bsum against a
// value-interleaved variant (each lane takes values, not pairs: consecutive
// lanes read consecutive 16-B magnitudes and sign bytes, so every wave
// instruction reads 1 KiB / 64 B contiguous; the per-pair constant text is
// added per sub-block).  Per-sub-block sums compared; whole encode timed.
#include "../../amphora_amd/csrc/exchange.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace amph { namespace {
__global__ __launch_bounds__(4 * kXBlock) void k_bsum_vals(const uint4* mag, const uint8_t* neg,
                                                          size_t npairs, size_t nb, uint64_t* bs) {
  __shared__ uint32_t ws[32];
  const size_t nvals = 2 * npairs;
  const size_t v0 = (size_t)blockIdx.x * (8 * kXBlock) + threadIdx.x, v1 = v0 + 4 * kXBlock;
  uint32_t l0 = 0, l1 = 0;
  if (v0 < nvals) {
    const uint4 d = mag[v0];
    l0 = ndigits128(d) + (neg[v0] != 0 && !is_zero(d));
  }
  if (v1 < nvals) {
    const uint4 d = mag[v1];
    l1 = ndigits128(d) + (neg[v1] != 0 && !is_zero(d));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    l0 += __shfl_xor(l0, o, 64);
    l1 += __shfl_xor(l1, o, 64);
  }
  if (__lane_id() == 0) {
    ws[threadIdx.x >> 6] = l0;
    ws[16 + (threadIdx.x >> 6)] = l1;
  }
  __syncthreads();
  const size_t sub = 4 * (size_t)blockIdx.x + threadIdx.x;
  if (threadIdx.x < 4 && sub < nb) {
    const uint32_t* w = ws + 8 * threadIdx.x;  // subs 0, 1: ws[0..15]; 2, 3: ws[16..31]
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += w[j];
    const size_t p0 = sub * kXBlock, np = min((size_t)kXBlock, npairs - p0);
    s += 12 * np - (p0 + np == npairs ? 1 : 0);  // {"a":,"b":} + ',' unless last
    bs[sub] = s;
  }
}
}}  // namespace amph::(anon)

__global__ void k_fill(uint4* mag, uint8_t* neg, size_t nvals) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvals; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull + 12345, a = (x ^ (x >> 29)) * 0xBF58476D1CE4E5B9ull;
    uint64_t b = (a ^ (a >> 31)) * 0x94D049BB133111EBull;
    const int sh = (int)(i % 7) * 17;
    mag[i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> (33 + sh % 31)) >> (i % 7 == 3 ? 31 : 0));
    if (i % 11 == 5) mag[i] = make_uint4((uint32_t)(a % 1000), 0, 0, 0);
    if (i % 13 == 7) mag[i] = make_uint4(0, 0, 0, 0);
    neg[i] = (uint8_t)((b >> 40) & 1);
  }
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 20;
  for (size_t npairs : {(size_t)8 << 20, (size_t)1000001}) {
    const size_t nvals = 2 * npairs;
    uint4* mag;
    uint8_t* neg;
    char* text;
    unsigned long long* len;
    CK(hipMalloc(&mag, nvals * 16));
    CK(hipMalloc(&neg, nvals));
    CK(hipMalloc(&text, xenc_max_bytes(npairs) + 64));
    CK(hipMalloc(&len, 8));
    void* s1;
    CK(hipMalloc(&s1, xenc_scratch_bytes(npairs)));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, mag, neg, nvals);
    const size_t nb = blocks_of(npairs, kXBlock);
    uint64_t *b0, *b1;
    CK(hipMalloc(&b0, 8 * nb)); CK(hipMalloc(&b1, 8 * nb));
    std::vector<uint64_t> ref(nb), got(nb);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    LaunchCfg c{0, 0, 256};
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
      const char* verdict = "";
      if (out) {
        CK(hipMemcpy(got.data(), out, 8 * nb, hipMemcpyDeviceToHost));
        verdict = out == b0 ? "(reference)" : got == ref ? "sums match" : "SUMS DIFFER";
      }
      printf("  %-14s median %7.1f us  min %7.1f us  %s\n", name, ts[ts.size() / 2] * 1e3, ts[0] * 1e3, verdict);
    };
    printf("npairs=%zu\n", npairs);
    run("bsum product", [&] { hipLaunchKernelGGL(k_xenc_bsum, dim3(blocks_of(nb, 4)), dim3(4 * kXBlock), 0, 0, mag, neg, npairs, nb, b0); }, b0);
    CK(hipMemcpy(ref.data(), b0, 8 * nb, hipMemcpyDeviceToHost));
    run("bsum values", [&] { hipLaunchKernelGGL(k_bsum_vals, dim3(blocks_of(nb, 4)), dim3(4 * kXBlock), 0, 0, mag, neg, npairs, nb, b1); }, b1);
    run("bsum product", [&] { hipLaunchKernelGGL(k_xenc_bsum, dim3(blocks_of(nb, 4)), dim3(4 * kXBlock), 0, 0, mag, neg, npairs, nb, b0); }, b0);
    run("encode (all)", [&] { CK(launch_exchange_encode(mag, neg, npairs, text, len, s1, c)); }, nullptr);
    CK(hipFree(mag)); CK(hipFree(neg)); CK(hipFree(text)); CK(hipFree(len)); CK(hipFree(s1));
    CK(hipFree(b0)); CK(hipFree(b1));
  }
  return 0;
}

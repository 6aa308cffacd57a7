// Where does the exchange-decode parse pass spend its time? (tool)
// 8 Mi FactorPairs of random 128-bit signed diffs are encoded on the GPU
// (launch_exchange_encode, Jackson's compact layout), then timed:
//   stage   each workgroup stages its 16 KiB window in LDS (and nothing else)
//   starts  + number starts per lane, block scan, LDS position list
//   parse   the product k_xdec_parse (count + scan done once beforehand)
#include "../../amphora_amd/csrc/exchange.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace amph { namespace {
template <int LEVEL>
__global__ __launch_bounds__(kDecBlock) void k_probe(Text text, unsigned long long* sink) {
  __shared__ uint4 win4[kWin / 16 + 1];
  __shared__ uint16_t pos[kMaxStarts];
  const size_t b0 = (size_t)blockIdx.x * kDecSpan;
  const long long w0 = (long long)b0 - kWinPad;
  for (int c = threadIdx.x; c < kWin / 16 + 1; c += kDecBlock) win4[c] = text.chunk(w0 + 16LL * c);
  __syncthreads();
  const uint8_t* win = reinterpret_cast<const uint8_t*>(win4);
  uint32_t acc;
  if constexpr (LEVEL == 0) {
    const int lo = kWinPad + kDecBytes * threadIdx.x;
    const uint4 c0 = win4[lo / 16], c1 = win4[lo / 16 + 1];
    acc = c0.x ^ c0.y ^ c0.z ^ c0.w ^ c1.x ^ c1.y ^ c1.z ^ c1.w;
  } else {
    const int lo = kWinPad + kDecBytes * threadIdx.x;
    const uint4 c0 = win4[lo / 16], c1 = win4[lo / 16 + 1];
    const uint32_t w[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    uint32_t m = starts32(w, swar_numchar((uint32_t)win[lo - 1] << 24));
    uint64_t total;
    const uint64_t first = block_excl_scan(__popc(m), &total);
    for (int k = (int)first; m; m &= m - 1, ++k) {
      const int at = kDecBytes * threadIdx.x + __ffs(m) - 1;
      if (k < kMaxStarts) pos[k] = (uint16_t)at;
    }
    __syncthreads();
    acc = pos[threadIdx.x % max((uint64_t)1, min(total, (uint64_t)kMaxStarts))];
  }
  if (acc == 0xFFFFFFFFu) atomicAdd(sink, 1ull);  // keeps the work live
}
}}  // namespace amph::(anon)

__global__ void k_fill_diffs(uint4* mag, uint8_t* neg, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull + 1, y = (x ^ (x >> 29)) * 0xBF58476D1CE4E5B9ull;
    mag[i] = make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 33));
    neg[i] = (uint8_t)(y & 1);
  }
}

int main() {
  const size_t npairs = (size_t)8 << 20, nvals = 2 * npairs;
  uint4 *mag, *mag2; uint8_t *neg, *neg2; char* text; void* scr; unsigned long long *len, *bad, *sink;
  CK(hipMalloc(&mag, nvals * 16)); CK(hipMalloc(&neg, nvals));
  CK(hipMalloc(&mag2, nvals * 16)); CK(hipMalloc(&neg2, nvals));
  CK(hipMalloc(&text, xenc_max_bytes(npairs))); CK(hipMalloc(&scr, xenc_scratch_bytes(npairs)));
  CK(hipMalloc(&len, 8)); CK(hipMalloc(&bad, 8)); CK(hipMalloc(&sink, 8));
  hipLaunchKernelGGL(k_fill_diffs, dim3(4096), dim3(256), 0, 0, mag, neg, nvals);
  LaunchCfg c{0, 0, 1024};
  CK(launch_exchange_encode(mag, neg, npairs, text, len, scr, c));
  unsigned long long L;
  CK(hipMemcpy(&L, len, 8, hipMemcpyDeviceToHost));
  printf("text %llu bytes for %zu pairs\n", L, npairs);
  const Text t{reinterpret_cast<const uint8_t*>(text), 0, (size_t)L};
  const size_t nb = (L + kDecSpan - 1) / kDecSpan;
  void* dscr;
  CK(hipMalloc(&dscr, xdec_scratch_bytes(L)));
  uint64_t* bscan = static_cast<uint64_t*>(dscr);
  uint64_t* bsum = bscan + nb + 1;
  CK(hipMemset(bad, 0x7F, 8));
  uint64_t* cnt2;  // the timed count pass writes here, not over the scanned prefix
  CK(hipMalloc(&cnt2, 8 * (nb + 1)));
  hipLaunchKernelGGL(k_xdec_count, dim3((unsigned)nb), dim3(kCntBlock), 0, 0, t, bscan);
  CK(scan_u64(bscan, nb, bsum, c));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char* names[] = {"stage", "starts", "parse", "count"};
  std::vector<float> ts[4];
  for (int r = 0; r < 23; ++r) for (int v = 0; v < 4; ++v) {
    CK(hipEventRecord(e0, 0));
    switch (v) {
      case 0: hipLaunchKernelGGL(k_probe<0>, dim3((unsigned)nb), dim3(kDecBlock), 0, 0, t, sink); break;
      case 1: hipLaunchKernelGGL(k_probe<1>, dim3((unsigned)nb), dim3(kDecBlock), 0, 0, t, sink); break;
      case 2: hipLaunchKernelGGL(k_xdec_parse, dim3((unsigned)nb), dim3(kDecBlock), 0, 0, t, bscan, nvals, mag2, neg2, bad); break;
      case 3: hipLaunchKernelGGL(k_xdec_count, dim3((unsigned)nb), dim3(kCntBlock), 0, 0, t, cnt2); break;
    }
    CK(hipGetLastError());
    CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 3) ts[v].push_back(ms);
  }
  unsigned long long hb;
  CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
  std::vector<uint4> a(1024), b(1024);
  CK(hipMemcpy(a.data(), mag, 1024 * 16, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), mag2, 1024 * 16, hipMemcpyDeviceToHost));
  bool same = true;
  for (int i = 0; i < 1024; ++i) same &= a[i].x == b[i].x && a[i].y == b[i].y && a[i].z == b[i].z && a[i].w == b[i].w;
  printf("bad=%llx first 1024 magnitudes round-trip=%d\n", hb, (int)same);
  for (int v = 0; v < 4; ++v) {
    std::sort(ts[v].begin(), ts[v].end());
    printf("  %-7s median %8.1f us\n", names[v], ts[v][ts[v].size() / 2] * 1e3);
  }
  return 0;
}

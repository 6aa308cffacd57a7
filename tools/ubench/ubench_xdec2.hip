// Exchange decode end to end (tool): 8 Mi FactorPairs of random 128-bit
// signed diffs encoded on the GPU (Jackson's compact layout), then the whole
// product launch_exchange_decode (count, scan, parse, check) timed; every
// decoded magnitude / sign compared with the encoder's input.
#ifndef XDEC_SRC
#define XDEC_SRC "../../amphora_amd/csrc/exchange.hip"
#endif
#include XDEC_SRC
#include <algorithm>
#include <cstdio>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_fill(uint4* mag, uint8_t* neg, size_t nvals, int full) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvals; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull + 12345, a = (x ^ (x >> 29)) * 0xBF58476D1CE4E5B9ull;
    uint64_t b = (a ^ (a >> 31)) * 0x94D049BB133111EBull;
    // magnitudes of assorted lengths (short ones every 7th), top bit clear
    const int sh = (int)(i % 7) * 17;
    mag[i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> (33 + sh % 31)) >> (i % 7 == 3 ? 31 : 0));
    if (i % 11 == 5) mag[i] = make_uint4((uint32_t)(a % 1000), 0, 0, 0);
    // full: |x - a| for x, a uniform below a 127-bit prime, as the party sends (38-39 digits)
    if (full) mag[i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32) >> 1);
    neg[i] = (uint8_t)((b >> 40) & 1);
  }
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 20;
  const int full = argc > 2 ? atoi(argv[2]) : 0;  // 1: full-length magnitudes (752 MB of text)
  const size_t npairs = (size_t)(argc > 3 ? atoi(argv[3]) : 8) << 20, nvals = 2 * npairs;  // argv[3]: Mi pairs
  uint4 *mag, *mag2;
  uint8_t *neg, *neg2;
  char* text;
  unsigned long long *len, *bad;
  CK(hipMalloc(&mag, nvals * 16)); CK(hipMalloc(&mag2, nvals * 16));
  CK(hipMalloc(&neg, nvals)); CK(hipMalloc(&neg2, nvals));
  const size_t cap = xenc_max_bytes(npairs);
  CK(hipMalloc(&text, cap + 64));
  CK(hipMalloc(&len, 8)); CK(hipMalloc(&bad, 8));
  void *s1, *s2;
  CK(hipMalloc(&s1, xenc_scratch_bytes(npairs)));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, mag, neg, nvals, full);
  LaunchCfg c{0, 0, 256};
  CK(launch_exchange_encode(mag, neg, npairs, text, len, s1, c));
  unsigned long long L;
  CK(hipMemcpy(&L, len, 8, hipMemcpyDeviceToHost));
  CK(hipMalloc(&s2, xdec_scratch_bytes(L)));
  printf("text %llu bytes for %zu pairs\n", L, npairs);
  {  // the encode that made it, timed the same way (text compared with the first run's)
    hipEvent_t f0, f1;
    CK(hipEventCreate(&f0)); CK(hipEventCreate(&f1));
    std::vector<char> ref(L), got(L);
    CK(hipMemcpy(ref.data(), text, L, hipMemcpyDeviceToHost));
    std::vector<float> te;
    for (int r = 0; r < R + 3; ++r) {
      CK(hipEventRecord(f0, 0));
      CK(launch_exchange_encode(mag, neg, npairs, text, len, s1, c));
      CK(hipEventRecord(f1, 0));
      CK(hipEventSynchronize(f1));
      float ms; CK(hipEventElapsedTime(&ms, f0, f1));
      if (r >= 3) te.push_back(ms);
    }
    unsigned long long L2;
    CK(hipMemcpy(&L2, len, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(got.data(), text, L, hipMemcpyDeviceToHost));
    std::sort(te.begin(), te.end());
    printf("encode %s, median %8.1f us  min %8.1f us  %6.2f TB/s of text\n",
           L2 == L && got == ref ? "text identical" : "TEXT DIFFERS", te[te.size() / 2] * 1e3, te[0] * 1e3,
           L / (te[te.size() / 2] * 1e-3) / 1e12);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<float> ts;
  for (int r = 0; r < R + 3; ++r) {
    CK(hipMemset(bad, 0x7F, 8));
    CK(hipEventRecord(e0, 0));
    CK(launch_exchange_decode(text, L, npairs, mag2, neg2, bad, s2, c));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 3) ts.push_back(ms);
  }
  std::vector<uint8_t> a(nvals * 16), b(nvals * 16), na(nvals), nb(nvals);
  CK(hipMemcpy(a.data(), mag, nvals * 16, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), mag2, nvals * 16, hipMemcpyDeviceToHost));
  CK(hipMemcpy(na.data(), neg, nvals, hipMemcpyDeviceToHost));
  CK(hipMemcpy(nb.data(), neg2, nvals, hipMemcpyDeviceToHost));
  size_t signs_bad = 0;
  for (size_t i = 0; i < nvals; ++i) {
    bool zero = true;
    for (int k = 0; k < 16; ++k) zero = zero && a[16 * i + k] == 0;
    if ((zero ? 0 : na[i]) != nb[i]) ++signs_bad;
  }
  unsigned long long hb;
  CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
  std::sort(ts.begin(), ts.end());
  printf("bad=%llx magnitudes %s, sign mismatches %zu\n", hb, a == b ? "identical" : "DIFFER", signs_bad);
  printf("decode median %8.1f us  min %8.1f us  %6.2f TB/s of text\n", ts[ts.size() / 2] * 1e3, ts[0] * 1e3,
         L / (ts[ts.size() / 2] * 1e-3) / 1e12);
  // the general pass: one '-' turned into a space (still valid JSON, one
  // value's sign flips) takes the whole text through k_xdec_slow
  std::vector<char> h(L);
  CK(hipMemcpy(h.data(), text, L, hipMemcpyDeviceToHost));
  size_t at = 0;
  while (at < L && h[at] != '-') ++at;
  const char sp = ' ';
  CK(hipMemcpy(text + at, &sp, 1, hipMemcpyHostToDevice));
  ts.clear();
  for (int r = 0; r < R + 3; ++r) {
    CK(hipMemset(bad, 0x7F, 8));
    CK(hipEventRecord(e0, 0));
    CK(launch_exchange_decode(text, L, npairs, mag2, neg2, bad, s2, c));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 3) ts.push_back(ms);
  }
  CK(hipMemcpy(b.data(), mag2, nvals * 16, hipMemcpyDeviceToHost));
  CK(hipMemcpy(nb.data(), neg2, nvals, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
  signs_bad = 0;
  for (size_t i = 0; i < nvals; ++i) {
    bool zero = true;
    for (int k = 0; k < 16; ++k) zero = zero && a[16 * i + k] == 0;
    if ((zero ? 0 : na[i]) != nb[i]) ++signs_bad;
  }
  std::sort(ts.begin(), ts.end());
  printf("general pass (a space at offset %zu): bad=%llx magnitudes %s, sign mismatches %zu (1 expected)\n", at, hb,
         a == b ? "identical" : "DIFFER", signs_bad);
  printf("decode median %8.1f us  min %8.1f us  %6.2f TB/s of text\n", ts[ts.size() / 2] * 1e3, ts[0] * 1e3,
         L / (ts[ts.size() / 2] * 1e-3) / 1e12);
  return 0;
}

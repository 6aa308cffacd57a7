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

// span form -> pair order (what k_open_post reads through its map window)
__global__ void k_unspan(XSpans x, size_t npairs, uint4* mag, uint8_t* neg) {
  const size_t k = (size_t)blockIdx.x * 128 + threadIdx.x;
  if (k >= npairs) return;
  const uint64_t tot = x.base[x.nb];
  const uint4 e = x.map[blockIdx.x];
  size_t sl[2];
  for (int h = 0; h < 2; ++h) {
    const size_t v = 2 * k + h, t = v - (size_t)blockIdx.x * 256;
    const uint32_t o1 = e.z & 0xFFFF, o2 = e.z >> 16;
    sl[h] = tot != 2 * npairs ? v
            : t < o1        ? (size_t)e.x * kXSpanSlots + e.y + t
            : t < o2        ? (size_t)(e.x + 1) * kXSpanSlots + t - o1
            : t < e.w       ? (size_t)(e.x + 2) * kXSpanSlots + t - o2
                            : ~(size_t)0;
  }
  if (sl[0] == ~(size_t)0 || sl[1] == ~(size_t)0) { neg[2 * k] = 0xEE; return; }  // (counted as mismatches)
  const size_t a = sl[0], b = sl[1];
  const bool sw = (x.neg[a] & 2) != 0;
  mag[2 * k] = sw ? x.mag[b] : x.mag[a];
  mag[2 * k + 1] = sw ? x.mag[a] : x.mag[b];
  neg[2 * k] = (sw ? x.neg[b] : x.neg[a]) & 1;
  neg[2 * k + 1] = (sw ? x.neg[a] : x.neg[b]) & 1;
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
  {  // the span form (one read of the text; the party session's partner decode)
    XSpans x{};
    x.nb = xspan_spans(L);
    const size_t slots = xspan_slots(L, npairs);
    CK(hipMalloc(&x.mag, slots * 16)); CK(hipMalloc(&x.neg, slots));
    CK(hipMalloc(&x.base, 8 * (x.nb + 1))); CK(hipMalloc(&x.map, 16 * xspan_map_words(npairs)));
    void* s3;
    CK(hipMalloc(&s3, xdec_spans_scratch_bytes(L)));
    std::vector<float> tsp;
    for (int r = 0; r < R + 3; ++r) {
      CK(hipMemset(bad, 0x7F, 8));
      CK(hipEventRecord(e0, 0));
      CK(launch_exchange_decode_spans(text, L, npairs, x, bad, s3, c));
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) tsp.push_back(ms);
    }
#ifdef XDEC_STAMPS
    {  // one more span decode with per-block phase clocks (thread 0 of each workgroup)
      unsigned long long* st;
      CK(hipMalloc(&st, 8 * 8 * x.nb));
      CK(hipMemset(st, 0, 8 * 8 * x.nb));
      CK(hipMemcpyToSymbol(HIP_SYMBOL(g_xstamps), &st, sizeof(st)));
      CK(hipMemset(bad, 0x7F, 8));
      CK(launch_exchange_decode_spans(text, L, npairs, x, bad, s3, c));
      CK(hipDeviceSynchronize());
      unsigned long long* none = nullptr;
      CK(hipMemcpyToSymbol(HIP_SYMBOL(g_xstamps), &none, sizeof(none)));
      std::vector<unsigned long long> h(8 * x.nb);
      CK(hipMemcpy(h.data(), st, 8 * 8 * x.nb, hipMemcpyDeviceToHost));
      double sum[6] = {0};
      size_t cntb = 0;
      for (size_t b = 1; b + 1 < x.nb; ++b) {
        const unsigned long long* t = &h[8 * b];
        if (!t[0] || !t[5]) continue;
        for (int i = 1; i <= 5; ++i) sum[i] += (double)(t[i] - t[i - 1]);
        ++cntb;
      }
      printf("stamps (clock64 cycles per workgroup, mean over %zu): staging %.0f, colons+scan %.0f, pos+barrier %.0f, "
             "parse (wave 0) %.0f, final barrier %.0f, total %.0f\n", cntb, sum[1] / cntb, sum[2] / cntb, sum[3] / cntb,
             sum[4] / cntb, sum[5] / cntb, (sum[1] + sum[2] + sum[3] + sum[4] + sum[5]) / cntb);
      CK(hipFree(st));
    }
#endif
    CK(hipMemset(mag2, 0, nvals * 16)); CK(hipMemset(neg2, 0, nvals));
    hipLaunchKernelGGL(k_unspan, dim3((unsigned)((npairs + 127) / 128)), dim3(128), 0, 0, x, npairs, mag2, neg2);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(b.data(), mag2, nvals * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(nb.data(), neg2, nvals, hipMemcpyDeviceToHost));
    unsigned long long hb2, tot;
    CK(hipMemcpy(&hb2, bad, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&tot, x.base + x.nb, 8, hipMemcpyDeviceToHost));
    size_t sb = 0;
    for (size_t i = 0; i < nvals; ++i) {
      bool zero = true;
      for (int k = 0; k < 16; ++k) zero = zero && a[16 * i + k] == 0;
      if ((zero ? 0 : na[i]) != nb[i]) ++sb;
    }
    std::sort(tsp.begin(), tsp.end());
    printf("spans: bad=%llx total=%llx (%s) magnitudes %s, sign mismatches %zu\n", hb2, tot,
           tot == nvals ? "span form" : "pair order", a == b ? "identical" : "DIFFER", sb);
    printf("decode_spans median %8.1f us  min %8.1f us  %6.2f TB/s of text\n", tsp[tsp.size() / 2] * 1e3,
           tsp[0] * 1e3, L / (tsp[tsp.size() / 2] * 1e-3) / 1e12);
    CK(hipFree(x.mag)); CK(hipFree(x.neg)); CK(hipFree(x.base)); CK(hipFree(x.map)); CK(hipFree(s3));
  }
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

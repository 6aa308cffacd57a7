// Exchange decode of TWO texts (tool): can the count pass of one overlap the
// compact pass of the other?  The party decodes N-1 partner texts; the count
// pass is HBM-bound (6.7 TB/s) and the compact pass latency-bound (~4.7 TB/s
// of its own traffic), so the second text's count may hide in the first's
// compact pass.  Times, on 8 Mi full-length FactorPairs per text:
//   seq   - both decodes on one stream (today's party path)
//   conc  - text B's decode on a second stream, launched together
//   stag  - text B's count + scan on a second stream after text A's scan, its
//           compact pass after text A's (the overlap the party could schedule)
// Every result compared with the encoder's input.
#include "../../amphora_amd/csrc/exchange.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void k_fill(uint4* mag, uint8_t* neg, size_t nvals) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvals; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull + 12345, a = (x ^ (x >> 29)) * 0xBF58476D1CE4E5B9ull;
    uint64_t b = (a ^ (a >> 31)) * 0x94D049BB133111EBull;
    mag[i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32) >> 1);
    neg[i] = (uint8_t)((b >> 40) & 1);
  }
}

struct Dec {
  uint4* mag;
  uint8_t* neg;
  unsigned long long* bad;
  void* scratch;
};

// launch_exchange_decode split at its scan: front = count + scan, back = compact,
// general and check passes (the same launches, in the same order)
static void front(const char* text, size_t len, const Dec& d, hipStream_t s) {
  const size_t mis = (uintptr_t)text & 15;
  const Text t{reinterpret_cast<const uint8_t*>(text) - mis, mis, mis + len};
  const size_t nb = blocks_of(t.L, kDecSpan);
  LaunchCfg c{s, 0, 256};
  uint64_t* bscan = static_cast<uint64_t*>(d.scratch);
  uint64_t* bsum = bscan + nb + 1;
  unsigned int* slow = reinterpret_cast<unsigned int*>(bsum + blocks_of(nb, kScanBlock) + 1);
  AMPH_LAUNCH(k_xdec_count, dim3(blocks_of(nb, kCntWaves)), dim3(64 * kCntWaves), c, t, bscan, nb, slow);
  CK(scan_u64(bscan, nb, bsum, c));
}
static void back(const char* text, size_t len, size_t npairs, const Dec& d, hipStream_t s) {
  const size_t mis = (uintptr_t)text & 15;
  const Text t{reinterpret_cast<const uint8_t*>(text) - mis, mis, mis + len};
  const size_t nb = blocks_of(t.L, kDecSpan);
  LaunchCfg c{s, 0, 256};
  uint64_t* bscan = static_cast<uint64_t*>(d.scratch);
  uint64_t* bsum = bscan + nb + 1;
  unsigned int* slow = reinterpret_cast<unsigned int*>(bsum + blocks_of(nb, kScanBlock) + 1);
  AMPH_LAUNCH(k_xdec_fast, dim3((unsigned)nb), dim3(kDecBlock), c, t, bscan, nb, 2 * npairs, d.mag, d.neg, slow);
  AMPH_LAUNCH(k_xdec_slow<ScanBases>, dim3((unsigned)std::min<size_t>(nb, kSlowGrid)), dim3(kDecBlock), c, t,
              ScanBases{bscan, nb}, nb, 2 * npairs, d.mag, d.neg, d.bad, (const unsigned int*)slow);
  AMPH_LAUNCH(k_xdec_check<ScanTotal>, dim3(1), dim3(256), c, t, ScanTotal{bscan, nb}, 2 * npairs, d.bad);
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 20;
  const size_t npairs = (size_t)(argc > 2 ? atoi(argv[2]) : 8) << 20, nvals = 2 * npairs;
  uint4* mag;
  uint8_t* neg;
  CK(hipMalloc(&mag, nvals * 16)); CK(hipMalloc(&neg, nvals));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, mag, neg, nvals);
  char *ta, *tb;
  unsigned long long* len;
  CK(hipMalloc(&ta, xenc_max_bytes(npairs) + 64)); CK(hipMalloc(&tb, xenc_max_bytes(npairs) + 64));
  CK(hipMalloc(&len, 8));
  void* s1;
  CK(hipMalloc(&s1, xenc_scratch_bytes(npairs)));
  LaunchCfg c{0, 0, 256};
  CK(launch_exchange_encode(mag, neg, npairs, ta, len, s1, c));
  CK(launch_exchange_encode(mag, neg, npairs, tb, len, s1, c));
  unsigned long long L;
  CK(hipMemcpy(&L, len, 8, hipMemcpyDeviceToHost));
  Dec d[2];
  for (auto& x : d) {
    CK(hipMalloc(&x.mag, nvals * 16)); CK(hipMalloc(&x.neg, nvals));
    CK(hipMalloc(&x.bad, 8)); CK(hipMalloc(&x.scratch, xdec_scratch_bytes(L)));
  }
  printf("two texts of %llu bytes, %zu pairs each\n", L, npairs);
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  hipEvent_t e0, e1, fa, fb, ready;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  CK(hipEventCreateWithFlags(&fa, hipEventDisableTiming)); CK(hipEventCreateWithFlags(&fb, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
  std::vector<uint8_t> want(nvals * 16), got(nvals * 16);
  std::vector<uint8_t> wneg(nvals), gneg(nvals);
  CK(hipMemcpy(want.data(), mag, nvals * 16, hipMemcpyDeviceToHost));
  CK(hipMemcpy(wneg.data(), neg, nvals, hipMemcpyDeviceToHost));
  const char* modes[] = {"seq", "conc", "stag"};
  for (int m = 0; m < 3; ++m) {
    std::vector<float> ts;
    for (int r = 0; r < R + 3; ++r) {
      for (auto& x : d) {
        CK(hipMemsetAsync(x.bad, 0x7F, 8, sa));
        CK(hipMemsetAsync(x.mag, 0, nvals * 16, sa));
      }
      CK(hipEventRecord(e0, sa));
      CK(hipStreamWaitEvent(sb, e0, 0));
      if (m == 0) {
        front(ta, L, d[0], sa); back(ta, L, npairs, d[0], sa);
        front(tb, L, d[1], sa); back(tb, L, npairs, d[1], sa);
      } else if (m == 1) {
        front(ta, L, d[0], sa); back(ta, L, npairs, d[0], sa);
        front(tb, L, d[1], sb); back(tb, L, npairs, d[1], sb);
      } else {
        front(ta, L, d[0], sa);
        CK(hipEventRecord(fa, sa));
        back(ta, L, npairs, d[0], sa);
        CK(hipStreamWaitEvent(sb, fa, 0));  // B's count overlaps A's compact pass
        front(tb, L, d[1], sb);
        CK(hipEventRecord(ready, sa));      // A done
        CK(hipStreamWaitEvent(sb, ready, 0));
        back(tb, L, npairs, d[1], sb);
      }
      CK(hipEventRecord(fb, sb));
      CK(hipStreamWaitEvent(sa, fb, 0));
      CK(hipEventRecord(e1, sa));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) ts.push_back(ms);
    }
    bool ok = true;
    for (auto& x : d) {
      unsigned long long hb;
      CK(hipMemcpy(&hb, x.bad, 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(got.data(), x.mag, nvals * 16, hipMemcpyDeviceToHost));
      CK(hipMemcpy(gneg.data(), x.neg, nvals, hipMemcpyDeviceToHost));
      ok = ok && hb == 0x7F7F7F7F7F7F7F7Full && got == want;
      for (size_t i = 0; ok && i < nvals; ++i) ok = gneg[i] == wneg[i];
    }
    std::sort(ts.begin(), ts.end());
    printf("%-4s two decodes median %8.1f us  min %8.1f us  %6.2f TB/s of text  %s\n", modes[m],
           ts[ts.size() / 2] * 1e3, ts[0] * 1e3, 2.0 * L / (ts[ts.size() / 2] * 1e-3) / 1e12,
           ok ? "exact" : "MISMATCH");
  }
  return 0;
}

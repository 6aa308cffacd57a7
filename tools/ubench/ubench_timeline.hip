// Timeline of one C2 K_MASK launch (1 Mi words, 2 parties, 1024 workgroups
// of 1024 threads): every workgroup records s_memrealtime (100 MHz) when its
// first wave starts and when its last wave is done, so the launch's ramp
// (first -> last workgroup start), the per-workgroup durations and the tail
// (last workgroup end vs the bulk) can be read off (tool, not product).
// The body is the product's k_mask<2, true> for one word per thread.
#include "../../amphora_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace amph { namespace {
__global__ __launch_bounds__(1024) void k_mask_tl(OdoSet odo, size_t words, const uint4* secrets,
                                                  uint4* out, unsigned long long* ff, Fp f,
                                                  unsigned long long* ts) {
  __shared__ unsigned long long t_first;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) t_first = t0;
  const size_t i = (size_t)blockIdx.x * 1024 + threadIdx.x;
  const W4 r2 = r2_word(f);
  if (i < words) {
    const uint4 s = ld(secrets + i);
    W4 a[5];
    recombine5<2, true>(odo, 2, i, f, a);
    const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
    st(out + i, mod_sub(mont_mul(w4(s), r2, f), a[0], f));
    report_fail(!ok, i, ff);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    ts[2 * blockIdx.x] = t_first;
    ts[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  }
}
}}  // namespace amph::(anon)

__global__ void k_init(uint4* buf, size_t W, int n, Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < W; i += stride) {
    auto hr = [&](uint64_t x) {
      x = x * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
      uint64_t a = (x ^ (x >> 29)) * 0x94D049BB133111EBull, b = (x * 0xBF58476D1CE4E5B9ull) ^ (x >> 31);
      return canon<true>(W4{{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)}}, f);
    };
    W4 v[5];
    for (int k = 0; k < 3; ++k) v[k] = hr(i * 64 + k);
    v[3] = mont_mul(v[0], v[1], f);
    v[4] = mont_mul(v[2], v[1], f);
    for (int k = 0; k < 5; ++k) {
      W4 rest = v[k];
      for (int j = 0; j < n - 1; ++j) {
        const W4 s0 = hr(i * 64 + 8 + k * 8 + j);
        buf[(size_t)(k * n + j) * W + i] = u4(s0);
        rest = mod_sub(rest, s0, f);
      }
      buf[(size_t)(k * n + n - 1) * W + i] = u4(rest);
    }
    buf[(size_t)5 * n * W + i] = u4(hr(i * 64 + 60));
  }
}

int main() {
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = p[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu; f.big = 1;
  const int n = 2;
  const size_t W = (size_t)1 << 20, G = W / 1024;
  uint4* buf;
  CK(hipMalloc(&buf, (size_t)(5 * n + 2) * W * 16));
  hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, buf, W, n, f);
  OdoSet odo{};
  for (int k = 0; k < 5; ++k) for (int j = 0; j < n; ++j) odo.f[k][j] = buf + (size_t)(k * n + j) * W;
  const uint4* sec = buf + (size_t)5 * n * W;
  uint4* out = buf + (size_t)(5 * n + 1) * W;
  unsigned long long *ff, *ts;
  CK(hipMalloc(&ff, 8)); CK(hipMemset(ff, 0x7f, 8));
  CK(hipMalloc(&ts, 16 * G));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<unsigned long long> h(2 * G);
  for (int rep = 0; rep < 6; ++rep) {
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k_mask_tl, dim3((unsigned)G), dim3(1024), 0, 0, odo, W, sec, out, ff, f, ts);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpy(h.data(), ts, 16 * G, hipMemcpyDeviceToHost));
    if (rep < 2) continue;
    unsigned long long s0 = ~0ull, s1 = 0, e_min = ~0ull, e1m = 0;
    std::vector<double> starts, ends, durs;
    for (size_t b = 0; b < G; ++b) { s0 = std::min(s0, h[2 * b]); s1 = std::max(s1, h[2 * b]); e1m = std::max(e1m, h[2 * b + 1]); e_min = std::min(e_min, h[2 * b + 1]); }
    for (size_t b = 0; b < G; ++b) {
      starts.push_back((h[2 * b] - s0) * 0.01);
      ends.push_back((h[2 * b + 1] - s0) * 0.01);
      durs.push_back((h[2 * b + 1] - h[2 * b]) * 0.01);
    }
    std::vector<double> ss = starts, ee = ends, dd = durs;
    std::sort(ss.begin(), ss.end()); std::sort(ee.begin(), ee.end()); std::sort(dd.begin(), dd.end());
    auto q = [](const std::vector<double>& v, double x) { return v[(size_t)(x * (v.size() - 1))]; };
    printf("rep %d event %.2f us | wg starts: p0 %.2f p25 %.2f p50 %.2f p75 %.2f p100 %.2f | ends: p0 %.2f p50 %.2f p90 %.2f p99 %.2f p100 %.2f | dur p0 %.2f p50 %.2f p100 %.2f us\n",
           rep, ms * 1e3, q(ss, 0), q(ss, .25), q(ss, .5), q(ss, .75), q(ss, 1), q(ee, 0), q(ee, .5), q(ee, .9), q(ee, .99), q(ee, 1),
           q(dd, 0), q(dd, .5), q(dd, 1));
    if (rep == 5) {  // first / second round of workgroups: starts histogram in 2 us bins
      int hist[40] = {0};
      for (double s : starts) hist[std::min(39, (int)(s / 2))]++;
      printf("start histogram (2 us bins):");
      for (int k = 0; k < 40; ++k) printf(" %d", hist[k]);
      printf("\n");
    }
  }
  return 0;
}

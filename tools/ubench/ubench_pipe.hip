// A/B (tool): K_MASK as in the product (one word per lane, full grid, all
// loads then all arithmetic per wave) against (a) amph_stream_probe, the
// same memory pattern with no arithmetic, and (b) a persistent,
// register-double-buffered K_MASK: each lane walks words i, i + stride, ...
// and issues the next word's 5N + 1 loads before the current word's
// arithmetic, so a wave's compute overlaps its own next loads instead of
// holding its slot with nothing in flight.  Outputs compared bytewise.
#include "../../amphora_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace amph { namespace {
template <int NP, int BS>
__global__ __launch_bounds__(BS) void k_mask_pipe(OdoSet odo, size_t words, const uint4* secrets,
                                                 uint4* out, unsigned long long* ff, Fp f) {
  const size_t stride = (size_t)gridDim.x * BS;
  size_t i = (size_t)blockIdx.x * BS + threadIdx.x;
  if (i >= words) return;
  const W4 r2 = r2_word(f);
  uint4 nraw[5][NP], ns;
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int j = 0; j < NP; ++j) nraw[k][j] = ld(odo.f[k][j] + i);
  ns = ld(secrets + i);
  for (; i < words; i += stride) {
    uint4 raw[5][NP];
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int j = 0; j < NP; ++j) raw[k][j] = nraw[k][j];
    const uint4 s = ns;
    const size_t nx = min(i + stride, words - 1);  // unconditional: no branch around the loads
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int j = 0; j < NP; ++j) nraw[k][j] = ld(odo.f[k][j] + nx);
    ns = ld(secrets + nx);
    W4 a[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      a[k] = canon<true>(w4(raw[k][0]), f);
#pragma unroll
      for (int j = 1; j < NP; ++j) a[k] = mod_add(a[k], canon<true>(w4(raw[k][j]), f), f);
    }
    const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
    st(out + i, mod_sub(mont_mul(w4(s), r2, f), a[0], f));
    report_fail(!ok, i, ff);
  }
}
}}  // namespace amph::(anon)

__global__ void k_init(uint4* buf, size_t W, int n, Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < W; i += stride) {
    W4 v[5];
    auto hr = [&](uint64_t x) {
      x = x * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
      uint64_t a = (x ^ (x >> 29)) * 0x94D049BB133111EBull, b = (x * 0xBF58476D1CE4E5B9ull) ^ (x >> 31);
      return canon<true>(W4{{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)}}, f);
    };
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

static Fp test_fp() {
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = p[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu;
  f.big = 1;
  return f;
}

template <int NP, int BS>
static void launch_pipe(const OdoSet& odo, size_t W, const uint4* sec, uint4* out, unsigned long long* ff,
                        Fp f, unsigned grid) {
  hipLaunchKernelGGL((k_mask_pipe<NP, BS>), dim3(grid), dim3(BS), 0, 0, odo, W, sec, out, ff, f);
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 20;
  Fp f = test_fp();
  struct Cfg { int n; size_t W; };
  for (Cfg cf : {Cfg{2, (size_t)1 << 20}, Cfg{2, (size_t)1 << 24}, Cfg{3, (size_t)1 << 24}}) {
    const int n = cf.n;
    const size_t W = cf.W;
    uint4* buf;
    CK(hipMalloc(&buf, (size_t)(5 * n + 3) * W * 16));
    hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, buf, W, n, f);
    CK(hipDeviceSynchronize());
    OdoSet odo{};
    for (int k = 0; k < 5; ++k) for (int j = 0; j < n; ++j) odo.f[k][j] = buf + (size_t)(k * n + j) * W;
    const uint4* sec = buf + (size_t)5 * n * W;
    uint4* out0 = buf + (size_t)(5 * n + 1) * W;
    uint4* out1 = buf + (size_t)(5 * n + 2) * W;
    unsigned long long* ff;
    CK(hipMalloc(&ff, 64 * 8));
    CK(hipMemset(ff, 0x7f, 64 * 8));
    // variants: 0 product, 1 probe, then pipe with (block, grid)
    struct PV { int bs; unsigned grid; };
    std::vector<PV> pv = {{256, 256 * 8}, {256, 256 * 12}, {256, 256 * 16}, {256, 256 * 24},
                          {512, 256 * 4}, {512, 256 * 8}, {1024, 256 * 2}, {1024, 256 * 4}};
    const int NV = 2 + (int)pv.size();
    std::vector<std::vector<float>> t(NV);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int r = 0; r < R + 3; ++r) for (int v = 0; v < NV; ++v) {
      LaunchCfg c{0, 0, 1024};
      CK(hipEventRecord(e0, 0));
      if (v == 0) CK(launch_mask_input(odo, n, W, sec, W, out0, ff, f, c));
      else if (v == 1) CK(launch_stream_probe(odo, n, W, sec, out1, c));
      else {
        const PV p = pv[v - 2];
        const unsigned g = (unsigned)std::min<size_t>(p.grid, (W + p.bs - 1) / p.bs);
        if (n == 2) {
          if (p.bs == 256) launch_pipe<2, 256>(odo, W, sec, out1, ff + v, f, g);
          else if (p.bs == 512) launch_pipe<2, 512>(odo, W, sec, out1, ff + v, f, g);
          else launch_pipe<2, 1024>(odo, W, sec, out1, ff + v, f, g);
        } else {
          if (p.bs == 256) launch_pipe<3, 256>(odo, W, sec, out1, ff + v, f, g);
          else if (p.bs == 512) launch_pipe<3, 512>(odo, W, sec, out1, ff + v, f, g);
          else launch_pipe<3, 1024>(odo, W, sec, out1, ff + v, f, g);
        }
        CK(hipGetLastError());
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) t[v].push_back(ms);
      if (r == R + 2 && v >= 2) {  // compare the last pipe output with the product's
        std::vector<uint8_t> a(W * 16), b(W * 16);
        CK(hipMemcpy(a.data(), out0, W * 16, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), out1, W * 16, hipMemcpyDeviceToHost));
        if (a != b) printf("  variant %d output DIFFERS\n", v);
      }
    }
    unsigned long long h[64];
    CK(hipMemcpy(h, ff, 64 * 8, hipMemcpyDeviceToHost));
    printf("N=%d W=%zu ff0=%llx\n", n, W, h[0]);
    for (int v = 0; v < NV; ++v) {
      std::sort(t[v].begin(), t[v].end());
      const double bytes = (80.0 * n + 32) * W, med = t[v][t[v].size() / 2];
      char name[64];
      if (v == 0) snprintf(name, sizeof name, "product k_mask");
      else if (v == 1) snprintf(name, sizeof name, "stream_probe");
      else snprintf(name, sizeof name, "pipe bs=%d grid=%u", pv[v - 2].bs, pv[v - 2].grid);
      printf("  %-24s median %9.2f us  min %9.2f us  %7.1f GB/s%s\n", name, med * 1e3, t[v][0] * 1e3,
             bytes / (med * 1e-3) / 1e9, (v >= 2 && h[v] != 0x7f7f7f7f7f7f7f7full) ? "  FF SET" : "");
    }
    CK(hipFree(buf)); CK(hipFree(ff));
  }
  return 0;
}

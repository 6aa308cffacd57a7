// A/B of the product kernels (kernels.hip, included) against hand variants
// at 16 Mi and 64 Mi words, N = 2 and 3 (tool, not product).
#include "../../amphora_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace amph { namespace {
// variant: unconditional secret load first, plain per-lane atomic on failure
template <int NP>
__global__ __launch_bounds__(1024) void k_mask_b(OdoSet odo, size_t words, const uint4* secrets,
                                                uint4* out, unsigned long long* ff, Fp f) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= words) return;
  const uint4 s = ld(secrets + i);
  W4 a[5];
  recombine5<NP, true>(odo, NP, i, f, a);
  const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
  st(out + i, mod_sub(mont_mul(w4(s), r2_word(f), f), a[0], f));
  if (!ok) atomicMin(ff, (unsigned long long)i);
}
// variant: party-major accumulation (lower register pressure)
template <int NP>
__global__ __launch_bounds__(1024) void k_mask_c(OdoSet odo, size_t words, const uint4* secrets,
                                                uint4* out, unsigned long long* ff, Fp f) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= words) return;
  const uint4 s = ld(secrets + i);
  W4 a[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) a[k] = canon<true>(w4(ld(odo.f[k][0] + i)), f);
#pragma unroll
  for (int j = 1; j < NP; ++j) {
    uint4 raw[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) raw[k] = ld(odo.f[k][j] + i);
#pragma unroll
    for (int k = 0; k < 5; ++k) a[k] = mod_add(a[k], canon<true>(w4(raw[k]), f), f);
  }
  const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
  st(out + i, mod_sub(mont_mul(w4(s), r2_word(f), f), a[0], f));
  if (!ok) atomicMin(ff, (unsigned long long)i);
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

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 15;
  Fp f = test_fp();
  const int n = 2;
  for (size_t W : {(size_t)1 << 24, (size_t)1 << 26}) {
    for (size_t pad : {(size_t)0, (size_t)4096, (size_t)65536 + 256, (size_t)(2 << 20), (size_t)(2 << 20) + 4096 * 3}) {
      const size_t stride = W * 16 + pad;  // bytes between consecutive arrays
      char* base;
      CK(hipMalloc(&base, (size_t)(5 * n + 2) * stride));
      uint4* tmp;
      CK(hipMalloc(&tmp, (size_t)(5 * n + 2) * W * 16));
      hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, tmp, W, n, f);
      CK(hipDeviceSynchronize());
      for (int a = 0; a < 5 * n + 2; ++a)
        CK(hipMemcpy(base + a * stride, tmp + (size_t)a * W, W * 16, hipMemcpyDeviceToDevice));
      CK(hipFree(tmp));
      OdoSet odo{};
      for (int k = 0; k < 5; ++k) for (int j = 0; j < n; ++j) odo.f[k][j] = (const uint4*)(base + (k * n + j) * stride);
      const uint4* sec = (const uint4*)(base + 5 * n * stride);
      uint4* out = (uint4*)(base + (5 * n + 1) * stride);
      unsigned long long* ff;
      CK(hipMalloc(&ff, 64));
      CK(hipMemset(ff, 0x7f, 64));
      std::vector<float> tm, tr;
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
      for (int r = 0; r < R + 3; ++r) for (int v = 0; v < 2; ++v) {
        LaunchCfg c{0, 0, 1024};
        CK(hipEventRecord(e0, 0));
        if (v == 0) launch_mask_input(odo, n, W, sec, W, out, ff, f, c);
        else launch_recombine_verify(odo, n, W, out, ff + 1, f, c);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) (v == 0 ? tm : tr).push_back(ms);
      }
      std::sort(tm.begin(), tm.end()); std::sort(tr.begin(), tr.end());
      unsigned long long h[2];
      CK(hipMemcpy(h, ff, 16, hipMemcpyDeviceToHost));
      printf("W=%zu pad=%zu ff=%llx/%llx  mask %8.1f us %6.1f GB/s   rv %8.1f us %6.1f GB/s\n", W, pad, h[0], h[1],
             tm[tm.size() / 2] * 1e3, 192.0 * W / (tm[tm.size() / 2] * 1e-3) / 1e9,
             tr[tr.size() / 2] * 1e3, 176.0 * W / (tr[tr.size() / 2] * 1e-3) / 1e9);
      CK(hipFree(base)); CK(hipFree(ff));
    }
  }
  return 0;
}

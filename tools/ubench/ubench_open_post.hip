// A/B (tool): recombineDiffs + K_ODO_POST as two launches (k_open, then
// k_odo_post; the opened values go through HBM) against the fused
// k_open_post, with each party's diff pairs loaded per lane (32-B stride) or
// staged through LDS.  Outputs compared bytewise.  16 Mi and 1 Mi words,
// N = 2 and 3.
#include "../../amphora_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static Fp test_fp() {
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = p[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu;
  f.big = 1;
  return f;
}

__global__ void k_fill(uint4* b, size_t n, Fp f, uint64_t salt) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = (i + salt) * 0x9E3779B97F4A7C15ull + 77, y = (x ^ (x >> 31)) * 0xBF58476D1CE4E5B9ull;
    W4 w = canon<true>(W4{{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 33)}}, f);
    if (i % 7 == 3) {
      W4 t; uint32_t c;
      t.v[0] = addc(w.v[0], f.p[0], 0, &c); t.v[1] = addc(w.v[1], f.p[1], c, &c);
      t.v[2] = addc(w.v[2], f.p[2], c, &c); t.v[3] = addc(w.v[3], f.p[3], c, &c);
      if (!c) w = t;
    }
    b[i] = u4(w);
  }
}
__global__ void k_signs(uint8_t* s, size_t n, uint64_t salt) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s[i] = (uint8_t)((((i + salt) * 0x9E3779B97F4A7C15ull) >> 61) & 1);
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 20;
  Fp f = test_fp();
  for (int n : {2, 3}) for (size_t W : {(size_t)1 << 24, (size_t)1 << 20}) {
    const size_t vals = 4 * W;
    SignedSet d{};
    std::vector<void*> allocs;
    for (int j = 0; j < n; ++j) {
      uint4* m; uint8_t* s;
      CK(hipMalloc(&m, vals * 16)); CK(hipMalloc(&s, vals));
      hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, m, vals, f, (uint64_t)j * 1000003);
      hipLaunchKernelGGL(k_signs, dim3(2048), dim3(256), 0, 0, s, vals, (uint64_t)j * 7919);
      d.mag[j] = m; d.neg[j] = (const uint32_t*)s;
      allocs.push_back(m); allocs.push_back(s);
    }
    uint4 *tri, *opened, *o[6];
    CK(hipMalloc(&tri, 12 * W * 16)); CK(hipMalloc(&opened, vals * 16));
    for (auto& p : o) CK(hipMalloc(&p, W * 16));
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, tri, 12 * W, f, 555);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const char* names[] = {"open+post", "fused_direct", "fused_lds"};
    std::vector<float> t[3];
    for (int p0 = 0; p0 < 2; ++p0) {
      for (auto& v : t) v.clear();
      for (int r = 0; r < R + 3; ++r) for (int v = 0; v < 3; ++v) {
        LaunchCfg c{0, 0, 1024};
        CK(hipEventRecord(e0, 0));
        if (v == 0) {
          CK(launch_open_diffs(d, n, W, opened, f, c));
          CK(launch_odo_post(opened, tri, W, p0, o[0], o[1], f, c));
        } else {
          CK(launch_open_post(d, n, tri, W, p0, o[2 * v], o[2 * v + 1], f, c, v == 2));
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) t[v].push_back(ms);
      }
      std::vector<uint8_t> h[6];
      for (int q = 0; q < 6; ++q) { h[q].resize(W * 16); CK(hipMemcpy(h[q].data(), o[q], W * 16, hipMemcpyDeviceToHost)); }
      const bool same = h[0] == h[2] && h[1] == h[3] && h[0] == h[4] && h[1] == h[5];
      printf("N=%d W=%zu p0=%d outputs %s\n", n, W, p0, same ? "identical" : "DIFFER");
      for (int v = 0; v < 3; ++v) {
        std::sort(t[v].begin(), t[v].end());
        const double bytes = (v == 0 ? (68.0 * n + 64) + 288 : 68.0 * n + 192 + 32) * W;
        const double med = t[v][t[v].size() / 2];
        printf("  %-13s median %9.2f us  min %9.2f us  %7.1f GB/s (own bytes)  %7.1f G words/s\n", names[v],
               med * 1e3, t[v][0] * 1e3, bytes / (med * 1e-3) / 1e9, W / (med * 1e-3) / 1e9);
      }
    }
    for (void* p : allocs) CK(hipFree(p));
    CK(hipFree(tri)); CK(hipFree(opened));
    for (auto& p : o) CK(hipFree(p));
  }
  return 0;
}

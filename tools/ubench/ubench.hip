// Microbenchmark for the K_MASK / K_RV design space (tool, not product).
// Variants run interleaved in one process (cdna_hip_programming.md rule 24),
// median of R rounds, at W = 1 Mi and 16 Mi words, N = 2 parties.
//
//   copy      same loads/stores as K_MASK, XOR instead of field math (ceiling)
//   math      K_MASK arithmetic on register-generated words, no loads
//   mask_nt   product kernel shape: nontemporal loads, grid cap 2048
//   mask_pl   plain loads
//   mask_full grid = W/256 (one word per thread, no grid stride)
//   mask_x2   two words per thread per iteration, loads of both issued first
//   mm2       K_MASK with mont_mul_v2 (alternative CIOS formulation)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../amphora_amd/csrc/field.hpp"

using namespace amph;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 ldv(const uint4* p) {
  if constexpr (NT) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *p;
  }
}

struct Arrs { const uint4* f[5][2]; };

// ---- alternative Montgomery product: 32-bit carry chains, mads only for products
__device__ __forceinline__ W4 mont_mul_v2(const W4& a, const W4& b, const Fp& f) {
  // t = (t0..t5); per i: t += a*b_i (two passes: low halves then high halves)
  uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0, c;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t bi = b.v[i];
    const uint64_t p0 = (uint64_t)a.v[0] * bi, p1 = (uint64_t)a.v[1] * bi;
    const uint64_t p2 = (uint64_t)a.v[2] * bi, p3 = (uint64_t)a.v[3] * bi;
    // add low words
    t0 = addc(t0, (uint32_t)p0, 0, &c);
    t1 = addc(t1, (uint32_t)p1, c, &c);
    t2 = addc(t2, (uint32_t)p2, c, &c);
    t3 = addc(t3, (uint32_t)p3, c, &c);
    t4 = addc(t4, 0, c, &c);
    t5 = c;
    // add high words shifted by one limb
    t1 = addc(t1, (uint32_t)(p0 >> 32), 0, &c);
    t2 = addc(t2, (uint32_t)(p1 >> 32), c, &c);
    t3 = addc(t3, (uint32_t)(p2 >> 32), c, &c);
    t4 = addc(t4, (uint32_t)(p3 >> 32), c, &c);
    t5 += c;
    const uint32_t m = t0 * f.n0;
    const uint64_t q0 = (uint64_t)m * f.p[0], q1 = (uint64_t)m * f.p[1];
    const uint64_t q2 = (uint64_t)m * f.p[2], q3 = (uint64_t)m * f.p[3];
    uint32_t u0 = addc(t0, (uint32_t)q0, 0, &c);
    (void)u0;
    t1 = addc(t1, (uint32_t)q1, c, &c);
    t2 = addc(t2, (uint32_t)q2, c, &c);
    t3 = addc(t3, (uint32_t)q3, c, &c);
    t4 = addc(t4, 0, c, &c);
    t5 += c;
    t1 = addc(t1, (uint32_t)(q0 >> 32), 0, &c);
    t2 = addc(t2, (uint32_t)(q1 >> 32), c, &c);
    t3 = addc(t3, (uint32_t)(q2 >> 32), c, &c);
    t4 = addc(t4, (uint32_t)(q3 >> 32), c, &c);
    t5 += c;
    t0 = t1; t1 = t2; t2 = t3; t3 = t4; t4 = t5; t5 = 0;
  }
  return reduce_once(W4{{t0, t1, t2, t3}}, t4, f);
}

template <int MM>
__device__ __forceinline__ W4 mm(const W4& a, const W4& b, const Fp& f) {
  if constexpr (MM == 2) return mont_mul_v2(a, b, f);
  else return mont_mul(a, b, f);
}

template <bool NT, int MM>
__device__ __forceinline__ void mask_word(const Arrs& A, const uint4* sec, uint4* out, size_t i,
                                          unsigned long long* ff, const Fp& f) {
  uint4 raw[5][2];
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int j = 0; j < 2; ++j) raw[k][j] = ldv<NT>(A.f[k][j] + i);
  const uint4 s = ldv<NT>(sec + i);
  W4 a[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) a[k] = mod_add(canon<true>(w4(raw[k][0]), f), canon<true>(w4(raw[k][1]), f), f);
  const bool ok = (int)eq(mm<MM>(a[0], a[1], f), a[3]) & (int)eq(mm<MM>(a[2], a[1], f), a[4]);
  out[i] = u4(mod_sub(mm<MM>(w4(s), r2_word(f), f), a[0], f));
  if (!ok) atomicMin(ff, (unsigned long long)i);
}

template <bool NT, int MM>
__global__ __launch_bounds__(256) void k_mask_v(Arrs A, const uint4* sec, uint4* out, size_t W,
                                               unsigned long long* ff, Fp f) {
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < W; i += stride)
    mask_word<NT, MM>(A, sec, out, i, ff, f);
}

__global__ __launch_bounds__(256) void k_mask_x2(Arrs A, const uint4* sec, uint4* out, size_t W,
                                                unsigned long long* ff, Fp f) {
  // each thread: words i and i + W/2 (W even), all 22 loads issued first
  const size_t half = W / 2;
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < half; i += stride) {
    uint4 raw[2][5][2], s[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int k = 0; k < 5; ++k)
#pragma unroll
        for (int j = 0; j < 2; ++j) raw[h][k][j] = ldv<true>(A.f[k][j] + i + h * half);
      s[h] = ldv<true>(sec + i + h * half);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      W4 a[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) a[k] = mod_add(canon<true>(w4(raw[h][k][0]), f), canon<true>(w4(raw[h][k][1]), f), f);
      const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
      out[i + h * half] = u4(mod_sub(mont_mul(w4(s[h]), r2_word(f), f), a[0], f));
      if (!ok) atomicMin(ff, (unsigned long long)(i + h * half));
    }
  }
}

// one word per thread, full grid, block size BS
template <int BS, bool NT, int MM>
__global__ __launch_bounds__(BS) void k_mask_f(Arrs A, const uint4* sec, uint4* out, size_t W,
                                              unsigned long long* ff, Fp f) {
  const size_t i = (size_t)blockIdx.x * BS + threadIdx.x;
  if (i < W) mask_word<NT, MM>(A, sec, out, i, ff, f);
}

// two words per thread (i, i + W/2), full grid over W/2
template <int BS>
__global__ __launch_bounds__(BS) void k_mask_f2(Arrs A, const uint4* sec, uint4* out, size_t W,
                                               unsigned long long* ff, Fp f) {
  const size_t half = W / 2;
  const size_t i = (size_t)blockIdx.x * BS + threadIdx.x;
  if (i >= half) return;
  uint4 raw[2][5][2], s[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int j = 0; j < 2; ++j) raw[h][k][j] = ldv<true>(A.f[k][j] + i + h * half);
    s[h] = ldv<true>(sec + i + h * half);
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    W4 a[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) a[k] = mod_add(canon<true>(w4(raw[h][k][0]), f), canon<true>(w4(raw[h][k][1]), f), f);
    const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
    out[i + h * half] = u4(mod_sub(mont_mul(w4(s[h]), r2_word(f), f), a[0], f));
    if (!ok) atomicMin(ff, (unsigned long long)(i + h * half));
  }
}

template <int BS>
__global__ __launch_bounds__(BS) void k_copy_f(Arrs A, const uint4* sec, uint4* out, size_t W) {
  const size_t i = (size_t)blockIdx.x * BS + threadIdx.x;
  if (i >= W) return;
  uint4 x = ldv<true>(sec + i);
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint4 y = ldv<true>(A.f[k][j] + i);
      x.x ^= y.x; x.y ^= y.y; x.z ^= y.z; x.w ^= y.w;
    }
  out[i] = x;
}

__global__ __launch_bounds__(256) void k_copy(Arrs A, const uint4* sec, uint4* out, size_t W) {
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < W; i += stride) {
    uint4 x = ldv<true>(sec + i);
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint4 y = ldv<true>(A.f[k][j] + i);
        x.x ^= y.x; x.y ^= y.y; x.z ^= y.z; x.w ^= y.w;
      }
    out[i] = x;
  }
}

__global__ __launch_bounds__(256) void k_math(uint4* out, size_t W, unsigned long long* ff, Fp f) {
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < W; i += stride) {
    const uint32_t x = (uint32_t)i * 2654435761u;
    W4 a[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      W4 r0{{x ^ (k * 77u), x + k, x * 3u + k, 0x12345678u ^ x}};
      W4 r1{{x + 9u * k, x ^ 0xdeadbeefu, x * 7u, x >> 3}};
      a[k] = mod_add(canon<true>(r0, f), canon<true>(r1, f), f);
    }
    const W4 s{{x, x + 1, x + 2, x + 3}};
    const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
    const W4 o = mod_sub(mont_mul(s, r2_word(f), f), a[0], f);
    if (!ok && o.v[0] == 0x9999u) atomicMin(ff, (unsigned long long)i);
    if (o.v[1] == 0x31337u) out[i] = u4(o);  // keep live, essentially never stored
  }
}

__device__ __forceinline__ W4 hrand(uint64_t x, const Fp& f) {
  x = x * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
  uint64_t a = x ^ (x >> 29), b = (x * 0xBF58476D1CE4E5B9ull) ^ (x >> 31);
  a *= 0x94D049BB133111EBull;
  return canon<true>(W4{{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)}}, f);
}

// honest 2-party ODO words + random secrets
__global__ void k_init(uint4* buf, size_t W, Fp f) {
  const size_t stride = (size_t)gridDim.x * 256;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < W; i += stride) {
    W4 v[5];
    for (int k = 0; k < 3; ++k) v[k] = hrand(i * 16 + k, f);
    v[3] = mont_mul(v[0], v[1], f);
    v[4] = mont_mul(v[2], v[1], f);
    for (int k = 0; k < 5; ++k) {
      const W4 s0 = hrand(i * 16 + 5 + k, f);
      buf[(size_t)(2 * k) * W + i] = u4(s0);
      buf[(size_t)(2 * k + 1) * W + i] = u4(mod_sub(v[k], s0, f));
    }
    buf[10 * W + i] = u4(hrand(i * 16 + 11, f));
  }
}

static Fp test_fp() {
  // p = 0x958907458f2136861bd7554a24340001, R^2 mod p = 0x2f93468814b3ee7f7f160429aa4cd152
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = p[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu;
  f.big = 1;
  return f;
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 30;
  Fp f = test_fp();
  for (size_t W : {(size_t)1 << 20, (size_t)1 << 24}) {
    uint4* buf;
    CK(hipMalloc(&buf, (size_t)12 * W * 16));
    hipLaunchKernelGGL(k_init, dim3(2048), dim3(256), 0, 0, buf, W, f);
    CK(hipDeviceSynchronize());
    Arrs A;
    for (int k = 0; k < 5; ++k)
      for (int j = 0; j < 2; ++j) A.f[k][j] = buf + (size_t)(k * 2 + j) * W;
    const uint4* sec = buf + 10 * W;
    uint4* out = buf + 11 * W;
    unsigned long long* ff;
    CK(hipMalloc(&ff, 16));
    CK(hipMemset(ff, 0x7f, 16));
    const unsigned g2048 = 2048, gfull = (unsigned)(W / 256), g1024 = 1024, g4096 = 4096;
    struct V { const char* name; int id; unsigned grid; };
    (void)g1024; (void)g4096;
    std::vector<V> vs = {{"mask_nt", 2, g2048},  {"full256", 10, gfull}, {"full256pl", 11, gfull},
                         {"full128", 12, gfull * 2}, {"full512", 13, gfull / 2}, {"full1024", 14, gfull / 4},
                         {"full_mm2", 15, gfull}, {"full_x2", 16, gfull / 2},
                         {"copyf256", 17, gfull}, {"copyf512", 18, gfull / 2}, {"copyf1024", 19, gfull / 4}};
    std::vector<std::vector<float>> t(vs.size());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < R + 3; ++r) {
      for (size_t v = 0; v < vs.size(); ++v) {
        CK(hipEventRecord(e0, 0));
        switch (vs[v].id) {
          case 0: hipLaunchKernelGGL(k_copy, dim3(vs[v].grid), dim3(256), 0, 0, A, sec, out, W); break;
          case 1: hipLaunchKernelGGL(k_math, dim3(vs[v].grid), dim3(256), 0, 0, out, W, ff, f); break;
          case 2: hipLaunchKernelGGL((k_mask_v<true, 1>), dim3(vs[v].grid), dim3(256), 0, 0, A, sec, out, W, ff, f); break;
          case 3: hipLaunchKernelGGL((k_mask_v<false, 1>), dim3(vs[v].grid), dim3(256), 0, 0, A, sec, out, W, ff, f); break;
          case 4: hipLaunchKernelGGL(k_mask_x2, dim3(vs[v].grid), dim3(256), 0, 0, A, sec, out, W, ff, f); break;
          case 5: hipLaunchKernelGGL((k_mask_v<true, 2>), dim3(vs[v].grid), dim3(256), 0, 0, A, sec, out, W, ff + 1, f); break;
          case 10: hipLaunchKernelGGL((k_mask_f<256, true, 1>), dim3(vs[v].grid), dim3(256), 0, 0, A, sec, out, W, ff, f); break;
          case 11: hipLaunchKernelGGL((k_mask_f<256, false, 1>), dim3(vs[v].grid), dim3(256), 0, 0, A, sec, out, W, ff, f); break;
          case 12: hipLaunchKernelGGL((k_mask_f<128, true, 1>), dim3(vs[v].grid), dim3(128), 0, 0, A, sec, out, W, ff, f); break;
          case 13: hipLaunchKernelGGL((k_mask_f<512, true, 1>), dim3(vs[v].grid), dim3(512), 0, 0, A, sec, out, W, ff, f); break;
          case 14: hipLaunchKernelGGL((k_mask_f<1024, true, 1>), dim3(vs[v].grid), dim3(1024), 0, 0, A, sec, out, W, ff, f); break;
          case 15: hipLaunchKernelGGL((k_mask_f<256, true, 2>), dim3(vs[v].grid), dim3(256), 0, 0, A, sec, out, W, ff + 1, f); break;
          case 16: hipLaunchKernelGGL((k_mask_f2<256>), dim3(vs[v].grid), dim3(256), 0, 0, A, sec, out, W, ff, f); break;
          case 17: hipLaunchKernelGGL((k_copy_f<256>), dim3(vs[v].grid), dim3(256), 0, 0, A, sec, out, W); break;
          case 18: hipLaunchKernelGGL((k_copy_f<512>), dim3(vs[v].grid), dim3(512), 0, 0, A, sec, out, W); break;
          case 19: hipLaunchKernelGGL((k_copy_f<1024>), dim3(vs[v].grid), dim3(1024), 0, 0, A, sec, out, W); break;
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) t[v].push_back(ms);
      }
    }
    const double bytes = 192.0 * W;  // K_MASK algorithmic bytes, N = 2
    unsigned long long hff[2];
    CK(hipMemcpy(hff, ff, 16, hipMemcpyDeviceToHost));
    printf("W=%zu (K_MASK N=2 algorithmic %.1f MB) first_fail=%llx mm2_first_fail=%llx\n", W, bytes / 1e6, hff[0], hff[1]);
    for (size_t v = 0; v < vs.size(); ++v) {
      std::sort(t[v].begin(), t[v].end());
      const float med = t[v][t[v].size() / 2], mn = t[v][0];
      printf("  %-11s grid %6u  median %8.2f us  min %8.2f us  -> %7.1f GB/s (median)\n", vs[v].name,
             vs[v].grid, med * 1e3, mn * 1e3, bytes / (med * 1e-3) / 1e9);
    }
    CK(hipFree(buf));
    CK(hipFree(ff));
  }
  return 0;
}

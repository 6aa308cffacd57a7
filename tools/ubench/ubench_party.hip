// A/B of party-kernel mappings (tool, not product): k_open and k_odo_post,
// product (word per lane) vs value/pair per lane vs LDS-staged triples.
#include "../../amphora_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstring>
#include <cstdio>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace amph { namespace {

// one opened value per lane: t in [0, 4W)
template <int NP>
__global__ __launch_bounds__(1024) void k_open_v(SignedSet d, size_t nvals, uint4* out, Fp f) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nvals) return;
  uint4 m[NP];
  uint8_t s[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    m[j] = ld(d.mag[j] + t);
    s[j] = reinterpret_cast<const uint8_t*>(d.neg[j])[t];
  }
  W4 acc = {};
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const W4 x = canon<true>(w4(m[j]), f);
    acc = s[j] ? mod_sub(acc, x, f) : mod_add(acc, x, f);
  }
  st(out + t, acc);
}

__device__ __forceinline__ W4 beaver(const W4& a, const W4& b, const W4& c, const uint4& Dr,
                                     const uint4& Er, bool p0, const Fp& f) {
  const W4 r2 = r2_word(f);
  const W4 D = mont_mul(w4(Dr), r2, f), E = mont_mul(w4(Er), r2, f);
  W4 acc = mod_add(canon<true>(c, f), mont_mul(D, b, f), f);
  acc = mod_add(acc, mont_mul(E, a, f), f);
  if (p0) acc = mod_add(acc, mont_mul(D, E, f), f);
  return acc;
}

// one Beaver pair per lane: k in [0, 2W)
__global__ __launch_bounds__(1024) void k_post_p(const uint4* opened, const uint4* triples,
                                                size_t pairs, int p0, uint4* ow, uint4* ou, Fp f) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= pairs) return;
  const uint4* t = triples + 6 * k;
  const uint4 a = ld(t), b = ld(t + 2), c = ld(t + 4);
  const uint4 D = ld(opened + 2 * k), E = ld(opened + 2 * k + 1);
  const W4 z = beaver(w4(a), w4(b), w4(c), D, E, p0, f);
  st((k & 1 ? ou : ow) + (k >> 1), z);
}

// one pair per lane, the block's triples staged through LDS with fully
// coalesced 16-B loads (6 per thread), values read back at a 112-B padded stride
template <int BS>
__global__ __launch_bounds__(BS) void k_post_l(const uint4* opened, const uint4* triples,
                                              size_t pairs, int p0, uint4* ow, uint4* ou, Fp f) {
  __shared__ uint4 lds[BS * 7];
  const size_t k0 = (size_t)blockIdx.x * BS;
  const size_t k = k0 + threadIdx.x;
  const size_t nblk = min((size_t)BS, pairs - k0);
  const uint4* src = triples + 6 * k0;
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    const size_t q = (size_t)r * BS + threadIdx.x;  // uint4 index within the block's triples
    if (q < 6 * nblk) {
      const size_t tri = q / 6, fld = q % 6;
      lds[tri * 7 + fld] = ld(src + q);
    }
  }
  uint4 D = make_uint4(0, 0, 0, 0), E = D;
  if (k < pairs) {
    D = ld(opened + 2 * k);
    E = ld(opened + 2 * k + 1);
  }
  __syncthreads();
  if (k >= pairs) return;
  const uint4 a = lds[threadIdx.x * 7], b = lds[threadIdx.x * 7 + 2], c = lds[threadIdx.x * 7 + 4];
  const W4 z = beaver(w4(a), w4(b), w4(c), D, E, p0, f);
  st((k & 1 ? ou : ow) + (k >> 1), z);
}
}}  // namespace amph::(anon)

static Fp test_fp() {
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = p[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu;
  f.big = 1;
  return f;
}

__global__ void k_fill(uint4* b, size_t n, Fp f) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull + 77, y = (x ^ (x >> 31)) * 0xBF58476D1CE4E5B9ull;
    b[i] = u4(canon<true>(W4{{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 33)}}, f));
  }
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 20;
  Fp f = test_fp();
  for (size_t W : {(size_t)1 << 20, (size_t)1 << 24}) {
    const int n = 2;
    uint4 *mag[2], *opened, *triples, *out, *ow, *ou, *ref_w, *ref_u;
    uint32_t* neg[2];
    for (int j = 0; j < n; ++j) {
      CK(hipMalloc(&mag[j], 4 * W * 16));
      CK(hipMalloc(&neg[j], 4 * W));
      hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, mag[j], 4 * W, f);
      CK(hipMemset(neg[j], 0x01, 4 * W));
    }
    CK(hipMalloc(&opened, 4 * W * 16)); CK(hipMalloc(&triples, 12 * W * 16)); CK(hipMalloc(&out, 4 * W * 16));
    CK(hipMalloc(&ow, W * 16)); CK(hipMalloc(&ou, W * 16)); CK(hipMalloc(&ref_w, W * 16)); CK(hipMalloc(&ref_u, W * 16));
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, opened, 4 * W, f);
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, triples, 12 * W, f);
    CK(hipDeviceSynchronize());
    SignedSet ss{};
    for (int j = 0; j < n; ++j) { ss.mag[j] = mag[j]; ss.neg[j] = neg[j]; }
    const char* names[] = {"open_prod", "open_v", "post_prod", "post_pair", "post_lds256", "post_lds512"};
    std::vector<std::vector<float>> t(6);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    LaunchCfg c{0, 0, 1024};
    launch_odo_post(opened, triples, W, 1, ref_w, ref_u, f, c);
    for (int r = 0; r < R + 3; ++r) for (int v = 0; v < 6; ++v) {
      CK(hipEventRecord(e0, 0));
      switch (v) {
        case 0: launch_open_diffs(ss, n, W, out, f, c); break;
        case 1: hipLaunchKernelGGL(k_open_v<2>, dim3((4 * W + 1023) / 1024), dim3(1024), 0, 0, ss, 4 * W, out, f); break;
        case 2: launch_odo_post(opened, triples, W, 1, ow, ou, f, c); break;
        case 3: hipLaunchKernelGGL(k_post_p, dim3((2 * W + 1023) / 1024), dim3(1024), 0, 0, opened, triples, 2 * W, 1, ow, ou, f); break;
        case 4: hipLaunchKernelGGL(k_post_l<256>, dim3((2 * W + 255) / 256), dim3(256), 0, 0, opened, triples, 2 * W, 1, ow, ou, f); break;
        case 5: hipLaunchKernelGGL(k_post_l<512>, dim3((2 * W + 511) / 512), dim3(512), 0, 0, opened, triples, 2 * W, 1, ow, ou, f); break;
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) t[v].push_back(ms);
      if (r == 0 && v >= 3) {  // correctness vs the product kernel
        std::vector<uint4> a(W), b(W);
        CK(hipMemcpy(a.data(), ow, W * 16, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), ref_w, W * 16, hipMemcpyDeviceToHost));
        bool okw = memcmp(a.data(), b.data(), W * 16) == 0;
        CK(hipMemcpy(a.data(), ou, W * 16, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), ref_u, W * 16, hipMemcpyDeviceToHost));
        printf("  %s matches product: %d\n", names[v], okw && memcmp(a.data(), b.data(), W * 16) == 0);
      }
    }
    printf("W=%zu (open %.0f B/word, post 288 B/word)\n", W, 68.0 * n + 64);
    for (int v = 0; v < 6; ++v) {
      std::sort(t[v].begin(), t[v].end());
      const double bytes = (v < 2 ? 68.0 * n + 64 : 288.0) * W;
      const double med = t[v][t[v].size() / 2];
      printf("  %-12s median %9.2f us  %7.1f GB/s\n", names[v], med * 1e3, bytes / (med * 1e-3) / 1e9);
    }
  }
  return 0;
}

// A/B (tool): the product K_ODO_POST (one reduction for the two Beaver cross
// products, field.hpp dot2_redc) against the previous formula with 4-5
// Montgomery products per pair (k_post_mm).  Product formula:
//   [z] = [c] + MM(REDC(D*[b] + E*[a]), R^2)          (non-player-0)
//   [z] = [c] + MM(REDC(D*([b]+[E]) + E*[a]), R^2)    (player 0, [E] = MM(E, R^2))
// since D*[b] + E*[a] = (Db + Ea) R and REDC(.) = Db + Ea mod p.
#include "../../amphora_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace amph { namespace {

template <bool BIG>
__global__ __launch_bounds__(kPairBlock) void k_post_mm(const uint4* opened, const uint4* triples,
                                                      size_t pairs, int p0, uint4* ow, uint4* ou, Fp f) {
  __shared__ uint4 tri[kPairBlock * 7];
  const size_t k0 = (size_t)blockIdx.x * kPairBlock;
  const size_t k = k0 + threadIdx.x;
  const size_t nblk = min((size_t)kPairBlock, pairs - k0);
  stage_tuples<6, kPairBlock>(tri, triples + 6 * k0, nblk);
  uint4 Dr = make_uint4(0, 0, 0, 0), Er = Dr;
  if (k < pairs) {
    Dr = ld(opened + 2 * k);
    Er = ld(opened + 2 * k + 1);
  }
  __syncthreads();
  if (k >= pairs) return;
  const W4 a = w4(tri[threadIdx.x * 7]), b = w4(tri[threadIdx.x * 7 + 2]);
  const W4 c = w4(tri[threadIdx.x * 7 + 4]);
  const W4 r2 = r2_word(f);
  // the previous product formula: 4-5 Montgomery products per pair
  const W4 D = mont_mul(w4(Dr), r2, f), E = mont_mul(w4(Er), r2, f);
  W4 z = mod_add(canon<BIG>(c, f), mont_mul(D, b, f), f);
  z = mod_add(z, mont_mul(E, a, f), f);
  if (p0) z = mod_add(z, mont_mul(D, E, f), f);
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

// raw words: canonical, or non-canonical [x] + p where that fits (every 7th)
__global__ void k_fill(uint4* b, size_t n, Fp f, int noncanon) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull + 77, y = (x ^ (x >> 31)) * 0xBF58476D1CE4E5B9ull;
    W4 w = canon<true>(W4{{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 33)}}, f);
    if (noncanon && i % 7 == 3) {
      W4 t; uint32_t c;
      t.v[0] = addc(w.v[0], f.p[0], 0, &c); t.v[1] = addc(w.v[1], f.p[1], c, &c);
      t.v[2] = addc(w.v[2], f.p[2], c, &c); t.v[3] = addc(w.v[3], f.p[3], c, &c);
      if (!c) w = t;
    }
    b[i] = u4(w);
  }
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 20;
  Fp f = test_fp();
  for (size_t W : {(size_t)1 << 20, (size_t)1 << 24}) {
    uint4 *opened, *triples, *ow, *ou, *rw, *ru;
    CK(hipMalloc(&opened, 4 * W * 16)); CK(hipMalloc(&triples, 12 * W * 16));
    CK(hipMalloc(&ow, W * 16)); CK(hipMalloc(&ou, W * 16)); CK(hipMalloc(&rw, W * 16)); CK(hipMalloc(&ru, W * 16));
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, opened, 4 * W, f, 0);
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, triples, 12 * W, f, 1);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    LaunchCfg c{0, 0, 1024};
    for (int p0 = 0; p0 < 2; ++p0) {
      CK(launch_odo_post(opened, triples, W, p0, rw, ru, f, c));
      hipLaunchKernelGGL((k_post_mm<true>), dim3((2 * W + kPairBlock - 1) / kPairBlock), dim3(kPairBlock), 0, 0,
                         opened, triples, 2 * W, p0, ow, ou, f);
      CK(hipDeviceSynchronize());
      std::vector<uint4> a(W), b(W);
      CK(hipMemcpy(a.data(), ow, W * 16, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), rw, W * 16, hipMemcpyDeviceToHost));
      bool ok = !memcmp(a.data(), b.data(), W * 16);
      CK(hipMemcpy(a.data(), ou, W * 16, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), ru, W * 16, hipMemcpyDeviceToHost));
      ok = ok && !memcmp(a.data(), b.data(), W * 16);
      printf("W=%zu p0=%d  mont_mul variant matches product kernel: %d\n", W, p0, ok);
      std::vector<float> t[2];
      for (int r = 0; r < R + 3; ++r) for (int v = 0; v < 2; ++v) {
        CK(hipEventRecord(e0, 0));
        if (v == 0) CK(launch_odo_post(opened, triples, W, p0, rw, ru, f, c));
        else hipLaunchKernelGGL((k_post_mm<true>), dim3((2 * W + kPairBlock - 1) / kPairBlock), dim3(kPairBlock), 0, 0,
                                opened, triples, 2 * W, p0, ow, ou, f);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) t[v].push_back(ms);
      }
      const char* nm[2] = {"product", "mont_mul"};
      for (int v = 0; v < 2; ++v) {
        std::sort(t[v].begin(), t[v].end());
        const double med = t[v][t[v].size() / 2];
        printf("  %-8s median %9.2f us  %7.1f GB/s (288 B/word)\n", nm[v], med * 1e3, 288.0 * W / (med * 1e-3) / 1e9);
      }
    }
    CK(hipFree(opened)); CK(hipFree(triples)); CK(hipFree(ow)); CK(hipFree(ou)); CK(hipFree(rw)); CK(hipFree(ru));
  }
  return 0;
}

// A/B (tool): K_ODO_PRE as shipped (each lane stores its pair's two diff
// magnitudes at a 32-B lane stride) against the same kernel with the
// magnitudes written back into the lane's own LDS triple slots and stored as
// one coalesced 16-B run per workgroup (k_pre_lds).  Bit-exact check included.
#include "../../amphora_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace amph { namespace {
__global__ __launch_bounds__(kPairBlock) void k_pre_lds(const uint4* share_data, int stride_w,
                                                       const uint4* masks, const uint4* triples,
                                                       size_t pairs, uint4* oy, uint4* orr,
                                                       uint4* ov, uint4* omag, uint16_t* oneg,
                                                       Fp f) {
  __shared__ uint4 tri[kPairBlock * 7];
  __shared__ uint4 msk[kPairBlock * 3];
  const size_t k0 = (size_t)blockIdx.x * kPairBlock;
  const size_t k = k0 + threadIdx.x;
  const size_t nblk = min((size_t)kPairBlock, pairs - k0);
  stage_tuples<6, kPairBlock>(tri, triples + 6 * k0, nblk);
  stage_tuples<2, kPairBlock>(msk, masks + 2 * k0, nblk);
  const size_t i = k >> 1;
  const bool even = (k & 1) == 0;
  uint4 yr = make_uint4(0, 0, 0, 0);
  if (k < pairs && even) yr = ld(share_data + (size_t)stride_w * i);
  __syncthreads();
  const unsigned lk = threadIdx.x, lpair0 = lk & ~1u;
  if (k < pairs) {
    const uint4 a = tri[lk * 7], b = tri[lk * 7 + 2];
    const uint4 m1 = msk[lpair0 * 3], m2 = msk[(lpair0 + 1) * 3];
    const uint4 x = even ? yr : m2;
    if (even) {
      oy[i] = yr;
      orr[i] = m1;
    } else {
      ov[i] = m2;
    }
    W4 d, e;
    const uint32_t sd = signed_diff(redc(w4(x), f), redc(w4(a), f), d);
    const uint32_t se = signed_diff(redc(w4(m1), f), redc(w4(b), f), e);
    tri[lk * 7] = u4(d);  // the lane's own slots: no other lane reads them
    tri[lk * 7 + 1] = u4(e);
    oneg[k] = (uint16_t)(sd | (se << 8));
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const size_t q = (size_t)r * kPairBlock + threadIdx.x;
    if (q < 2 * nblk) omag[2 * k0 + q] = tri[(q >> 1) * 7 + (q & 1)];
  }
}
}}  // namespace amph::(anon)

__global__ void k_fill(uint4* b, size_t n, Fp f) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull + 77, y = (x ^ (x >> 31)) * 0xBF58476D1CE4E5B9ull;
    b[i] = u4(canon<true>(W4{{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 33)}}, f));
  }
}

int main() {
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = p[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu; f.big = 1;
  for (size_t W : {(size_t)1 << 20, (size_t)1 << 24}) {
    const size_t P = 2 * W;
    uint4 *sh, *mk, *tr, *o[2][4];
    uint16_t* ng[2];
    CK(hipMalloc(&sh, 2 * W * 16)); CK(hipMalloc(&mk, 2 * P * 16)); CK(hipMalloc(&tr, 6 * P * 16));
    for (int v = 0; v < 2; ++v) {
      for (int j = 0; j < 3; ++j) CK(hipMalloc(&o[v][j], W * 16));
      CK(hipMalloc(&o[v][3], 2 * P * 16));
      CK(hipMalloc(&ng[v], P * 2));
    }
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, sh, 2 * W, f);
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, mk, 2 * P, f);
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, tr, 6 * P, f);
    LaunchCfg c{0, 0, 1024};
    std::vector<float> t[2];
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const dim3 g((unsigned)((P + kPairBlock - 1) / kPairBlock));
    for (int r = 0; r < 23; ++r) for (int v = 0; v < 2; ++v) {
      CK(hipEventRecord(e0, 0));
      if (v == 0) launch_odo_pre(sh, 2, mk, tr, W, o[0][0], o[0][1], o[0][2], o[0][3], (uint32_t*)ng[0], f, c);
      else hipLaunchKernelGGL(k_pre_lds, g, dim3(kPairBlock), 0, 0, sh, 2, mk, tr, P, o[1][0], o[1][1], o[1][2], o[1][3], ng[1], f);
      CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) t[v].push_back(ms);
    }
    bool same = true;
    for (int j = 0; j < 4; ++j) {
      const size_t nb = (j < 3 ? W : 2 * P) * 16;
      std::vector<char> a(nb), b(nb);
      CK(hipMemcpy(a.data(), o[0][j], nb, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), o[1][j], nb, hipMemcpyDeviceToHost));
      same &= memcmp(a.data(), b.data(), nb) == 0;
    }
    std::vector<char> a(P * 2), b(P * 2);
    CK(hipMemcpy(a.data(), ng[0], P * 2, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), ng[1], P * 2, hipMemcpyDeviceToHost));
    same &= memcmp(a.data(), b.data(), P * 2) == 0;
    for (auto& v : t) std::sort(v.begin(), v.end());
    printf("W=%zu same=%d prod %.2f us %.1f GB/s | lds-stores %.2f us %.1f GB/s\n", W, (int)same,
           t[0][10] * 1e3, 404.0 * W / (t[0][10] * 1e-3) / 1e9, t[1][10] * 1e3, 404.0 * W / (t[1][10] * 1e-3) / 1e9);
  }
}

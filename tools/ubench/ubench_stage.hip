// A/B (tool): K_ODO_PRE and K_ODO_POST as shipped (the workgroup's whole AoS
// tuples staged in LDS, 7 / 3 uint4 per pair) against compact staging: only
// the tuple fields the kernel uses are loaded and kept in LDS (PRE: a, b of
// each triple and the mask value, 3 + 1 uint4 per pair; POST: a, b, c, 3 uint4
// per pair), so the LDS tile shrinks 40 -> 16 KiB (PRE) and 28 -> 12 KiB
// (POST) and more workgroups fit a CU.  The HBM bytes are the same: the MAC
// fields share 64-B lines with the used ones.  Bit-exact check included.
#include "../../amphora_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace amph { namespace {
// Fields of an S-uint4 tuple selected by NEED (bit f = field f) land in LDS
// at tuple * STR + (rank of f among the selected fields).
template <int S, unsigned NEED, int STR, int BS>
__device__ __forceinline__ void stage_fields(uint4* lds, const uint4* src, size_t ntuples) {
#pragma unroll
  for (int r = 0; r < S; ++r) {
    const size_t q = (size_t)r * BS + threadIdx.x;
    const unsigned fld = (unsigned)(q % S);
    if (q < (size_t)S * ntuples && ((NEED >> fld) & 1u))
      lds[(q / S) * STR + __popc(NEED & ((1u << fld) - 1u))] = ld(src + q);
  }
}

__global__ __launch_bounds__(kPairBlock) void k_pre_c(const uint4* share_data, int stride_w,
                                                     const uint4* masks, const uint4* triples,
                                                     size_t pairs, uint4* oy, uint4* orr,
                                                     uint4* ov, uint4* omag, uint16_t* oneg, Fp f) {
  __shared__ uint4 tri[kPairBlock * 3];
  __shared__ uint4 msk[kPairBlock];
  const size_t k0 = (size_t)blockIdx.x * kPairBlock;
  const size_t k = k0 + threadIdx.x;
  const size_t nblk = min((size_t)kPairBlock, pairs - k0);
  stage_fields<6, 0x5u, 3, kPairBlock>(tri, triples + 6 * k0, nblk);
  stage_fields<2, 0x1u, 1, kPairBlock>(msk, masks + 2 * k0, nblk);
  const size_t i = k >> 1;
  const bool even = (k & 1) == 0;
  uint4 yr = make_uint4(0, 0, 0, 0);
  if (k < pairs && even) yr = ld(share_data + (size_t)stride_w * i);
  __syncthreads();
  if (k >= pairs) return;
  const unsigned lk = threadIdx.x, lpair0 = lk & ~1u;
  const uint4 a = tri[lk * 3], b = tri[lk * 3 + 1];
  const uint4 m1 = msk[lpair0], m2 = msk[lpair0 + 1];
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
  st(omag + 2 * k, d);
  st(omag + 2 * k + 1, e);
  oneg[k] = (uint16_t)(sd | (se << 8));
}

__global__ __launch_bounds__(kPairBlock) void k_post_c(const uint4* opened, const uint4* triples,
                                                      size_t pairs, int p0, uint4* ow, uint4* ou,
                                                      Fp f) {
  __shared__ uint4 tri[kPairBlock * 3];
  const size_t k0 = (size_t)blockIdx.x * kPairBlock;
  const size_t k = k0 + threadIdx.x;
  const size_t nblk = min((size_t)kPairBlock, pairs - k0);
  stage_fields<6, 0x15u, 3, kPairBlock>(tri, triples + 6 * k0, nblk);
  uint4 Dr = make_uint4(0, 0, 0, 0), Er = Dr;
  if (k < pairs) {
    Dr = ld(opened + 2 * k);
    Er = ld(opened + 2 * k + 1);
  }
  __syncthreads();
  if (k >= pairs) return;
  const W4 a = w4(tri[threadIdx.x * 3]), b = w4(tri[threadIdx.x * 3 + 1]);
  const W4 c = w4(tri[threadIdx.x * 3 + 2]);
  const W4 r2 = r2_word(f);
  const W4 D = canon<true>(w4(Dr), f), E = canon<true>(w4(Er), f);
  const W4 bb = p0 ? mod_add(canon<true>(b, f), mont_mul(E, r2, f), f) : b;
  const W4 x = dot2_redc(D, bb, E, a, f);
  st((k & 1 ? ou : ow) + (k >> 1), mod_add(canon<true>(c, f), mont_mul(x, r2, f), f));
}
}}  // namespace amph::(anon)

__global__ void k_fill(uint4* b, size_t n, Fp f, uint64_t salt) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = (i + salt) * 0x9E3779B97F4A7C15ull + 77, y = (x ^ (x >> 31)) * 0xBF58476D1CE4E5B9ull;
    b[i] = u4(canon<true>(W4{{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 33)}}, f));
  }
}

static bool same_dev(const void* a, const void* b, size_t n) {
  std::vector<char> x(n), y(n);
  CK(hipMemcpy(x.data(), a, n, hipMemcpyDeviceToHost));
  CK(hipMemcpy(y.data(), b, n, hipMemcpyDeviceToHost));
  return memcmp(x.data(), y.data(), n) == 0;
}

static float median(std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; }

int main() {
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = p[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu; f.big = 1;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (size_t W : {(size_t)1 << 20, (size_t)1 << 22, (size_t)1 << 24}) {
    const size_t P = 2 * W;
    uint4 *sh, *mk, *tr, *op, *o[2][4], *ow[2], *ou[2];
    uint16_t* ng[2];
    CK(hipMalloc(&sh, 2 * W * 16)); CK(hipMalloc(&mk, 2 * P * 16)); CK(hipMalloc(&tr, 6 * P * 16));
    CK(hipMalloc(&op, 2 * P * 16));
    for (int v = 0; v < 2; ++v) {
      for (int j = 0; j < 3; ++j) CK(hipMalloc(&o[v][j], W * 16));
      CK(hipMalloc(&o[v][3], 2 * P * 16));
      CK(hipMalloc(&ng[v], P * 2));
      CK(hipMalloc(&ow[v], W * 16)); CK(hipMalloc(&ou[v], W * 16));
    }
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, sh, 2 * W, f, 1ull);
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, mk, 2 * P, f, 2ull << 40);
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, tr, 6 * P, f, 3ull << 40);
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, 0, op, 2 * P, f, 4ull << 40);
    LaunchCfg c{0, 0, 1024};
    std::vector<float> t[6];
    const dim3 g((unsigned)((P + kPairBlock - 1) / kPairBlock));
    for (int r = 0; r < 23; ++r) for (int v = 0; v < 6; ++v) {
      CK(hipEventRecord(e0, 0));
      switch (v) {
        case 0: launch_odo_pre(sh, 2, mk, tr, W, o[0][0], o[0][1], o[0][2], o[0][3], (uint32_t*)ng[0], f, c); break;
        case 1: hipLaunchKernelGGL(k_pre_c, g, dim3(kPairBlock), 0, 0, sh, 2, mk, tr, P, o[1][0], o[1][1], o[1][2], o[1][3], ng[1], f); break;
        case 2: launch_odo_post(op, tr, W, 0, ow[0], ou[0], f, c); break;
        case 3: hipLaunchKernelGGL(k_post_c, g, dim3(kPairBlock), 0, 0, op, tr, P, 0, ow[1], ou[1], f); break;
        case 4: launch_odo_post(op, tr, W, 1, ow[0], ou[0], f, c); break;
        case 5: hipLaunchKernelGGL(k_post_c, g, dim3(kPairBlock), 0, 0, op, tr, P, 1, ow[1], ou[1], f); break;
      }
      CK(hipGetLastError());
      CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) t[v].push_back(ms);
    }
    bool same_pre = true;
    for (int j = 0; j < 4; ++j) same_pre &= same_dev(o[0][j], o[1][j], (j < 3 ? W : 2 * P) * 16);
    same_pre &= same_dev(ng[0], ng[1], P * 2);
    const bool same_post = same_dev(ow[0], ow[1], W * 16) && same_dev(ou[0], ou[1], W * 16);  // player 0 (last run)
    const double bpre = 404.0 * W, bpost = 288.0 * W;
    printf("W=%zu pre: prod %.2f us %.1f GB/s | compact %.2f us %.1f GB/s same=%d\n", W,
           median(t[0]) * 1e3, bpre / (median(t[0]) * 1e-3) / 1e9, median(t[1]) * 1e3,
           bpre / (median(t[1]) * 1e-3) / 1e9, (int)same_pre);
    printf("W=%zu post p1: prod %.2f us %.1f GB/s | compact %.2f us %.1f GB/s\n", W,
           median(t[2]) * 1e3, bpost / (median(t[2]) * 1e-3) / 1e9, median(t[3]) * 1e3,
           bpost / (median(t[3]) * 1e-3) / 1e9);
    printf("W=%zu post p0: prod %.2f us %.1f GB/s | compact %.2f us %.1f GB/s same=%d\n", W,
           median(t[4]) * 1e3, bpost / (median(t[4]) * 1e-3) / 1e9, median(t[5]) * 1e3,
           bpost / (median(t[5]) * 1e-3) / 1e9, (int)same_post);
    CK(hipFree(sh)); CK(hipFree(mk)); CK(hipFree(tr)); CK(hipFree(op));
    for (int v = 0; v < 2; ++v) {
      for (int j = 0; j < 4; ++j) CK(hipFree(o[v][j]));
      CK(hipFree(ng[v])); CK(hipFree(ow[v])); CK(hipFree(ou[v]));
    }
  }
  return 0;
}

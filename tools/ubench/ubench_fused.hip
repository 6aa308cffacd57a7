// A/B (tool, not product): the C2 step as two launches (k_mask then k_rv)
// vs ONE launch whose workgroups split between the two bodies (first the
// mask blocks then the rv blocks, or interleaved), vs two streams.
#include "../../amphora_amd/csrc/kernels.hip"
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace amph { namespace {
template <int NP, int MODE>  // MODE 0: mask blocks first; 1: interleaved
__global__ __launch_bounds__(1024) void k_fused(OdoSet mo, const uint4* secrets, uint4* mout,
                                               unsigned long long* mff, OdoSet so, uint4* y,
                                               unsigned long long* sff, size_t words,
                                               unsigned mblocks, Fp f) {
  unsigned b = blockIdx.x;
  bool mask;
  if (MODE == 0) {
    mask = b < mblocks;
    if (!mask) b -= mblocks;
  } else {
    mask = (b & 1) == 0;
    b >>= 1;
  }
  const size_t i = (size_t)b * blockDim.x + threadIdx.x;
  if (i >= words) return;
  W4 a[5];
  if (mask) {
    const uint4 s = ld(secrets + i);
    recombine5<NP, true>(mo, NP, i, f, a);
    const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
    st(mout + i, mod_sub(mont_mul(w4(s), r2_word(f), f), a[0], f));
    report_fail(!ok, i, mff);
  } else {
    recombine5<NP, true>(so, NP, i, f, a);
    const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
    st(y + i, redc(a[0], f));
    report_fail(!ok, i, sff);
  }
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

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 50;
  Fp f = test_fp();
  const int n = 2;
  for (size_t W : {(size_t)1 << 20, (size_t)1 << 22, (size_t)1 << 24}) {
    uint4 *mb, *sb, *sec, *mout, *y, *mout2, *y2;
    unsigned long long* ff;
    CK(hipMalloc(&mb, 5 * n * W * 16)); CK(hipMalloc(&sb, 5 * n * W * 16)); CK(hipMalloc(&sec, W * 16));
    CK(hipMalloc(&mout, W * 16)); CK(hipMalloc(&y, W * 16)); CK(hipMalloc(&mout2, W * 16)); CK(hipMalloc(&y2, W * 16));
    CK(hipMalloc(&ff, 16));
    OutSet om{}, os{};
    OdoSet mo{}, so{};
    for (int k = 0; k < 5; ++k) for (int j = 0; j < n; ++j) {
      om.f[k][j] = mb + (size_t)(k * n + j) * W; mo.f[k][j] = om.f[k][j];
      os.f[k][j] = sb + (size_t)(k * n + j) * W; so.f[k][j] = os.f[k][j];
    }
    LaunchCfg c{0, 0, 1024};
    CK(launch_synth_odos(om, n, W, 1, nullptr, -1, 0, f, c));
    CK(launch_synth_odos(os, n, W, 2, nullptr, -1, 0, f, c));
    CK(launch_synth_words(sec, W, 3, f, c));
    CK(hipMemset(ff, 0x7F, 16));
    CK(hipDeviceSynchronize());
    hipStream_t s2; CK(hipStreamCreate(&s2));
    hipEvent_t e0, e1, ej; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&ej));
    const unsigned mbk = (unsigned)((W + 1023) / 1024);
    const char* names[] = {"two_launches", "fused_seq", "fused_inter", "two_streams"};
    std::vector<float> t[4];
    for (int r = 0; r < R + 3; ++r) for (int v = 0; v < 4; ++v) {
      CK(hipEventRecord(e0, 0));
      switch (v) {
        case 0:
          CK(launch_mask_input(mo, n, W, sec, W, mout, ff, f, c));
          CK(launch_recombine_verify(so, n, W, y, ff + 1, f, c));
          break;
        case 1: hipLaunchKernelGGL((k_fused<2, 0>), dim3(2 * mbk), dim3(1024), 0, 0, mo, sec, mout2, ff, so, y2, ff + 1, W, mbk, f); break;
        case 2: hipLaunchKernelGGL((k_fused<2, 1>), dim3(2 * mbk), dim3(1024), 0, 0, mo, sec, mout2, ff, so, y2, ff + 1, W, mbk, f); break;
        case 3: {
          CK(hipEventRecord(ej, 0)); CK(hipStreamWaitEvent(s2, ej, 0));
          CK(launch_mask_input(mo, n, W, sec, W, mout, ff, f, c));
          LaunchCfg c2 = c; c2.stream = s2;
          CK(launch_recombine_verify(so, n, W, y, ff + 1, f, c2));
          CK(hipEventRecord(ej, s2)); CK(hipStreamWaitEvent(0, ej, 0));
          break;
        }
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) t[v].push_back(ms);
      if (r == 0 && (v == 1 || v == 2)) {
        std::vector<uint4> a(W), b(W);
        CK(hipMemcpy(a.data(), mout, W * 16, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), mout2, W * 16, hipMemcpyDeviceToHost));
        bool ok = !memcmp(a.data(), b.data(), W * 16);
        CK(hipMemcpy(a.data(), y, W * 16, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), y2, W * 16, hipMemcpyDeviceToHost));
        ok = ok && !memcmp(a.data(), b.data(), W * 16);
        unsigned long long h[2]; CK(hipMemcpy(h, ff, 16, hipMemcpyDeviceToHost));
        printf("  %s matches: %d  ff %llx %llx\n", names[v], ok, h[0], h[1]);
      }
    }
    printf("W=%zu  (368 B/word)\n", W);
    for (int v = 0; v < 4; ++v) {
      std::sort(t[v].begin(), t[v].end());
      const double med = t[v][t[v].size() / 2], mn = t[v][0];
      printf("  %-13s median %8.2f us  min %8.2f us  %7.1f GB/s  %6.2f Gwords/s\n", names[v], med * 1e3, mn * 1e3,
             368.0 * W / (med * 1e-3) / 1e9, W / (med * 1e-3) / 1e9);
    }
    CK(hipFree(mb)); CK(hipFree(sb)); CK(hipFree(sec)); CK(hipFree(mout)); CK(hipFree(y)); CK(hipFree(mout2)); CK(hipFree(y2)); CK(hipFree(ff));
  }
  return 0;
}

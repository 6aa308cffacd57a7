// A/B (tool): the fused wire kernels as the product library runs them back to
// back -- 31 launches of k_rv_b64, then 31 of k_mask_b64 (records out), timed
// as one span each, 5 spans per kernel -- built from WIRE_SRC so that two
// builds of wire.hip can be run alternately on one box.  4 Mi words x 3
// parties; prints an FNV hash of each kernel's output so the builds can be
// checked bit-identical.
#ifndef WIRE_SRC
#define WIRE_SRC "../../amphora_amd/csrc/wire.hip"
#endif
#include "../../amphora_amd/csrc/kernels.hip"
#include WIRE_SRC
#include "../../amphora_amd/csrc/codec.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// The kernels' access patterns with no decode or field arithmetic: every lane
// loads its 16-character unit of each of the 5N texts (the same addresses, in
// the same order), XORs them, and lanes < 3/4 of the workgroup write 16 bytes
// (K_RV: the canonical secret) or read a secret and write a 24-byte record
// (K_MASK) -- what the box's HBM delivers for these streams.
template <int NP, int BS, bool MASK>
__global__ __launch_bounds__(BS) void k_wire_probe(TextSet tx, size_t words, const uint4* secrets, uint4* out_y,
                                                   char* out24) {
  const size_t unit = (size_t)blockIdx.x * BS + threadIdx.x;
  uint4 x = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const uint4 v = ld(reinterpret_cast<const uint4*>(tx.t[k][j]) + unit);
      x.x ^= v.x; x.y ^= v.y; x.z ^= v.z; x.w ^= v.w;
    }
  __shared__ uint4 l[BS];
  l[threadIdx.x] = x;
  __syncthreads();
  const size_t word = (size_t)blockIdx.x * Wire<BS>::words + threadIdx.x;
  if (threadIdx.x < Wire<BS>::words && word < words) {
    uint4 v = l[threadIdx.x + BS / 4];
    if (MASK) {
      const uint4 s = ld(secrets + word);
      v.x ^= s.x; v.y ^= s.y;
      uint2* o = reinterpret_cast<uint2*>(out24 + 24 * word);
      o[0] = make_uint2(v.x, v.y); o[1] = make_uint2(v.z, v.w); o[2] = make_uint2(s.z, s.w);
    } else {
      st_out(out_y + word, w4(v));
    }
  }
}

static uint64_t fnv(const std::vector<uint8_t>& v) {
  uint64_t h = 1469598103934665603ull;
  for (uint8_t b : v) h = (h ^ b) * 1099511628211ull;
  return h;
}

int main(int argc, char** argv) {
  constexpr int NP = 3, BS = 256, L = 31;
  const size_t W = (size_t)(argc > 1 ? atoi(argv[1]) : 4) << 20;
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = p[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu;
  f.big = 1;
  const size_t nb = 16 * W, nc = 4 * ((nb + 2) / 3), stride = (nc + 255) & ~(size_t)255;
  const uint32_t pad = (uint32_t)((3 - nb % 3) % 3);
  uint4 *raw, *y;
  char *text, *rec;
  unsigned long long* fl;
  CK(hipMalloc(&raw, (5 * NP + 1) * nb));
  CK(hipMalloc(&text, 5 * NP * stride));
  CK(hipMalloc(&y, nb));
  CK(hipMalloc(&rec, 24 * W));
  CK(hipMalloc(&fl, 4 * 8));
  CK(hipMemset(fl, 0x7f, 4 * 8));
  OutSet os{};
  for (int k = 0; k < 5; ++k) for (int j = 0; j < NP; ++j) os.f[k][j] = raw + (k * NP + j) * W;
  LaunchCfg c{0, 0, 256};
  CK(launch_synth_odos(os, NP, W, 77, nullptr, -1, 0, f, c));
  CK(launch_synth_words(raw + 5 * NP * W, W, 78, f, c));
  TextSet tx{};
  for (int k = 0; k < 5; ++k) for (int j = 0; j < NP; ++j) {
    char* t = text + (k * NP + j) * stride;
    CK(launch_b64_encode((const uint8_t*)os.f[k][j], nb, t, c));
    tx.t[k][j] = t;
  }
  CK(hipDeviceSynchronize());
  const dim3 g((unsigned)((W + Wire<BS>::words - 1) / Wire<BS>::words));
  const uint4* sec = raw + 5 * NP * W;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  uint4* py;
  char* prec;
  CK(hipMalloc(&py, nb));
  CK(hipMalloc(&prec, 24 * W));
  std::vector<float> t[4];
  for (int r = 0; r < 6; ++r) for (int v = 0; v < 4; ++v) {
    CK(hipEventRecord(e0, 0));
    for (int l = 0; l < L; ++l) {
      if (v == 0) hipLaunchKernelGGL((k_rv_b64<NP, true, BS>), g, dim3(BS), 0, 0, tx, NP, W, nc, pad, y, fl, fl + 1, f);
      else if (v == 1) hipLaunchKernelGGL((k_mask_b64<NP, true, BS>), g, dim3(BS), 0, 0, tx, NP, W, nc, pad, sec, W, nullptr, rec, fl + 2, fl + 3, f);
      else if (v == 2) hipLaunchKernelGGL((k_wire_probe<NP, BS, false>), g, dim3(BS), 0, 0, tx, W, sec, py, prec);
      else hipLaunchKernelGGL((k_wire_probe<NP, BS, true>), g, dim3(BS), 0, 0, tx, W, sec, py, prec);
    }
    CK(hipGetLastError());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 1) t[v].push_back(ms * 1e3f / L);
  }
  std::vector<uint8_t> a(nb), b(24 * W);
  CK(hipMemcpy(a.data(), y, nb, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), rec, 24 * W, hipMemcpyDeviceToHost));
  unsigned long long h[4];
  CK(hipMemcpy(h, fl, 32, hipMemcpyDeviceToHost));
  printf("%s: y %016llx rec %016llx flags %llx %llx %llx %llx\n", WIRE_SRC, (unsigned long long)fnv(a),
         (unsigned long long)fnv(b), h[0], h[1], h[2], h[3]);
  const char* names[4] = {"k_rv_b64", "k_mask_b64", "probe rv", "probe mask"};
  const double bytes[4] = {5.0 * NP * nc + nb, 5.0 * NP * nc + nb + 24.0 * W, 5.0 * NP * nc + nb,
                           5.0 * NP * nc + nb + 24.0 * W};
  for (int v = 0; v < 4; ++v) {
    std::sort(t[v].begin(), t[v].end());
    printf("  %-11s %d back-to-back launches: median %8.2f us per launch, min %8.2f (5 spans), %6.2f TB/s\n",
           names[v], L, t[v][t[v].size() / 2], t[v][0], bytes[v] / (t[v][t[v].size() / 2] * 1e-6) / 1e12);
  }
  return 0;
}

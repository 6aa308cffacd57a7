// A/B (tool): the fused wire kernels with WAVE-LOCAL decode buffers (no
// workgroup barrier per field group) against the product k_rv_b64 /
// k_mask_b64, 4 Mi words x 3 parties, interleaved launches, outputs compared.
//
// Product: per field every lane of the 256-lane workgroup decodes one
// 16-character unit into a workgroup LDS buffer; after each group of G fields
// a __syncthreads, then lanes 0..191 (waves 0-2) read their 16-byte words.
// Variant: each wave decodes its 64 units into its OWN 768-byte buffer and its
// lanes 0..47 read the 48 words those units hold -- the same LDS round trip
// with no s_barrier (a wave's LDS operations complete in order), at the price
// of 4 consumer waves at 48 lanes where the product has 3 at 64.
// Result (round 6): per isolated launch -3 % / -6 % (k_mask_b64 / k_rv_b64,
// profiles/r06_wire_wave_ab.txt; the counters: waits 56.8 -> 48.2 % of wave
// cycles, VALU +15.6 %, profiles/r06_wire_pmc_wave_ab.json), but +3 % / 0 %
// in 31 back-to-back launches (ubench_wire_sustained.hip,
// profiles/r06_wire_wave_sustained_ab.txt): rejected, the product keeps the
// workgroup buffers.
#include "../../amphora_amd/csrc/kernels.hip"
#include "../../amphora_amd/csrc/wire.hip"
#include "../../amphora_amd/csrc/codec.hip"
#include <algorithm>
#include <cstdio>
#include <vector>

using namespace amph;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

namespace {

constexpr int kWW = 48;  // words per wave (64 units x 12 bytes / 16)

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Sum the 5 x NP fields of this wave's 48 words (lanes < 48), fast tiles only.
template <int NP, int PD>
__device__ __forceinline__ void wave_fields(const TextSet& tx, size_t nchars, size_t unit, uint32_t* buf, W4 (&acc)[5],
                                            unsigned long long* bad, const Fp& f, const uint8_t* lutp, bool consumer) {
  uint4 raw[5][NP];
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int q = 0; q < PD && q < 5 * NP; ++q) raw[q / NP][q % NP] = ld(reinterpret_cast<const uint4*>(tx.t[q / NP][q % NP]) + unit);
#pragma unroll
  for (int k = 0; k < 5; ++k) {
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const int ahead = k * NP + j + PD;
      if (ahead < 5 * NP)
        raw[ahead / NP][ahead % NP] = ld(reinterpret_cast<const uint4*>(tx.t[ahead / NP][ahead % NP]) + unit);
      uint32_t o[3], badb = 0;
      dec_unit16_lut(raw[k][j], o, badb, lutp);
      if (badb & 0x80u) bad_unit(raw[k][j], j, k, nchars, unit, bad);
      buf[3 * lane] = o[0];
      buf[3 * lane + 1] = o[1];
      buf[3 * lane + 2] = o[2];
      wave_sync_lds();
      if (consumer) {
        const uint4 v = reinterpret_cast<const uint4*>(buf)[lane];
        const W4 x = canon<true>(w4(v), f);
        acc[k] = j == 0 ? x : mod_add(acc[k], x, f);
      }
      wave_sync_lds();  // (reads done before the next field's writes: in order within a wave)
    }
  }
}

template <int NP, int BS, int PD>
__global__ __launch_bounds__(BS) void k_rv_b64_wave(TextSet tx, size_t words, size_t nchars, uint4* out_y,
                                                    unsigned long long* ff, unsigned long long* bad, Fp f) {
  __shared__ uint32_t lds[BS / 64][3 * 64];
  __shared__ uint32_t lutw[kLutBytes / 4];
  uint8_t* lutp = reinterpret_cast<uint8_t*>(lutw);
  b64_lut_fill(lutp);
  __syncthreads();
  if (!(((size_t)blockIdx.x + 1) * Wire<BS>::chars + 4 <= nchars)) return;  // (A/B: fast tiles only)
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t unit = (size_t)blockIdx.x * BS + threadIdx.x;
  const size_t word = (size_t)blockIdx.x * Wire<BS>::words + wv * kWW + lane;
  const bool consumer = lane < kWW && word < words;
  W4 acc[5];
  wave_fields<NP, PD>(tx, nchars, unit, lds[wv], acc, bad, f, lutp, consumer);
  if (lane < kWW) {
    bool ok = true;
    if (consumer) {
      ok = (int)eq(mont_mul_v(acc[0], acc[1], f), acc[3]) & (int)eq(mont_mul_v(acc[2], acc[1], f), acc[4]);
      st_out(out_y + word, redc(acc[0], f));
    }
    report_fail(consumer && !ok, word, ff);
  }
}

template <int NP, int BS, int PD>
__global__ __launch_bounds__(BS) void k_mask_b64_wave(TextSet tx, size_t words, size_t nchars, const uint4* secrets,
                                                      size_t n_secrets, char* out24, unsigned long long* ff,
                                                      unsigned long long* bad, Fp f) {
  __shared__ uint32_t lds[BS / 64][6 * kWW];  // decode buffer (192 dwords), then the wave's 48 records
  __shared__ uint32_t lutw[kLutBytes / 4];
  uint8_t* lutp = reinterpret_cast<uint8_t*>(lutw);
  b64_lut_fill(lutp);
  __syncthreads();
  if (!(((size_t)blockIdx.x + 1) * Wire<BS>::chars + 4 <= nchars)) return;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t unit = (size_t)blockIdx.x * BS + threadIdx.x;
  const size_t w0 = (size_t)blockIdx.x * Wire<BS>::words + wv * kWW;
  const size_t word = w0 + lane;
  const bool consumer = lane < kWW && word < words;
  const bool has_secret = lane < kWW && word < n_secrets;
  W4 acc[5];
  wave_fields<NP, PD>(tx, nchars, unit, lds[wv], acc, bad, f, lutp, consumer);
  uint4 s = make_uint4(0, 0, 0, 0);
  if (has_secret) s = ld(secrets + word);
  uint32_t g[6];
  if (lane < kWW) {
    bool ok = true;
    if (consumer) ok = (int)eq(mont_mul_v(acc[0], acc[1], f), acc[3]) & (int)eq(mont_mul_v(acc[2], acc[1], f), acc[4]);
    report_fail(consumer && !ok, word, ff);
    if (has_secret) {
      const uint4 m = u4(mod_sub(mont_mul_v(w4(s), r2_word(f), f), acc[0], f));
      enc_word24(m, g);
    }
  }
  uint32_t* l = lds[wv];
  if (has_secret)
#pragma unroll
    for (int q = 0; q < 6; ++q) l[6 * lane + q] = g[q];
  wave_sync_lds();
  const size_t nrec = w0 < n_secrets ? min((size_t)kWW, n_secrets - w0) : 0;
  char* dst = out24 + 24 * w0;
  if (nrec == (size_t)kWW) {
    for (int q = lane; q < 6 * kWW / 4; q += 64)
      reinterpret_cast<uint4*>(dst)[q] = make_uint4(l[4 * q], l[4 * q + 1], l[4 * q + 2], l[4 * q + 3]);
  } else {
    for (size_t q = lane; q < 6 * nrec; q += 64) reinterpret_cast<uint32_t*>(dst)[q] = l[q];
  }
}

Fp test_fp() {
  Fp f{};
  const uint32_t p[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = p[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu;
  f.big = 1;
  return f;
}

}  // namespace

int main(int argc, char** argv) {
  constexpr int NP = 3, BS = 256;
  const int R = argc > 1 ? atoi(argv[1]) : 30;
  const size_t W = (size_t)(argc > 2 ? atoi(argv[2]) : 4) << 20;
  Fp f = test_fp();
  const size_t nb = 16 * W, nc = 4 * ((nb + 2) / 3), stride = (nc + 255) & ~(size_t)255;
  const uint32_t pad = (uint32_t)((3 - nb % 3) % 3);
  uint4 *raw, *y[2];
  char *text, *rec[2];
  unsigned long long* fl;
  CK(hipMalloc(&raw, (5 * NP + 1) * nb));
  CK(hipMalloc(&text, 5 * NP * stride));
  for (int v = 0; v < 2; ++v) { CK(hipMalloc(&y[v], nb)); CK(hipMalloc(&rec[v], 24 * W)); }
  CK(hipMalloc(&fl, 16 * 8));
  CK(hipMemset(fl, 0x7f, 16 * 8));
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
  const char* names[6] = {"k_rv_b64 product", "k_rv_b64 wave PD3", "k_mask_b64 product", "k_mask_b64 wave PD3",
                          "k_rv_b64 wave PD5", "k_mask_b64 wave PD5"};
  std::vector<float> t[6];
  for (int r = 0; r < R + 3; ++r) for (int v = 0; v < 6; ++v) {
    CK(hipEventRecord(e0, 0));
    switch (v) {
      case 0: hipLaunchKernelGGL((k_rv_b64<NP, true, BS>), g, dim3(BS), 0, 0, tx, NP, W, nc, pad, y[0], fl, fl + 1, f); break;
      case 1: hipLaunchKernelGGL((k_rv_b64_wave<NP, BS, 3>), g, dim3(BS), 0, 0, tx, W, nc, y[1], fl + 2, fl + 3, f); break;
      case 2: hipLaunchKernelGGL((k_mask_b64<NP, true, BS>), g, dim3(BS), 0, 0, tx, NP, W, nc, pad, sec, W, nullptr, rec[0], fl + 4, fl + 5, f); break;
      case 3: hipLaunchKernelGGL((k_mask_b64_wave<NP, BS, 3>), g, dim3(BS), 0, 0, tx, W, nc, sec, W, rec[1], fl + 6, fl + 7, f); break;
      case 4: hipLaunchKernelGGL((k_rv_b64_wave<NP, BS, 5>), g, dim3(BS), 0, 0, tx, W, nc, y[1], fl + 8, fl + 9, f); break;
      case 5: hipLaunchKernelGGL((k_mask_b64_wave<NP, BS, 5>), g, dim3(BS), 0, 0, tx, W, nc, sec, W, rec[1], fl + 10, fl + 11, f); break;
    }
    CK(hipGetLastError());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (r >= 3) t[v].push_back(ms);
  }
  // compare every word of the fast tiles (the variant skips the last, partial one)
  const size_t full_words = (size_t)(g.x - 1) * Wire<BS>::words;
  std::vector<uint8_t> a(nb), b(nb), ra(24 * W), rb(24 * W);
  CK(hipMemcpy(a.data(), y[0], nb, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), y[1], nb, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ra.data(), rec[0], 24 * W, hipMemcpyDeviceToHost));
  CK(hipMemcpy(rb.data(), rec[1], 24 * W, hipMemcpyDeviceToHost));
  const bool same_y = std::equal(a.begin(), a.begin() + 16 * full_words, b.begin());
  const bool same_r = std::equal(ra.begin(), ra.begin() + 24 * full_words, rb.begin());
  unsigned long long h[12];
  CK(hipMemcpy(h, fl, 12 * 8, hipMemcpyDeviceToHost));
  printf("N=%d W=%zu: canonical secrets %s, records %s over %zu words; flags", NP, W, same_y ? "identical" : "DIFFER",
         same_r ? "identical" : "DIFFER", full_words);
  for (int i = 0; i < 12; ++i) printf(" %llx", h[i]);
  printf("\n");
  for (int v = 0; v < 6; ++v) {
    std::sort(t[v].begin(), t[v].end());
    printf("  %-22s median %8.2f us  min %8.2f us\n", names[v], t[v][t[v].size() / 2] * 1e3, t[v][0] * 1e3);
  }
  return 0;
}

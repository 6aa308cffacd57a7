// Occupancy sweep (tool) of the LDS form of the fused wire kernels
// (amphora_amd/csrc/wire.hip) at 4 Mi words x 3 parties: compiled once per
// (AMPH_WIRE_G fields per barrier, AMPH_WIRE_PD load prefetch depth)
// variant; the inputs (honest ODOs, their base64 text) and the reference
// outputs come from the product library through its C ABI, so every variant
// is checked bit-exact against libamphora_hip's own k_rv_b64 / k_mask_b64.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DAMPH_WIRE_G=3 -DAMPH_WIRE_PD=2 \
//     -Iinclude tools/ubench/ubench_wire_occ.hip -Lamphora_amd -lamphora_hip -o /tmp/u
#define AMPH_WIRE_KERNELS_ONLY 1
#include "../../amphora_amd/csrc/wire.hip"

#include <cstdio>
#include <cstring>
#include <vector>

#include "amphora.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
#define CA(x) do { int st = (x); if (st) { printf("ABI %d: %s @%d\n", st, amph_last_error(), __LINE__); exit(1);} } while (0)

using namespace amph;

static void le16(const char* hex_be, uint8_t out[16]) {
  for (int i = 0; i < 16; ++i) { unsigned v; std::sscanf(hex_be + 2 * (15 - i), "%2x", &v); out[i] = (uint8_t)v; }
}

int main(int argc, char** argv) {
  const size_t W = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (size_t)4 << 20;
  const int R = argc > 2 ? std::atoi(argv[2]) : 20;
  constexpr int NP = 3, BS = kWireBlock;
  uint8_t p[16], r[16], ri[16];
  le16("958907458f2136861bd7554a24340001", p);
  le16("6a76f8ba70dec979e428aab5dbcbffff", r);
  le16("64b363aaebadc239c970b543e5633b46", ri);
  amph_ctx* ctx;
  CA(amph_ctx_create(p, r, ri, 0, &ctx));
  const size_t nb = 16 * W, nc = 4 * ((nb + 2) / 3), stride = (nc + 255) & ~(size_t)255;
  const uint32_t pad = (uint32_t)((3 - nb % 3) % 3);
  uint8_t *raw, *sec, *y_ref, *y_var, *rec_ref, *rec_var;
  char* text;
  unsigned long long* fl;
  CK(hipMalloc(&raw, 5 * NP * nb));
  CK(hipMalloc(&sec, nb));
  CK(hipMalloc(&text, 5 * NP * stride));
  CK(hipMalloc(&y_ref, nb)); CK(hipMalloc(&y_var, nb));
  CK(hipMalloc(&rec_ref, 24 * W)); CK(hipMalloc(&rec_var, 24 * W));
  CK(hipMalloc(&fl, 64));
  std::vector<uint8_t*> fields(5 * NP);
  for (int i = 0; i < 5 * NP; ++i) fields[i] = raw + i * nb;
  CA(amph_synth_odos(ctx, 7, NP, W, fields.data(), nullptr, -1, 0, nullptr));
  CA(amph_synth_words(ctx, 8, W, sec, nullptr));
  TextSet tx{};
  amph_odo_b64 ob[NP];
  for (int k = 0; k < 5; ++k)
    for (int j = 0; j < NP; ++j) {
      char* t = text + (k * NP + j) * stride;
      CA(amph_base64_encode(ctx, fields[k * NP + j], nb, t, AMPH_F_DEVICE, nullptr));
      tx.t[k][j] = t;
    }
  for (int j = 0; j < NP; ++j)
    ob[j] = amph_odo_b64{tx.t[0][j], tx.t[1][j], tx.t[2][j], tx.t[3][j], tx.t[4][j], nc};
  CK(hipDeviceSynchronize());
  // reference outputs: the product library
  CA(amph_recombine_verify_b64(ctx, ob, NP, W, y_ref, (int64_t*)fl, (int64_t*)fl + 1, AMPH_F_DEVICE, nullptr));
  CA(amph_mask_input_b64(ctx, ob, NP, W, sec, W, nullptr, (char*)rec_ref, (int64_t*)fl + 2, (int64_t*)fl + 3,
                         AMPH_F_DEVICE, nullptr));
  Fp f{};
  const uint32_t pw[4] = {0x24340001u, 0x1bd7554au, 0x8f213686u, 0x95890745u};
  const uint32_t r2[4] = {0xaa4cd152u, 0x7f160429u, 0x14b3ee7fu, 0x2f934688u};
  for (int i = 0; i < 4; ++i) { f.p[i] = pw[i]; f.r2[i] = r2[i]; }
  f.n0 = 0x2433ffffu;
  f.big = 1;
  const bool reg = argc > 3 && std::strcmp(argv[3], "reg") == 0;  // the register form instead
  const dim3 g(reg ? (unsigned)(((W + kWireRegWords - 1) / kWireRegWords + kWireRegBlock - 1) / kWireRegBlock)
                   : (unsigned)((W + Wire<BS>::words - 1) / Wire<BS>::words));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float ms_rv = 0, ms_mask = 0;
  for (int it = 0; it < 2; ++it) {  // warm-up pass, then the timed pass
    CK(hipMemset(fl + 4, 0x7f, 32));
    CK(hipEventRecord(e0));
    for (int i = 0; i < R; ++i)
      if (reg)
        hipLaunchKernelGGL((k_rv_b64_reg<NP, true, kWireRegBlock>), g, dim3(kWireRegBlock), 0, 0, tx, NP, W, nc, pad,
                           (uint4*)y_var, fl + 4, fl + 5, f);
      else
        hipLaunchKernelGGL((k_rv_b64<NP, true, BS>), g, dim3(BS), 0, 0, tx, NP, W, nc, pad, (uint4*)y_var, fl + 4, fl + 5, f);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms_rv, e0, e1));
    CK(hipEventRecord(e0));
    for (int i = 0; i < R; ++i)
      if (reg)
        hipLaunchKernelGGL((k_mask_b64_reg<NP, true, kWireRegBlock>), g, dim3(kWireRegBlock), 0, 0, tx, NP, W, nc,
                           pad, (const uint4*)sec, W, nullptr, (char*)rec_var, fl + 6, fl + 7, f);
      else
        hipLaunchKernelGGL((k_mask_b64<NP, true, BS>), g, dim3(BS), 0, 0, tx, NP, W, nc, pad, (const uint4*)sec, W,
                           nullptr, (char*)rec_var, fl + 6, fl + 7, f);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms_mask, e0, e1));
  }
  std::vector<uint8_t> a(24 * W), b(24 * W);
  CK(hipMemcpy(a.data(), y_ref, nb, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), y_var, nb, hipMemcpyDeviceToHost));
  const bool ok_rv = std::memcmp(a.data(), b.data(), nb) == 0;
  CK(hipMemcpy(a.data(), rec_ref, 24 * W, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), rec_var, 24 * W, hipMemcpyDeviceToHost));
  const bool ok_mask = std::memcmp(a.data(), b.data(), 24 * W) == 0;
  unsigned long long h[8];
  CK(hipMemcpy(h, fl, 64, hipMemcpyDeviceToHost));
  const bool verdicts = h[4] == (unsigned long long)AMPH_NO_FAILURE && h[6] == (unsigned long long)AMPH_NO_FAILURE &&
                        h[5] == (unsigned long long)AMPH_NO_FAILURE && h[7] == (unsigned long long)AMPH_NO_FAILURE;
  hipFuncAttributes at;
  CK(hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&k_mask_b64<NP, true, BS>)));
  const double text_bytes = 5.0 * NP * nc;
  printf("{\"form\": \"%s\", \"G\": %d, \"PD\": %d, \"words\": %zu, \"vgpr_mask\": %d, \"lds_bytes\": %zu, "
         "\"k_rv_b64_us\": %.1f, \"k_mask_b64_us\": %.1f, \"mask_TBps\": %.3f, \"bit_exact\": %s}\n",
         reg ? "reg" : "lds", AMPH_WIRE_G, AMPH_WIRE_PD, W, at.numRegs, (size_t)at.sharedSizeBytes, 1e3 * ms_rv / R, 1e3 * ms_mask / R,
         (text_bytes + 16.0 * W + 24.0 * W) / (ms_mask / R * 1e-3) / 1e12,
         ok_rv && ok_mask && verdicts ? "true" : "false");
  return ok_rv && ok_mask && verdicts ? 0 : 1;
}

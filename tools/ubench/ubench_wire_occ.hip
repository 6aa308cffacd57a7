// Occupancy sweep (tool) of the LDS form of the fused wire kernels, with the
// two alternative forms measured in round 4 and rejected (their source lives
// here now): the register form (a lane owns 3 words = 64 characters, no LDS,
// no barrier: 451-535 us vs 305-345) and the persistent software-pipelined
// K_MASK (next tile's loads in flight during the decode: 264 VGPRs, 740 us).
// Original header: Occupancy sweep (tool) of the LDS form of the fused wire kernels
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

// ---- measured-and-rejected forms (round 4), kept here for the record ------------
namespace amph {
namespace {
// The same decode without the offset search: the validity bits of the 16
// characters are ANDed into okacc (stays 0x80808080 while every character
// is in the alphabet), so a caller that decodes many units keeps one
// branch-free accumulator and locates a bad character only if one exists.
__device__ __forceinline__ void dec_unit16_acc(const uint4 v, uint32_t (&o)[3], uint32_t& okacc) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t g[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t val;
    const uint32_t x = dec4_values(w[q], val);
    okacc &= val;
    g[q] = (__builtin_amdgcn_udot4(x, 0x00000140u, 0u, false) << 12) |
           __builtin_amdgcn_udot4(x, 0x01400000u, 0u, false);
  }
  o[0] = __builtin_amdgcn_perm(g[1], g[0], 0x06000102u);
  o[1] = __builtin_amdgcn_perm(g[2], g[1], 0x05060001u);
  o[2] = __builtin_amdgcn_perm(g[3], g[2], 0x04050600u);
}

// ---- register form of the fused wire kernels (no LDS, no barrier) --------------
// 64 characters of a field are exactly 48 bytes = 3 words, so a lane that owns
// THREE consecutive words reads its 64 characters (four 16-byte loads, lanes
// 64 B apart) and has every byte of its words in its own registers after the
// decode: no LDS transpose, no barrier, every wave independent of the others.
// Fields are consumed in the order y, r, w, v, u so that w is checked against
// y r and dropped before v and u are summed (48 live accumulator registers
// instead of 60); one field's four loads are issued before the previous
// field's decode.
constexpr int kWireRegBlock = 256;
constexpr int kWireRegWords = 3;  // words per lane

// one party's field: this lane's 64 characters (units 4 lane .. 4 lane + 3)
// -> its three words.  FAST: full units, validity ANDed into okacc (the
// offset of a bad character is searched for afterwards, wreg_find_bad);
// otherwise per character (padding, the text's end) with the offset reported
// at once.
template <bool FAST>
__device__ __forceinline__ void wreg_unit_words(const uint4 (&raw)[4], const char* t, size_t lane,
                                                size_t nchars, uint32_t pad, int fieldno,
                                                unsigned long long* bad, uint32_t& okacc,
                                                W4 (&x)[kWireRegWords]) {
  uint32_t o[12];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    uint32_t q[3];
    if constexpr (FAST) {
      dec_unit16_acc(raw[u], q, okacc);
      // one unit at a time: interleaving the four units' 16 independent group
      // decodes costs ~100 VGPRs for little VALU latency to hide
      __builtin_amdgcn_sched_barrier(0);
    } else {
      const size_t unit = 4 * lane + u;
      const uint32_t fb = dec_unit_slow(t, unit, nchars, pad, q);
      if (fb != 0xFFFFFFFFu) atomicMin(bad, (unsigned long long)((size_t)fieldno * nchars + 16 * unit + fb));
    }
    o[3 * u] = q[0];
    o[3 * u + 1] = q[1];
    o[3 * u + 2] = q[2];
  }
#pragma unroll
  for (int m = 0; m < kWireRegWords; ++m) x[m] = W4{{o[4 * m], o[4 * m + 1], o[4 * m + 2], o[4 * m + 3]}};
}

// a lane whose characters were not all valid (okacc): the first bad offset
// of every field, re-read one unit at a time (rare: a malformed response)
__device__ __forceinline__ void wreg_find_bad(const TextSet& tx, int n, size_t lane, size_t nchars, uint32_t pad,
                                           unsigned long long* bad) {
  for (int j = 0; j < n; ++j)
    for (int k = 0; k < 5; ++k)
      for (int u = 0; u < 4; ++u) {
        uint32_t q[3];
        const size_t unit = 4 * lane + u;
        const uint32_t fb = dec_unit_slow(tx.t[k][j], unit, nchars, pad, q);
        if (fb != 0xFFFFFFFFu) atomicMin(bad, (unsigned long long)((size_t)(5 * j + k) * nchars + 16 * unit + fb));
      }
}

template <int NP, bool BIG, bool FAST>
__device__ __forceinline__ void wreg_field(const TextSet& tx, int k, int n, size_t lane, size_t nchars,
                                           uint32_t pad, unsigned long long* bad, uint32_t& okacc,
                                           W4 (&acc)[kWireRegWords], const Fp& f) {
  // A runtime loop over the parties (not unrolled): the compiler then cannot
  // interleave several parties' or fields' decodes, which took every lane to
  // 256 VGPRs (one wave per SIMD) when the whole verify was unrolled.  The
  // next party's four loads are issued before this party's decode.
  const int np = NP > 0 ? NP : n;
  uint4 raw[4] = {};
  if constexpr (FAST) {
#pragma unroll
    for (int u = 0; u < 4; ++u) raw[u] = ld(reinterpret_cast<const uint4*>(tx.t[k][0]) + 4 * lane + u);
  }
#pragma unroll 1
  for (int j = 0; j < np; ++j) {
    uint4 next[4] = {};
    if constexpr (FAST) {
      if (j + 1 < np)
#pragma unroll
        for (int u = 0; u < 4; ++u) next[u] = ld(reinterpret_cast<const uint4*>(tx.t[k][j + 1]) + 4 * lane + u);
    }
    W4 x[kWireRegWords];
    wreg_unit_words<FAST>(raw, tx.t[k][j], lane, nchars, pad, 5 * j + k, bad, okacc, x);
#pragma unroll
    for (int m = 0; m < kWireRegWords; ++m) {
      const W4 c = canon<BIG>(x[m], f);
      acc[m] = j == 0 ? c : mod_add(acc[m], c, f);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) raw[u] = next[u];
  }
}

// y, r, w -> check w == y r; v, u -> check u == v r.  ok[m]: word m verified
template <int NP, bool BIG, bool FAST>
__device__ __forceinline__ void wreg_verify(const TextSet& tx, int n, size_t lane, size_t nchars, uint32_t pad,
                                            unsigned long long* bad, W4 (&y)[kWireRegWords],
                                            bool (&ok)[kWireRegWords], const Fp& f) {
  uint32_t okacc = 0x80808080u;
  W4 r[kWireRegWords], t[kWireRegWords];
  wreg_field<NP, BIG, FAST>(tx, 0, n, lane, nchars, pad, bad, okacc, y, f);
  wreg_field<NP, BIG, FAST>(tx, 1, n, lane, nchars, pad, bad, okacc, r, f);
  wreg_field<NP, BIG, FAST>(tx, 3, n, lane, nchars, pad, bad, okacc, t, f);  // w
#pragma unroll
  for (int m = 0; m < kWireRegWords; ++m) {  // one product at a time (each ~30 live temporaries)
    ok[m] = eq(mont_mul_v(y[m], r[m], f), t[m]);
    __builtin_amdgcn_sched_barrier(0);
  }
  W4 v[kWireRegWords];
  wreg_field<NP, BIG, FAST>(tx, 2, n, lane, nchars, pad, bad, okacc, v, f);
  wreg_field<NP, BIG, FAST>(tx, 4, n, lane, nchars, pad, bad, okacc, t, f);  // u
#pragma unroll
  for (int m = 0; m < kWireRegWords; ++m) {
    ok[m] = ok[m] & eq(mont_mul_v(v[m], r[m], f), t[m]);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (FAST && okacc != 0x80808080u) wreg_find_bad(tx, n, lane, nchars, pad, bad);
}

// smallest failing word of the wave (lanes own ascending word ranges)
__device__ __forceinline__ void wreg_report(const bool (&fail)[kWireRegWords], size_t word0,
                                            unsigned long long* ff) {
  size_t first = ~(size_t)0;
#pragma unroll
  for (int m = kWireRegWords - 1; m >= 0; --m)
    if (fail[m]) first = word0 + m;
  report_fail(first != ~(size_t)0, first, ff);
}

template <int NP, bool BIG, int BS>
__global__ __launch_bounds__(BS) void k_rv_b64_reg(TextSet tx, int n, size_t words, size_t nchars,
                                               uint32_t pad, uint4* out_y, unsigned long long* ff,
                                               unsigned long long* bad, Fp f) {
  const size_t lane = (size_t)blockIdx.x * BS + threadIdx.x;
  const size_t word0 = kWireRegWords * lane;
  if (word0 >= words) return;  // whole lanes past the last word: nothing to read or write
  const bool fast = ((size_t)blockIdx.x + 1) * BS * 64 + 4 <= nchars;
  W4 y[kWireRegWords];
  bool ok[kWireRegWords];
  if (fast) wreg_verify<NP, BIG, true>(tx, n, lane, nchars, pad, bad, y, ok, f);
  else wreg_verify<NP, BIG, false>(tx, n, lane, nchars, pad, bad, y, ok, f);
  bool fail[kWireRegWords];
#pragma unroll
  for (int m = 0; m < kWireRegWords; ++m) {
    const bool in = word0 + m < words;
    fail[m] = in && !ok[m];
    if (in) st_out(out_y + word0 + m, redc(y[m], f));
  }
  wreg_report(fail, word0, ff);
}

template <int NP, bool BIG, int BS>
__global__ __launch_bounds__(BS) void k_mask_b64_reg(TextSet tx, int n, size_t words, size_t nchars,
                                                 uint32_t pad, const uint4* secrets, size_t n_secrets,
                                                 uint4* out16, char* out24, unsigned long long* ff,
                                                 unsigned long long* bad, Fp f) {
  const size_t lane = (size_t)blockIdx.x * BS + threadIdx.x;
  const size_t word0 = kWireRegWords * lane;
  if (word0 >= words) return;
  uint4 s[kWireRegWords];
#pragma unroll
  for (int m = 0; m < kWireRegWords; ++m)
    s[m] = word0 + m < n_secrets ? ld(secrets + word0 + m) : make_uint4(0, 0, 0, 0);
  const bool fast = ((size_t)blockIdx.x + 1) * BS * 64 + 4 <= nchars;
  W4 y[kWireRegWords];
  bool ok[kWireRegWords];
  if (fast) wreg_verify<NP, BIG, true>(tx, n, lane, nchars, pad, bad, y, ok, f);
  else wreg_verify<NP, BIG, false>(tx, n, lane, nchars, pad, bad, y, ok, f);
  bool fail[kWireRegWords];
#pragma unroll
  for (int m = 0; m < kWireRegWords; ++m) {
    const size_t w = word0 + m;
    fail[m] = w < words && !ok[m];
    if (w < n_secrets) {
      const W4 mk = mod_sub(mont_mul_v(w4(s[m]), r2_word(f), f), y[m], f);
      if (out16) st_out(out16 + w, mk);
      if (out24) {  // 24-byte record: three 8-byte stores (lanes 72 B apart)
        uint32_t g[6];
        enc_word24(u4(mk), g);
        uint2* d = reinterpret_cast<uint2*>(out24 + 24 * w);
        d[0] = make_uint2(g[0], g[1]);
        d[1] = make_uint2(g[2], g[3]);
        d[2] = make_uint2(g[4], g[5]);
      }
    }
  }
  wreg_report(fail, word0, ff);
}

// K_MASK from the wire as a persistent, software-pipelined loop: each
// workgroup walks tiles blockIdx.x, + gridDim.x, ... and issues the NEXT
// tile's 5N text loads (and secret) before decoding the current one, so its
// own loads are in flight while it decodes -- the one-tile-per-workgroup
// kernel loads, then decodes, with nothing in flight in between.
template <int NP, bool BIG, int BS>
__global__ __launch_bounds__(BS) void k_mask_b64_pipe(TextSet tx, int n, size_t words, size_t nchars,
                                                  uint32_t pad, const uint4* secrets, size_t n_secrets,
                                                  uint4* out16, char* out24, unsigned long long* ff,
                                                  unsigned long long* bad, Fp f) {
  static_assert(NP > 0, "compile-time party count");
  constexpr int WW = Wire<BS>::words;
  __shared__ uint32_t lds[WireGroups<NP>::bufs < 2 ? 2 : WireGroups<NP>::bufs][3 * BS];
  const size_t tiles = (words + WW - 1) / WW;
  // tiles whose characters all lie before the text's last 4 (full units)
  const size_t fast_tiles = nchars >= 4 ? min(tiles, (nchars - 4) / Wire<BS>::chars) : 0;
  uint4 raw[5][NP];
  uint4 s = make_uint4(0, 0, 0, 0);
  auto load_tile = [&](size_t t) {
    if (t < fast_tiles) wire_load<NP, BS>(tx, raw, t);
    const size_t w = t * WW + threadIdx.x;
    s = threadIdx.x < WW && w < n_secrets ? ld(secrets + w) : make_uint4(0, 0, 0, 0);
  };
  size_t t = blockIdx.x;
  if (t < tiles) load_tile(t);
  for (; t < tiles; t += gridDim.x) {
    uint4 cur[5][NP];
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int j = 0; j < NP; ++j) cur[k][j] = raw[k][j];
    const uint4 sc = s;
    if (t + gridDim.x < tiles) load_tile(t + gridDim.x);  // in flight during this tile's decode
    W4 acc[5];
    if (t < fast_tiles) wire_fields<NP, BIG, true, BS>(tx, n, nchars, pad, words, cur, lds, acc, bad, f, t);
    else wire_fields<NP, BIG, false, BS>(tx, n, nchars, pad, words, cur, lds, acc, bad, f, t);
    mask_tile_out<NP, BS>(t, words, sc, n_secrets, acc, out16, out24, ff, lds, f);
    __syncthreads();  // the next tile's decode reuses the LDS buffers
  }
}

}  // namespace
}  // namespace amph

using namespace amph;

// The memory pattern of k_mask_b64 with no decode, no arithmetic (every lane
// loads its 16-character unit of each of the 5N fields, XORs them, and the
// first 3/4 of the lanes write a 24-byte record): what this access pattern
// reaches on this box.
template <int NP, int BS>
__global__ __launch_bounds__(BS) void k_wire_probe(TextSet tx, size_t words, const uint4* secrets, char* out24) {
  constexpr int WW = Wire<BS>::words;
  const size_t unit = (size_t)blockIdx.x * BS + threadIdx.x;
  const size_t word = (size_t)blockIdx.x * WW + threadIdx.x;
  uint4 x = threadIdx.x < WW && word < words ? ld(secrets + word) : make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const uint4 v = ld(reinterpret_cast<const uint4*>(tx.t[k][j]) + unit);
      x.x ^= v.x; x.y ^= v.y; x.z ^= v.z; x.w ^= v.w;
    }
  if (threadIdx.x < WW && word < words) {
    uint2* d = reinterpret_cast<uint2*>(out24 + 24 * word);
    d[0] = make_uint2(x.x, x.y);
    d[1] = make_uint2(x.z, x.w);
    d[2] = make_uint2(x.x ^ x.z, x.y ^ x.w);
  }
}

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
  const bool pipe = argc > 3 && std::strcmp(argv[3], "pipe") == 0;  // persistent pipelined K_MASK
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int wpc = argc > 4 ? std::atoi(argv[4]) : 3;
  if (argc > 3 && std::strcmp(argv[3], "probe") == 0) {
    const dim3 gp((unsigned)((W + Wire<BS>::words - 1) / Wire<BS>::words));
    hipEvent_t a0, a1;
    CK(hipEventCreate(&a0)); CK(hipEventCreate(&a1));
    float ms = 0;
    for (int it = 0; it < 2; ++it) {
      CK(hipEventRecord(a0));
      for (int i = 0; i < R; ++i)
        hipLaunchKernelGGL((k_wire_probe<NP, BS>), gp, dim3(BS), 0, 0, tx, W, (const uint4*)sec, (char*)rec_var);
      CK(hipEventRecord(a1)); CK(hipEventSynchronize(a1)); CK(hipEventElapsedTime(&ms, a0, a1));
    }
    const double b = 5.0 * NP * nc + 16.0 * W + 24.0 * W;
    printf("{\"form\": \"probe\", \"words\": %zu, \"us\": %.1f, \"TBps\": %.3f}\n", W, 1e3 * ms / R,
           b / (ms / R * 1e-3) / 1e12);
    return 0;
  }
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
      if (pipe)
        hipLaunchKernelGGL((k_mask_b64_pipe<NP, true, BS>), dim3(cus * wpc), dim3(BS), 0, 0, tx, NP, W, nc, pad,
                           (const uint4*)sec, W, nullptr, (char*)rec_var, fl + 6, fl + 7, f);
      else if (reg)
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
  CK(hipFuncGetAttributes(&at, pipe ? reinterpret_cast<const void*>(&k_mask_b64_pipe<NP, true, BS>)
                                    : reinterpret_cast<const void*>(&k_mask_b64<NP, true, BS>)));
  const double text_bytes = 5.0 * NP * nc;
  printf("{\"form\": \"%s\", \"wg_per_cu\": %d, \"G\": %d, \"PD\": %d, \"words\": %zu, \"vgpr_mask\": %d, \"lds_bytes\": %zu, "
         "\"k_rv_b64_us\": %.1f, \"k_mask_b64_us\": %.1f, \"mask_TBps\": %.3f, \"bit_exact\": %s}\n",
         pipe ? "pipe" : reg ? "reg" : "lds", pipe ? wpc : 0, AMPH_WIRE_G, AMPH_WIRE_PD, W, at.numRegs, (size_t)at.sharedSizeBytes, 1e3 * ms_rv / R, 1e3 * ms_mask / R,
         (text_bytes + 16.0 * W + 24.0 * W) / (ms_mask / R * 1e-3) / 1e12,
         ok_rv && ok_mask && verdicts ? "true" : "false");
  return ok_rv && ok_mask && verdicts ? 0 : 1;
}

// The fused wire-format kernels: K_RV / K_MASK straight from the base64 text
// of the ODO fields (getSecret / createSecret with Jackson's base64 decode of
// every byte[] field, DefaultAmphoraClient.java:150-170,206-217): the text is
// decoded in the workgroup and consumed through LDS.  Bound: the decode's
// integer VALU work ("Wire kernels, round 4": a register form
// without LDS, a persistent software-pipelined form and an occupancy sweep
// were measured and rejected -- tools/ubench/ubench_wire_occ.hip).
#include <cstdlib>
#include <string>

#include "b64.hpp"
#include "devio.hpp"

namespace amph {
namespace {

// ---- fused wire-format kernels ----------------------------------------------
// The client receives each party's ODO as base64 text (VerifiableSecretShare /
// OutputDeliveryObject JSON, Jackson's Base64Variants.MIME_NO_LINEFEEDS) and
// sends each masked word as a 24-character record (MaskedInputData).  Decoding
// the 5N fields to HBM and then running K_RV / K_MASK moves 4/3 x 80N + 2 x 80N
// bytes per word; these kernels decode the text in the workgroup and consume
// it from LDS, so the decoded words never reach HBM (K_RV from text: 4/3 x
// 80N + 16 B/word).
//
// A workgroup of kWireBlock lanes owns 16 x kWireBlock characters of every
// field = 12 x kWireBlock bytes = kWireWords words.  Per field every lane
// decodes one 16-character unit (4 groups) and writes its 12 bytes to LDS;
// after a barrier the first kWireWords lanes (whole waves: the last quarter of
// the waves only decode) read their 16-byte word and add it into the field's
// sum.  Two LDS buffers alternate, so one barrier per field suffices.  The
// text's final group may carry '=' padding: the workgroup that holds it
// (or any character past the text) takes the per-character path.
constexpr int kWireBlock = 256;  // workgroup size: 256 > 512 > 1024 by 15-50 % (tools/ubench/ubench_wire.hip)
template <int BS>
struct Wire {
  static constexpr int words = BS * 3 / 4;          // words per workgroup
  static constexpr size_t chars = (size_t)16 * BS;  // characters per field per workgroup
};

// One 16-character unit of a field's text, checked character by character:
// positions >= nchars decode as 'A' (zero bits, beyond the last word);
// the final `pad` positions must be '=' (decoded as 'A'), '=' anywhere else
// is invalid like any non-alphabet character.  Returns the unit's first
// invalid offset (or 0xFFFFFFFF) and its 12 bytes in o.
__device__ __forceinline__ uint32_t dec_unit_slow(const char* t, size_t unit, size_t nchars,
                                                  uint32_t pad, uint32_t (&o)[3]) {
  uint32_t w[4] = {0, 0, 0, 0}, forced = 0xFFFFFFFFu;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const size_t pos = 16 * unit + q;
    uint32_t ch = pos < nchars ? (uint8_t)t[pos] : (uint32_t)'A';
    if (pos < nchars && pos + pad >= nchars) {
      if (ch != '=' && forced == 0xFFFFFFFFu) forced = q;
      ch = 'A';
    }
    w[q >> 2] |= ch << (8 * (q & 3));
  }
  const uint32_t fb = dec_unit16(make_uint4(w[0], w[1], w[2], w[3]), o);
  return min(fb, forced);
}

// Sum field k over the parties from the text, consuming it through LDS.  raw:
// this lane's units, loaded up front on the fast path (FAST).
// Fast-path loads: kWirePrefetch > 0 issues field f + kWirePrefetch's load
// while field f is decoded (fewer live VGPRs); 0 issues all 5N up front.
#ifndef AMPH_WIRE_PD
#define AMPH_WIRE_PD 3  // with the LDS-table decode: 73-77 VGPRs at 3 parties (0: 99-101)
#endif
constexpr int kWirePrefetch = AMPH_WIRE_PD;

// Fields decoded per barrier (AMPH_WIRE_G): G units of text go to LDS before
// each barrier (2G buffers alternate, or all 5N at once, one barrier in all,
// when G >= 5N).
#ifndef AMPH_WIRE_G
// 3: 6 buffers + the 256-byte decode table = 18.7 KB per block, so LDS allows
// 6 waves per SIMD as the VGPRs do (G = 5: 30.3 KB, 5 waves); k_mask_b64
// -5 % at 4 Mi x 3 (profiles/r05_wire_lut_ab.txt).  r02: G = 5 was 2-5 % over 1.
#define AMPH_WIRE_G 3
#endif
template <int NP>
struct WireGroups {
  static constexpr int F = 5 * (NP > 0 ? NP : 1);  // fields (runtime party counts: G = 1)
  static constexpr int G = NP > 0 ? (AMPH_WIRE_G < F ? AMPH_WIRE_G : F) : 1;
  static constexpr int bufs = G >= F ? F : 2 * G;
};

// A fast-path unit with a bad character (rare): locate the first one and
// report (party j, field k) in ODO order, then the offset -- the same
// atomicMin the per-character path makes.
__device__ __forceinline__ void bad_unit(const uint4 v, int j, int k, size_t nchars, size_t unit,
                                         unsigned long long* bad) {
  uint32_t o[3];
  const uint32_t fb = dec_unit16(v, o);
  atomicMin(bad, (unsigned long long)((size_t)(5 * j + k) * nchars + 16 * unit + fb));
}

template <int NP, bool BIG, bool FAST, int BS>
__device__ __forceinline__ void wire_fields(const TextSet& tx, int n, size_t nchars, uint32_t pad,
                                            size_t words, uint4 (&raw)[5][NP > 0 ? NP : 1],
                                            uint32_t (*lds)[3 * BS], W4 (&acc)[5],
                                            unsigned long long* bad, const Fp& f, size_t tile,
                                            const uint8_t* lutp) {
  constexpr int G = WireGroups<NP>::G, NB = WireGroups<NP>::bufs;
  const size_t unit = tile * BS + threadIdx.x;
  const size_t word = tile * Wire<BS>::words + threadIdx.x;
  const bool consumer = threadIdx.x < Wire<BS>::words && word < words;
  const int np = NP > 0 ? NP : n;
  int slot = 0;  // LDS buffer of the next field
#pragma unroll
  for (int k = 0; k < 5; ++k) {
#pragma unroll
    for (int j = 0; j < (NP > 0 ? NP : kMaxParties); ++j) {
      if (NP == 0 && j >= np) break;
      uint32_t o[3];
      if constexpr (FAST && NP > 0) {
        if constexpr (kWirePrefetch > 0) {
          const int ahead = k * NP + j + kWirePrefetch;
          if (ahead < 5 * NP)
            raw[ahead / NP][ahead % NP] = ld(reinterpret_cast<const uint4*>(tx.t[ahead / NP][ahead % NP]) + unit);
        }
        uint32_t badb = 0;  // the per-unit branch also bounds the LDS reads' live ranges: one
        dec_unit16_lut(raw[k][j], o, badb, lutp);  // check after the last field took 117-256 VGPRs
        if (badb & 0x80u) bad_unit(raw[k][j], j, k, nchars, unit, bad);
      } else if constexpr (FAST) {
        const uint4 v = ld(reinterpret_cast<const uint4*>(tx.t[k][j]) + unit);
        uint32_t badb = 0;
        dec_unit16_lut(v, o, badb, lutp);
        if (badb & 0x80u) bad_unit(v, j, k, nchars, unit, bad);
      } else {
        const uint32_t fb = dec_unit_slow(tx.t[k][j], unit, nchars, pad, o);
        if (fb != 0xFFFFFFFFu)  // (party j, field k) in ODO order, then the offset
          atomicMin(bad, (unsigned long long)((size_t)(5 * j + k) * nchars + 16 * unit + fb));
      }
      uint32_t* l = lds[slot];
      l[3 * threadIdx.x] = o[0];
      l[3 * threadIdx.x + 1] = o[1];
      l[3 * threadIdx.x + 2] = o[2];
      const int fi = k * (NP > 0 ? NP : 1) + j;  // flat field index (G = 1 for runtime counts)
      const bool group_end = G == 1 || (fi + 1) % G == 0 || fi + 1 == WireGroups<NP>::F;
      if (group_end) {
        __syncthreads();
        if (consumer) {
          // the group's fields, oldest first: fields fi - m, m = cnt-1 .. 0
          const int cnt = G == 1 ? 1 : (fi % G) + 1;
#pragma unroll
          for (int m = (G == 1 ? 0 : G - 1); m >= 0; --m) {
            if (m >= cnt) continue;
            const int ff = fi - m, kk = G == 1 ? k : ff / (NP > 0 ? NP : 1), jj = G == 1 ? j : ff % (NP > 0 ? NP : 1);
            const int sl = (slot - m + NB) % NB;
            const uint4 v = reinterpret_cast<const uint4*>(lds[sl])[threadIdx.x];
            const W4 x = canon<BIG>(w4(v), f);
            acc[kk] = jj == 0 ? x : mod_add(acc[kk], x, f);
          }
        }
      }
      slot = (slot + 1) % NB;
    }
  }
}

template <int NP, int BS>
__device__ __forceinline__ void wire_load(const TextSet& tx, uint4 (&raw)[5][NP > 0 ? NP : 1], size_t tile) {
  if constexpr (NP > 0) {
    const size_t unit = tile * BS + threadIdx.x;
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int j = 0; j < NP; ++j)
        if (kWirePrefetch == 0 || k * NP + j < kWirePrefetch)
          raw[k][j] = ld(reinterpret_cast<const uint4*>(tx.t[k][j]) + unit);
  }
}

// K_MASK from the wire, after a tile's fields are summed: verify, mask the
// secret, and write the masked word and / or its 24-character record (each
// lane its own, as three nontemporal 8-byte stores).
template <int NP, int BS>
__device__ __forceinline__ void mask_tile_out(size_t tile, size_t words, const uint4 s, size_t n_secrets,
                                              W4 (&acc)[5], uint4* out16, char* out24,
                                              unsigned long long* ff, uint32_t (*lds)[3 * BS], const Fp& f) {
  constexpr int WW = Wire<BS>::words;
  const size_t word = tile * WW + threadIdx.x;
  const bool has_secret = threadIdx.x < WW && word < n_secrets;
  uint32_t g[6];
  if (threadIdx.x < WW) {
    const bool in = word < words;
    bool ok = true;
    if (in) ok = (int)eq(mont_mul_v(acc[0], acc[1], f), acc[3]) & (int)eq(mont_mul_v(acc[2], acc[1], f), acc[4]);
    report_fail(in && !ok, word, ff);
    if (has_secret) {
      const uint4 m = u4(mod_sub(mont_mul_v(w4(s), r2_word(f), f), acc[0], f));
      if (out16) st_out(out16 + word, w4(m));
      enc_word24(m, g);
    }
  }
  if (!out24 || !has_secret) return;
  // records: each lane streams its own 24 bytes as three nontemporal 8-byte
  // stores; a wave's three store instructions cover its 1536 contiguous
  // bytes, which the L2 merges into whole lines.  Round 5 staged the
  // workgroup's records in LDS and stored 16-byte runs behind two barriers:
  // sustained k_mask_b64 277.8 -> 265.6 us at 4 Mi x 3 (plain 8-byte stores:
  // 274.2), 0.95-0.96 of its access-pattern probe
  // (profiles/r06_wire_record_stores_ab.txt)
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  u32x2* o = reinterpret_cast<u32x2*>(out24 + 24 * word);
  __builtin_nontemporal_store(u32x2{g[0], g[1]}, o);
  __builtin_nontemporal_store(u32x2{g[2], g[3]}, o + 1);
  __builtin_nontemporal_store(u32x2{g[4], g[5]}, o + 2);
}

// Waves per SIMD the register allocation must allow (0: the compiler's choice;
// tools/ubench A/B knob, spills below ~96 VGPRs).
#ifndef AMPH_WIRE_WPE
#define AMPH_WIRE_WPE 0
#endif
#if AMPH_WIRE_WPE > 0
#define AMPH_WIRE_OCC __attribute__((amdgpu_waves_per_eu(AMPH_WIRE_WPE)))
#else
#define AMPH_WIRE_OCC
#endif

// K_RV from the wire: the N parties' base64 ODO fields -> canonical secrets,
// MAC verify (getSecret, DefaultAmphoraClient.java:206-217 incl. the Jackson
// base64 decode of every field).  bad: min (5 party + field) * nchars + offset
// of an invalid character.
template <int NP, bool BIG, int BS>
__global__ __launch_bounds__(BS) AMPH_WIRE_OCC void k_rv_b64(TextSet tx, int n, size_t words, size_t nchars,
                                           uint32_t pad, uint4* out_y, unsigned long long* ff,
                                           unsigned long long* bad, Fp f) {
  __shared__ uint32_t lds[WireGroups<NP>::bufs < 2 ? 2 : WireGroups<NP>::bufs][3 * BS];
  __shared__ uint32_t lutw[kLutBytes / 4];
  uint8_t* lutp = reinterpret_cast<uint8_t*>(lutw);
  b64_lut_fill(lutp);
  __syncthreads();
  W4 acc[5];
  uint4 raw[5][NP > 0 ? NP : 1];
  const bool fast = ((size_t)blockIdx.x + 1) * Wire<BS>::chars + 4 <= nchars;
  if (fast) {
    wire_load<NP, BS>(tx, raw, blockIdx.x);
    wire_fields<NP, BIG, true, BS>(tx, n, nchars, pad, words, raw, lds, acc, bad, f, blockIdx.x, lutp);
  } else {
    wire_fields<NP, BIG, false, BS>(tx, n, nchars, pad, words, raw, lds, acc, bad, f, blockIdx.x, lutp);
  }
  const size_t word = (size_t)blockIdx.x * Wire<BS>::words + threadIdx.x;
  if (threadIdx.x < Wire<BS>::words) {  // whole waves
    const bool in = word < words;
    bool ok = true;
    if (in) {
      ok = (int)eq(mont_mul_v(acc[0], acc[1], f), acc[3]) & (int)eq(mont_mul_v(acc[2], acc[1], f), acc[4]);
      st_out(out_y + word, redc(acc[0], f));
    }
    report_fail(in && !ok, word, ff);
  }
}

// K_MASK from the wire: the N parties' base64 Input Mask ODO fields + the
// secrets -> verify the masks, masked[i] = toGfp((s_i - m_i) mod p) for
// i < n_secrets, written as raw words (out16) and/or as the 24-character
// base64 records of MaskedInputData (out24, staged through LDS and stored as
// coalesced 16-byte runs).  createSecret, DefaultAmphoraClient.java:150-170.
template <int NP, bool BIG, int BS>
__global__ __launch_bounds__(BS) AMPH_WIRE_OCC void k_mask_b64(TextSet tx, int n, size_t words, size_t nchars,
                                             uint32_t pad, const uint4* secrets, size_t n_secrets,
                                             uint4* out16, char* out24, unsigned long long* ff,
                                             unsigned long long* bad, Fp f) {
  constexpr int WW = Wire<BS>::words;
  __shared__ uint32_t lds[WireGroups<NP>::bufs < 2 ? 2 : WireGroups<NP>::bufs][3 * BS];
  __shared__ uint32_t lutw[kLutBytes / 4];
  uint8_t* lutp = reinterpret_cast<uint8_t*>(lutw);
  b64_lut_fill(lutp);
  __syncthreads();
  W4 acc[5];
  uint4 raw[5][NP > 0 ? NP : 1];
  const size_t word = (size_t)blockIdx.x * WW + threadIdx.x;
  const bool has_secret = threadIdx.x < WW && word < n_secrets;
  const bool fast = ((size_t)blockIdx.x + 1) * Wire<BS>::chars + 4 <= nchars;
  if (fast) {
    wire_load<NP, BS>(tx, raw, blockIdx.x);
    wire_fields<NP, BIG, true, BS>(tx, n, nchars, pad, words, raw, lds, acc, bad, f, blockIdx.x, lutp);
  } else {
    wire_fields<NP, BIG, false, BS>(tx, n, nchars, pad, words, raw, lds, acc, bad, f, blockIdx.x, lutp);
  }
  // the secret after the decode: loaded up front it held 4 VGPRs through it
  // (98 VGPRs: 4 waves per SIMD instead of 5); the other waves hide its latency
  uint4 s = make_uint4(0, 0, 0, 0);
  if (has_secret) s = ld(secrets + word);
  mask_tile_out<NP, BS>(blockIdx.x, words, s, n_secrets, acc, out16, out24, ff, lds, f);
}


}  // namespace

#ifndef AMPH_WIRE_KERNELS_ONLY  // (tools/ubench: the kernels without the launchers' instantiations)
hipError_t launch_rv_b64(const TextSet& tx, int n, size_t words, size_t nchars, uint32_t pad,
                         uint4* out_y, unsigned long long* ff, unsigned long long* bad, const Fp& f,
                         const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  constexpr int BS = kWireBlock;
  const dim3 g((unsigned)((words + Wire<BS>::words - 1) / Wire<BS>::words));
#define L(NP, BIG) AMPH_LAUNCH((k_rv_b64<NP, BIG, BS>), g, dim3(BS), c, tx, n, words, nchars, pad, out_y, ff, bad, f)
  if (f.big) { AMPH_DISPATCH_NP(n, true, L) } else { AMPH_DISPATCH_NP(n, false, L) }
#undef L
  return hipGetLastError();
}

hipError_t launch_mask_b64(const TextSet& tx, int n, size_t words, size_t nchars, uint32_t pad,
                           const uint4* secrets, size_t n_secrets, uint4* out16, char* out24,
                           unsigned long long* ff, unsigned long long* bad, const Fp& f,
                           const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  constexpr int BS = kWireBlock;
  const dim3 g((unsigned)((words + Wire<BS>::words - 1) / Wire<BS>::words));
#define L(NP, BIG) AMPH_LAUNCH((k_mask_b64<NP, BIG, BS>), g, dim3(BS), c, tx, n, words, nchars, pad, secrets, n_secrets, out16, out24, ff, bad, f)
  if (f.big) { AMPH_DISPATCH_NP(n, true, L) } else { AMPH_DISPATCH_NP(n, false, L) }
#undef L
  return hipGetLastError();
}

#endif  // AMPH_WIRE_KERNELS_ONLY

}  // namespace amph

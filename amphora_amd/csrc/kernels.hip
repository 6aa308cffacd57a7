// Share-arithmetic kernels for gfx950 (MI355X).  One 128-bit word per lane,
// grid-stride over the word index; every load/store is a 16-byte
// global_load/store_dwordx4, so a wave touches 1 KiB contiguous per field
// array (fully coalesced).  All work is HBM-bound integer arithmetic (no
// MFMA): see DESIGN.md for the roofline of each kernel.
//
// Reference rows each kernel replaces:
//   k_rv         A2 x5 + A3 + A4  client SecretShareUtil.java:53-141,
//                                 DefaultAmphoraClient.java:476-505
//   k_mask       K_RV + A5        DefaultAmphoraClient.java:150-160, SecretShareUtil.java:65-68
//   k_recombine  A2               SecretShareUtil.java:70-90
//   k_verify     A3               SecretShareUtil.java:102-141
//   k_conv       A6               service calculation/SecretShareUtil.java:58-107
//   k_odo_pre    A7 + A8 + A9 pre OutputDeliveryService.java:75-139,186-200
//   k_open       A9 open          OutputDeliveryService.java:231-272
//   k_odo_post   A9 post + A8     OutputDeliveryService.java:147-152,274-286
#include "kernels.hpp"

#include <hip/hip_ext.h>

#include "b64.hpp"
#include "decimal.hpp"
#include "devio.hpp"

namespace amph {

namespace {

// Sum over parties of one field at word i, canonical Montgomery form.
template <int NP, bool BIG>
__device__ __forceinline__ W4 sum_field(const uint4* const* src, int n, size_t i, const Fp& f) {
  if constexpr (NP > 0) {
    uint4 raw[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) raw[j] = ld(src[j] + i);
    W4 acc = canon<BIG>(w4(raw[0]), f);
#pragma unroll
    for (int j = 1; j < NP; ++j) acc = mod_add(acc, canon<BIG>(w4(raw[j]), f), f);
    return acc;
  } else {
    W4 acc = canon<BIG>(w4(ld(src[0] + i)), f);
    for (int j = 1; j < n; ++j) acc = mod_add(acc, canon<BIG>(w4(ld(src[j] + i)), f), f);
    return acc;
  }
}

// Loads of all 5 fields are issued before any arithmetic (the compiler keeps
// them in flight: 5N outstanding dwordx4 per lane).
template <int NP, bool BIG>
__device__ __forceinline__ void recombine5(const OdoSet& odo, int n, size_t i, const Fp& f,
                                           W4 (&acc)[5]) {
  if constexpr (NP > 0) {
    uint4 raw[5][NP];
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int j = 0; j < NP; ++j) raw[k][j] = ld(odo.f[k][j] + i);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      acc[k] = canon<BIG>(w4(raw[k][0]), f);
#pragma unroll
      for (int j = 1; j < NP; ++j) acc[k] = mod_add(acc[k], canon<BIG>(w4(raw[k][j]), f), f);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 5; ++k) acc[k] = sum_field<0, BIG>(odo.f[k], n, i, f);
  }
}

// WRITE_Y = false: verify only (the tail of an Input Mask ODO set that has
// more words than secrets, DefaultAmphoraClient.java:153-160).
template <int NP, bool BIG, bool WRITE_Y = true>
__global__ __launch_bounds__(kMaxBlock) void k_rv(OdoSet odo, int n, size_t words, uint4* out_y,
                                              unsigned long long* ff, Fp f, size_t ibase = 0) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
    W4 a[5];
    recombine5<NP, BIG>(odo, n, i, f, a);
    const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
    if constexpr (WRITE_Y) st_out(out_y + i, redc(a[0], f));
    report_fail(!ok, ibase + i, ff);
  }
}

#ifndef MASK_SECRET_MUL
#define MASK_SECRET_MUL mont_mul_v
#endif

// One secret per word (the launcher covers words beyond the secrets with a
// verify-only k_rv): the secret load is unconditional and issued first, which
// measured 10 % faster at 3 parties than a per-lane guarded load.
template <int NP, bool BIG>
__global__ __launch_bounds__(kMaxBlock) void k_mask(OdoSet odo, int n, size_t words,
                                                const uint4* secrets, uint4* out,
                                                unsigned long long* ff, Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const W4 r2 = r2_word(f);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
    const uint4 s = ld(secrets + i);
    W4 a[5];
    recombine5<NP, BIG>(odo, n, i, f, a);
    const bool ok = (int)eq(mont_mul(a[0], a[1], f), a[3]) & (int)eq(mont_mul(a[2], a[1], f), a[4]);
    // the secret's product in the product-scanning form: 64 instead of 65
    // VGPRs at 3 parties (8 waves per SIMD: two 1024-lane workgroups per CU)
    st_out(out + i, mod_sub(MASK_SECRET_MUL(w4(s), r2, f), a[0], f));
    report_fail(!ok, i, ff);
  }
}

template <int NP, bool BIG>
__global__ __launch_bounds__(kMaxBlock) void k_recombine(ShareSet sh, int n, size_t words,
                                                     uint4* out, Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride)
    st_out(out + i, redc(sum_field<NP, BIG>(sh.s, n, i, f), f));
}

template <bool BIG>
__global__ __launch_bounds__(kMaxBlock) void k_verify(const uint4* y, const uint4* r, const uint4* u,
                                                  const uint4* v, const uint4* w, size_t words,
                                                  unsigned long long* ff, Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
    const W4 Y = canon<BIG>(w4(ld(y + i)), f), R = canon<BIG>(w4(ld(r + i)), f);
    const W4 V = canon<BIG>(w4(ld(v + i)), f);
    const W4 Wd = w4(ld(w + i)), Ud = w4(ld(u + i));
    // y r R^-1 == w R^-1  <=>  y r == w (mod p); host guarantees w, u < p
    const bool ok = (int)eq(mont_mul(Y, R, f), redc(Wd, f)) & (int)eq(mont_mul(V, R, f), redc(Ud, f));
    report_fail(!ok, i, ff);
  }
}

// signed x - a of canonical integers: magnitude, returns 1 if negative
__device__ __forceinline__ uint32_t signed_diff(const W4& x, const W4& a, W4& mag) {
  W4 d, e;
  const uint32_t neg = sub128(x, a, d);
  sub128(a, x, e);
  mag = sel(neg != 0, e, d);
  return neg;
}

// AoS tuple staging: a workgroup's contiguous run of tuples (S uint4 each) is
// read with fully coalesced 16-B loads (consecutive lanes, consecutive uint4)
// into LDS at a padded stride of S+1 uint4 (breaks the power-of-two bank
// pattern of the per-lane reads), then each lane reads its own tuple's fields.
template <int S, int BS>
__device__ __forceinline__ void stage_tuples(uint4* lds, const uint4* src, size_t ntuples) {
  if (ntuples == (size_t)BS) {
    // a whole workgroup's run: all S loads in flight before the first LDS
    // write (the guarded loop below made the compiler wait for each load
    // before issuing the next -- S dependent HBM latencies per workgroup)
    uint4 v[S];
#pragma unroll
    for (int r = 0; r < S; ++r) v[r] = ld(src + (size_t)r * BS + threadIdx.x);
#pragma unroll
    for (int r = 0; r < S; ++r) {
      const int q = r * BS + threadIdx.x;
      lds[(q / S) * (S + 1) + q % S] = v[r];
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < S; ++r) {
    const size_t q = (size_t)r * BS + threadIdx.x;
    if (q < (size_t)S * ntuples) lds[(q / S) * (S + 1) + q % S] = ld(src + q);
  }
}

constexpr int kPairBlock = 128;  // pairs per workgroup of the LDS-staged kernels (256: 1-2 % slower at 16 Mi, 512: 2-12 %)

// K_CONV, one word per lane; the workgroup's input-mask tuples (value||mac,
// 32 B) come in and its output shares (value||mac) go out as coalesced 16-B
// runs through LDS (stage_tuples; each lane overwrites only its own tuple's
// slots with its results).  5.54 -> 6.06 TB/s at 16 Mi words over direct
// 32-B-stride loads and stores (tools/ubench/ubench_conv.hip).
template <bool BIG>
__global__ __launch_bounds__(kPairBlock) void k_conv(const uint4* masked, const uint4* tuples,
                                                    size_t words, W4 alpha, int use_zero,
                                                    uint4* out, Fp f) {
  __shared__ uint4 buf[3 * kPairBlock];
  const size_t i0 = (size_t)blockIdx.x * kPairBlock, i = i0 + threadIdx.x;
  const size_t nblk = min((size_t)kPairBlock, words - i0);
  stage_tuples<2, kPairBlock>(buf, tuples + 2 * i0, nblk);
  uint4 mr = make_uint4(0, 0, 0, 0);
  if (i < words) mr = ld(masked + i);
  __syncthreads();
  if (i < words) {
    const W4 m = canon<BIG>(w4(mr), f);
    const W4 val = canon<BIG>(w4(buf[3 * threadIdx.x]), f);
    const W4 mac = canon<BIG>(w4(buf[3 * threadIdx.x + 1]), f);
    buf[3 * threadIdx.x] = u4(use_zero ? val : mod_add(val, m, f));
    buf[3 * threadIdx.x + 1] = u4(mod_add(mac, mont_mul(m, alpha, f), f));
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const size_t q = (size_t)r * kPairBlock + threadIdx.x;
    if (q < 2 * nblk) st_party(out + 2 * i0 + q, buf[(q >> 1) * 3 + (q & 1)]);
  }
}

// K_ODO_PRE, one Beaver pair per lane (k = 2i: (y_i, r_i), k = 2i+1: (v_i, r_i);
// r_i = value of mask tuple 2i, v_i = value of mask tuple 2i+1), the
// workgroup's triples (96 B) and mask tuples (32 B) staged through LDS.
// Even lanes also write the raw y_i and r_i copies, odd lanes v_i (each
// output optional).  (Writing the base64 text of y, r and v here instead of the
// raw copies -- 64 instead of 48 + 112 B per word with the separate base64
// pass -- measured 389-396 us against 290 + 3 x 30 at 4 Mi words: the
// encoding's VALU work in every workgroup cost more than the traffic it saved.)
// lens (the party session): the exchange text length of this workgroup's
// 128 FactorPairs -- the exchange encoder's first pass (k_xenc_bsum), which
// would read the diffs back, done where they are made.
template <bool LENS>
__global__ __launch_bounds__(kPairBlock) void k_odo_pre(const uint4* share_data, int stride_w,
                                                       const uint4* masks, const uint4* triples,
                                                       size_t pairs, uint4* oy, uint4* orr,
                                                       uint4* ov, uint4* omag, uint16_t* oneg,
                                                       Fp f, uint64_t* lens) {
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
  uint32_t len = 0;
  if (k < pairs) {
    const unsigned lk = threadIdx.x, lpair0 = lk & ~1u;
    const uint4 a = tri[lk * 7], b = tri[lk * 7 + 2];
    const uint4 m1 = msk[lpair0 * 3], m2 = msk[(lpair0 + 1) * 3];
    const uint4 x = even ? yr : m2;
    if (even) {
      if (oy) st_party(oy + i, yr);
      if (orr) st_party(orr + i, m1);
    } else if (ov) {
      st_party(ov + i, m2);
    }
    W4 d, e;
    const uint32_t sd = signed_diff(redc(w4(x), f), redc(w4(a), f), d);
    const uint32_t se = signed_diff(redc(w4(m1), f), redc(w4(b), f), e);
    st_party(omag + 2 * k, u4(d));
    st_party(omag + 2 * k + 1, u4(e));
    oneg[k] = (uint16_t)(sd | (se << 8));
    if constexpr (LENS) len = xentry_len(u4(d), sd, u4(e), se, k + 1 == pairs);
  }
  if constexpr (!LENS) return;
  // (the wave sums reuse the triples' LDS once every lane is past it: one
  // more word of LDS would cost a workgroup per CU -- 20 KiB x 8 fills it)
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) len += __shfl_xor(len, o, 64);
  uint32_t* wlen = reinterpret_cast<uint32_t*>(tri);
  __syncthreads();
  if (__lane_id() == 0) wlen[threadIdx.x >> 6] = len;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < kPairBlock / 64; ++w) t += wlen[w];
    lens[blockIdx.x] = t;
  }
}

// recombineDiffs: one opened value per lane (value t of 4 per source word),
// so every load and store is a consecutive 16-B (or 1-B sign) access
// (3x the bandwidth of a word-per-lane mapping, tools/ubench/ubench_party.hip).
template <int NP, bool BIG>
__global__ __launch_bounds__(kMaxBlock) void k_open(SignedSet d, int n, size_t nvals, uint4* out,
                                                Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < nvals; t += stride) {
    W4 acc = {};
    if constexpr (NP > 0) {
      uint4 m[NP];
      uint8_t s[NP];
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        m[j] = ld(d.mag[j] + t);
        s[j] = reinterpret_cast<const uint8_t*>(d.neg[j])[t];
      }
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const W4 x = canon<BIG>(w4(m[j]), f);
        acc = s[j] ? mod_sub(acc, x, f) : mod_add(acc, x, f);
      }
    } else {
      for (int j = 0; j < n; ++j) {
        const W4 x = canon<BIG>(w4(ld(d.mag[j] + t)), f);
        acc = reinterpret_cast<const uint8_t*>(d.neg[j])[t] ? mod_sub(acc, x, f) : mod_add(acc, x, f);
      }
    }
    st_out(out + t, acc);
  }
}

// K_ODO_POST, one Beaver pair per lane: [z_k] = [c] + [D b + E a] (+ [D E]
// for player 0).  With D, E canonical integers and [a], [b] wire words,
// D [b] + E [a] = (D b + E a) R, so ONE reduction of the full-width sum
// gives D b + E a mod p (dot2_redc) and one mont_mul by R^2 puts it back in
// the Montgomery domain; player 0 folds D E in as D ([b] + [E]).  2-3
// Montgomery-sized products per pair instead of 4-5
// (tools/ubench/ubench_post.hip: 4-9 % faster at 16 Mi words, bit-exact).
// The workgroup's triples are staged through LDS (2x the direct strided
// loads at 16 Mi words, tools/ubench/ubench_party.hip).  Even k -> w, odd k -> u.
template <bool BIG>
__global__ __launch_bounds__(kPairBlock) void k_odo_post(const uint4* opened,
                                                        const uint4* triples, size_t pairs,
                                                        int p0, uint4* ow, uint4* ou, Fp f) {
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
  const W4 D = canon<BIG>(w4(Dr), f), E = canon<BIG>(w4(Er), f);
  const W4 bb = p0 ? mod_add(canon<BIG>(b, f), mont_mul(E, r2, f), f) : b;
  const W4 x = dot2_redc(D, bb, E, a, f);  // D b + E a (+ D E), canonical
  st_out((k & 1 ? ou : ow) + (k >> 1), mod_add(canon<BIG>(c, f), mont_mul(x, r2, f), f));
}

// recombineDiffs fused into K_ODO_POST (OutputDeliveryService.java:223-228,
// 231-286): one Beaver pair per lane opens D = sum_j +-d_j and E = sum_j +-e_j
// from every party's signed diffs and goes straight on to the product share,
// so the opened values never round-trip through HBM (the two-launch path
// writes and re-reads 64 B per word: 488 -> 360 B/word at N = 2, 556 -> 428
// at N = 3).  Each party's diff pair (2 x 16 B) is one 32-B-strided lane
// access; STAGE_MAG instead brings the workgroup's run of them in through LDS
// like the triples (tools/ubench/ubench_open_post.hip measures both).
// Pair k's two diffs from a party in the exchange decode's span form
// (XSpans).  The workgroup's 256 values (kXMapValues) lie in spans s0, s0 + 1,
// s0 + 2 (a full span holds >= 167 values: a value's text is at most 49
// bytes); span_win reads the total and the workgroup's map window (s0 and
// the three span boundaries inside it, completed by the decode) as two
// independent uniform loads, issued before the triples are staged so their
// latency hides under the staging; span_slot then places each value by three
// compares (a loop over further bases only if a span were shorter).  In text
// order a pair may list "b" first (bit 1 of its byte): d, e are swapped back.
// When the general pass ran (fail bits in base[nb], or a count other than
// 2 pairs) the values sit in pair order, slot = index.
static_assert(kXMapValues == 2 * kPairBlock, "one map entry per k_open_post workgroup");
struct SpanWin {
  uint4 e;  // the workgroup's map window
  bool pair_order;
};

__device__ __forceinline__ void span_win(const uint64_t* base, const uint4* map, size_t nb, size_t pairs,
                                         SpanWin& w) {
  w.pair_order = base[nb] != 2 * pairs;
  w.e = map[blockIdx.x];  // (not used in pair order)
}

// slot of value v (in this workgroup's window)
__device__ __forceinline__ size_t span_slot(const SpanWin& w, const uint64_t* base, size_t nb, size_t v) {
  if (w.pair_order) return v;
  const size_t t = v - (size_t)blockIdx.x * kXMapValues, s0 = w.e.x;
  const uint32_t o1 = w.e.z & 0xFFFFu, o2 = w.e.z >> 16;
  if (t < o1) return s0 * kXSpanSlots + w.e.y + t;
  if (t < o2) return (s0 + 1) * kXSpanSlots + (t - o1);
  if (t < w.e.w) return (s0 + 2) * kXSpanSlots + (t - o2);
  size_t s = s0 + 3;
  while (s < nb && base[s + 1] <= v) ++s;
  return s * kXSpanSlots + (v - base[s]);
}

__device__ __forceinline__ void span_pair(const uint4* mag, const uint8_t* negb, const uint64_t* base, size_t nb,
                                          const SpanWin& w, size_t k, uint4& md, uint4& me, uint32_t& sg) {
  const size_t a = span_slot(w, base, nb, 2 * k), b = span_slot(w, base, nb, 2 * k + 1);
  const uint4 x = ld(mag + a), y = ld(mag + b);
  const uint32_t nx = negb[a], ny = negb[b];
  const bool swap = (nx & 2u) != 0;
  md = swap ? y : x;
  me = swap ? x : y;
  sg = swap ? ((ny & 1u) | ((nx & 1u) << 8)) : ((nx & 1u) | ((ny & 1u) << 8));
}

// SPAN: parties 1 .. NP-1 are partners in the span form, party 0 this party's
// pair-ordered diffs (the party session) -- known at compile time, so the
// partners' window loads are issued together instead of one kernel-argument
// test and wait per party.
template <int NP, bool BIG, bool STAGE_MAG, bool SPAN>
__global__ __launch_bounds__(kPairBlock) void k_open_post(SignedSet d, int n, const uint4* triples,
                                                         size_t pairs, int p0, uint4* ow, uint4* ou,
                                                         Fp f) {
  constexpr int kMagSlots = STAGE_MAG ? (NP > 0 ? NP : 1) * kPairBlock * 3 : 0;
  __shared__ uint4 lds[kPairBlock * 7 + kMagSlots];
  uint4* tri = lds;
  const size_t k0 = (size_t)blockIdx.x * kPairBlock;
  const size_t k = k0 + threadIdx.x;
  const size_t nblk = min((size_t)kPairBlock, pairs - k0);
  SpanWin sw[NP > 0 ? NP : 1];
  if constexpr (NP > 0) {
#pragma unroll
    for (int j = 0; j < NP; ++j)
      if (SPAN && j > 0) span_win(d.sbase[j], d.smap[j], d.snb[j], pairs, sw[j]);
  }
  stage_tuples<6, kPairBlock>(tri, triples + 6 * k0, nblk);
  W4 D = {}, E = {};
  if constexpr (NP > 0) {
    uint4 md[NP], me[NP];
    uint32_t sg[NP];
    if constexpr (STAGE_MAG) {
#pragma unroll
      for (int j = 0; j < NP; ++j)
        stage_tuples<2, kPairBlock>(lds + kPairBlock * 7 + j * kPairBlock * 3, d.mag[j] + 2 * k0, nblk);
    }
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      if (SPAN && j > 0) {  // a partner's decoded text in span form
        md[j] = me[j] = make_uint4(0, 0, 0, 0);
        sg[j] = 0;
        if (k < pairs)
          span_pair(d.mag[j], reinterpret_cast<const uint8_t*>(d.neg[j]), d.sbase[j], d.snb[j], sw[j], k, md[j],
                    me[j], sg[j]);
        continue;
      }
      if constexpr (!STAGE_MAG) {
        md[j] = k < pairs ? ld(d.mag[j] + 2 * k) : make_uint4(0, 0, 0, 0);
        me[j] = k < pairs ? ld(d.mag[j] + 2 * k + 1) : make_uint4(0, 0, 0, 0);
      }
      sg[j] = k < pairs ? reinterpret_cast<const uint16_t*>(d.neg[j])[k] : 0;
    }
    __syncthreads();
    if (k >= pairs) return;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      if constexpr (STAGE_MAG) {
        md[j] = lds[kPairBlock * 7 + j * kPairBlock * 3 + 3 * threadIdx.x];
        me[j] = lds[kPairBlock * 7 + j * kPairBlock * 3 + 3 * threadIdx.x + 1];
      }
      const W4 x = canon<BIG>(w4(md[j]), f), y = canon<BIG>(w4(me[j]), f);
      D = (sg[j] & 0xFF) ? mod_sub(D, x, f) : mod_add(D, x, f);
      E = (sg[j] >> 8) ? mod_sub(E, y, f) : mod_add(E, y, f);
    }
  } else {
    __syncthreads();
    if (k >= pairs) return;
    for (int j = 0; j < n; ++j) {
      uint4 mx, my;
      uint32_t s;
      if (d.sbase[j]) {
        SpanWin w;
        span_win(d.sbase[j], d.smap[j], d.snb[j], pairs, w);
        span_pair(d.mag[j], reinterpret_cast<const uint8_t*>(d.neg[j]), d.sbase[j], d.snb[j], w, k, mx, my, s);
      } else {
        s = reinterpret_cast<const uint16_t*>(d.neg[j])[k];
        mx = ld(d.mag[j] + 2 * k);
        my = ld(d.mag[j] + 2 * k + 1);
      }
      const W4 x = canon<BIG>(w4(mx), f), y = canon<BIG>(w4(my), f);
      D = (s & 0xFF) ? mod_sub(D, x, f) : mod_add(D, x, f);
      E = (s >> 8) ? mod_sub(E, y, f) : mod_add(E, y, f);
    }
  }
  // K_ODO_POST on the opened (canonical) D, E
  const W4 a = w4(tri[threadIdx.x * 7]), b = w4(tri[threadIdx.x * 7 + 2]);
  const W4 c = w4(tri[threadIdx.x * 7 + 4]);
  const W4 r2 = r2_word(f);
  const W4 bb = p0 ? mod_add(canon<BIG>(b, f), mont_mul(E, r2, f), f) : b;
  const W4 x = dot2_redc(D, bb, E, a, f);
  st_out((k & 1 ? ou : ow) + (k >> 1), mod_add(canon<BIG>(c, f), mont_mul(x, r2, f), f));
}

// MpSpdzIntegrationUtils.toGfp / fromGfp over arrays, and maskInput with
// canonical masks (SecretShareUtil.java:65-68 word by word).
template <bool BIG>
__global__ __launch_bounds__(kMaxBlock) void k_to_gfp(const uint4* in, size_t words, uint4* out, Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const W4 r2 = r2_word(f);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride)
    st(out + i, mont_mul(w4(ld(in + i)), r2, f));
}

__global__ __launch_bounds__(kMaxBlock) void k_from_gfp(const uint4* in, size_t words, uint4* out, Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride)
    st(out + i, redc(w4(ld(in + i)), f));
}

template <bool BIG>
__global__ __launch_bounds__(kMaxBlock) void k_mask_words(const uint4* secrets, const uint4* masks,
                                                      size_t words, uint4* out, Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const W4 r2 = r2_word(f);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
    const W4 s = mont_mul(w4(ld(secrets + i)), r2, f), m = mont_mul(w4(ld(masks + i)), r2, f);
    st(out + i, mod_sub(s, m, f));
  }
}

// ---- synthetic inputs ------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

template <bool BIG>
__device__ __forceinline__ W4 rand_fe(uint64_t seed, uint64_t ctr, const Fp& f) {
  const uint64_t a = splitmix64(seed ^ splitmix64(2 * ctr)), b = splitmix64(seed ^ splitmix64(2 * ctr + 1));
  return canon<BIG>(W4{{(uint32_t)b, (uint32_t)(b >> 32), (uint32_t)a, (uint32_t)(a >> 32)}}, f);
}

template <bool BIG>
__global__ __launch_bounds__(kMaxBlock) void k_synth(OutSet out, int n, size_t words, uint64_t seed,
                                                 uint4* plain_y, long long fault, int permille,
                                                 Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const W4 one = redc(r2_word(f), f);  // [1] = R mod p
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
    const uint64_t base = (uint64_t)i * 64;
    W4 val[5];
    val[0] = rand_fe<BIG>(seed, base + 0, f);
    val[1] = rand_fe<BIG>(seed, base + 1, f);
    val[2] = rand_fe<BIG>(seed, base + 2, f);
    val[3] = mont_mul(val[0], val[1], f);
    val[4] = mont_mul(val[2], val[1], f);
    if (plain_y) st(plain_y + i, redc(val[0], f));
    for (int k = 0; k < 5; ++k) {
      W4 rest = val[k];
      for (int j = 0; j < n; ++j) {
        W4 sh;
        if (j < n - 1) {
          sh = rand_fe<BIG>(seed, base + 8 + 8 * k + j, f);
          rest = mod_sub(rest, sh, f);
        } else {
          sh = rest;
        }
        if (k == 3 && (long long)i == fault && j == (n > 1 ? 1 : 0)) sh = mod_add(sh, one, f);
        if (BIG && permille > 0) {
          const uint64_t h = splitmix64(seed ^ splitmix64(base + 48 + 8 * k + j));
          if ((int)(h % 1000) < permille) {
            W4 t;
            uint32_t c;
            t.v[0] = addc(sh.v[0], f.p[0], 0, &c);
            t.v[1] = addc(sh.v[1], f.p[1], c, &c);
            t.v[2] = addc(sh.v[2], f.p[2], c, &c);
            t.v[3] = addc(sh.v[3], f.p[3], c, &c);
            if (!c) sh = t;  // raw word [x] + p, still < 2^128
          }
        }
        st(out.f[k][j] + i, sh);
      }
    }
  }
}

// Measurement only: K_MASK's exact memory pattern (the same 5N + 1 nontemporal
// 16-B loads per lane, one 16-B store, same grid) with the field arithmetic
// replaced by an XOR, so bench.py can time, in the same run and on the same
// box, what this access pattern achieves at this size with nothing else to do.
template <int NP>
__global__ __launch_bounds__(kMaxBlock) void k_stream_probe(OdoSet odo, int n, size_t words,
                                                        const uint4* secrets, uint4* out) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
    uint4 x = ld(secrets + i);
    const int np = NP > 0 ? NP : n;
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int j = 0; j < (NP > 0 ? NP : kMaxParties); ++j) {
        if (NP == 0 && j >= np) break;
        const uint4 v = ld(odo.f[k][j] + i);
        x.x ^= v.x;
        x.y ^= v.y;
        x.z ^= v.z;
        x.w ^= v.w;
      }
    st_out(out + i, w4(x));
  }
}

template <bool BIG>
__global__ __launch_bounds__(kMaxBlock) void k_synth_words(uint4* out, size_t count, uint64_t seed,
                                                       Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride)
    st(out + i, rand_fe<BIG>(seed, i, f));
}

// One word per thread over a full grid: measured faster than a capped
// grid-stride loop (tools/ubench: 1.1-1.15x at 1-16 Mi words).  grid_cap > 0
// caps the grid (the kernels grid-stride past it).
unsigned grid_for(size_t words, const LaunchCfg& c) {
  size_t g = (words + c.block - 1) / c.block;
  if (c.grid_cap > 0 && g > (size_t)c.grid_cap) g = (size_t)c.grid_cap;
  if (g > 0x7FFFFFFFu) g = 0x7FFFFFFFu;
  if (g == 0) g = 1;
  return (unsigned)g;
}

// Dispatch helpers: party count is a template parameter for 1..4 (the
// configurations Amphora deploys), runtime loop above that.

}  // namespace

hipError_t launch_recombine_verify(const OdoSet& odo, int n, size_t words, uint4* out_y,
                                   unsigned long long* ff, const Fp& f, const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  const unsigned g = grid_for(words, c);
#define L(NP, BIG) AMPH_LAUNCH((k_rv<NP, BIG>), dim3(g), dim3(c.block), c, odo, n, words, out_y, ff, f, (size_t)0)
  if (f.big) { AMPH_DISPATCH_NP(n, true, L) } else { AMPH_DISPATCH_NP(n, false, L) }
#undef L
  return hipGetLastError();
}

hipError_t launch_mask_input(const OdoSet& odo, int n, size_t words, const uint4* secrets,
                             size_t n_secrets, uint4* out, unsigned long long* ff, const Fp& f,
                             const LaunchCfg& c) {
  if (n_secrets > words) n_secrets = words;
  if (n_secrets > 0) {
    const unsigned g = grid_for(n_secrets, c);
    LaunchCfg c1 = c;  // timing events bracket both launches when there is a tail
    if (words > n_secrets) c1.ev_stop = nullptr;
#define L(NP, BIG) AMPH_LAUNCH((k_mask<NP, BIG>), dim3(g), dim3(c.block), c1, odo, n, n_secrets, secrets, out, ff, f)
    if (f.big) { AMPH_DISPATCH_NP(n, true, L) } else { AMPH_DISPATCH_NP(n, false, L) }
#undef L
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (words > n_secrets) {
    // verify-only tail, reporting global word indices into the same word
    OdoSet tail = odo;
    for (int k = 0; k < 5; ++k)
      for (int j = 0; j < n; ++j) tail.f[k][j] = odo.f[k][j] + n_secrets;
    const size_t tw = words - n_secrets;
    const unsigned g = grid_for(tw, c);
    LaunchCfg c2 = c;
    if (n_secrets > 0) c2.ev_start = nullptr;
#define L(NP, BIG) AMPH_LAUNCH((k_rv<NP, BIG, false>), dim3(g), dim3(c.block), c2, tail, n, tw, (uint4*)nullptr, ff, f, n_secrets)
    if (f.big) { AMPH_DISPATCH_NP(n, true, L) } else { AMPH_DISPATCH_NP(n, false, L) }
#undef L
  }
  return hipGetLastError();
}

hipError_t launch_recombine(const ShareSet& sh, int n, size_t words, uint4* out, const Fp& f,
                            const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  const unsigned g = grid_for(words, c);
#define L(NP, BIG) AMPH_LAUNCH((k_recombine<NP, BIG>), dim3(g), dim3(c.block), c, sh, n, words, out, f)
  if (f.big) { AMPH_DISPATCH_NP(n, true, L) } else { AMPH_DISPATCH_NP(n, false, L) }
#undef L
  return hipGetLastError();
}

hipError_t launch_verify(const uint4* y, const uint4* r, const uint4* u, const uint4* v,
                         const uint4* w, size_t words, unsigned long long* ff, const Fp& f,
                         const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  const unsigned g = grid_for(words, c);
  if (f.big) AMPH_LAUNCH((k_verify<true>), dim3(g), dim3(c.block), c, y, r, u, v, w, words, ff, f);
  else AMPH_LAUNCH((k_verify<false>), dim3(g), dim3(c.block), c, y, r, u, v, w, words, ff, f);
  return hipGetLastError();
}

hipError_t launch_convert_share(const uint4* masked, const uint4* tuples, size_t words, W4 alpha,
                                int use_zero, uint4* out, const Fp& f, const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  const dim3 g((unsigned)((words + kPairBlock - 1) / kPairBlock));
  if (f.big) AMPH_LAUNCH((k_conv<true>), g, dim3(kPairBlock), c, masked, tuples, words, alpha, use_zero, out, f);
  else AMPH_LAUNCH((k_conv<false>), g, dim3(kPairBlock), c, masked, tuples, words, alpha, use_zero, out, f);
  return hipGetLastError();
}

hipError_t launch_odo_pre(const uint4* share_data, int stride_w, const uint4* masks,
                          const uint4* triples, size_t words, uint4* oy, uint4* orr, uint4* ov,
                          uint4* omag, uint32_t* oneg, const Fp& f, const LaunchCfg& c, uint64_t* lens) {
  if (words == 0) return hipSuccess;
  const size_t pairs = 2 * words;
  static_assert(kPairBlock == kXLenPairs, "one exchange length per K_ODO_PRE workgroup");
  const dim3 g((unsigned)((pairs + kPairBlock - 1) / kPairBlock));
  if (lens)
    AMPH_LAUNCH(k_odo_pre<true>, g, dim3(kPairBlock), c, share_data, stride_w, masks, triples, pairs, oy, orr, ov,
                omag, (uint16_t*)oneg, f, lens);
  else
    AMPH_LAUNCH(k_odo_pre<false>, g, dim3(kPairBlock), c, share_data, stride_w, masks, triples, pairs, oy, orr, ov,
                omag, (uint16_t*)oneg, f, lens);
  return hipGetLastError();
}

hipError_t launch_open_diffs(const SignedSet& d, int n, size_t words, uint4* out, const Fp& f,
                             const LaunchCfg& c) {
  for (int j = 0; j < n; ++j)
    if (d.sbase[j]) return hipErrorInvalidValue;  // span form: k_open_post only
  if (words == 0) return hipSuccess;
  const size_t nvals = 4 * words;
  const unsigned g = grid_for(nvals, c);
#define L(NP, BIG) AMPH_LAUNCH((k_open<NP, BIG>), dim3(g), dim3(c.block), c, d, n, nvals, out, f)
  if (f.big) { AMPH_DISPATCH_NP(n, true, L) } else { AMPH_DISPATCH_NP(n, false, L) }
#undef L
  return hipGetLastError();
}

hipError_t launch_odo_post(const uint4* opened, const uint4* triples, size_t words, int p0,
                           uint4* ow, uint4* ou, const Fp& f, const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  const size_t pairs = 2 * words;
  const dim3 g((unsigned)((pairs + kPairBlock - 1) / kPairBlock));
  if (f.big) AMPH_LAUNCH((k_odo_post<true>), g, dim3(kPairBlock), c, opened, triples, pairs, p0, ow, ou, f);
  else AMPH_LAUNCH((k_odo_post<false>), g, dim3(kPairBlock), c, opened, triples, pairs, p0, ow, ou, f);
  return hipGetLastError();
}

hipError_t launch_open_post(const SignedSet& d, int n, const uint4* triples, size_t words, int p0,
                            uint4* ow, uint4* ou, const Fp& f, const LaunchCfg& c, bool stage_mag) {
  for (int j = 0; j < n && stage_mag; ++j)
    if (d.sbase[j]) return hipErrorInvalidValue;  // span form: direct loads only
  if (words == 0) return hipSuccess;
  const size_t pairs = 2 * words;
  const dim3 g((unsigned)((pairs + kPairBlock - 1) / kPairBlock));
  // span-form partners: all of parties 1 .. n-1 (the session), never party 0
  const bool span = n > 1 && d.sbase[1];
  for (int j = 0; j < n; ++j)
    if ((d.sbase[j] != nullptr) != (span && j > 0)) return hipErrorInvalidValue;
#define L(NP, BIG)                                                                                        \
  if (stage_mag) AMPH_LAUNCH((k_open_post<NP, BIG, true, false>), g, dim3(kPairBlock), c, d, n, triples, \
                             pairs, p0, ow, ou, f);                                                      \
  else if (span) AMPH_LAUNCH((k_open_post<NP, BIG, false, true>), g, dim3(kPairBlock), c, d, n, triples, \
                             pairs, p0, ow, ou, f);                                                      \
  else AMPH_LAUNCH((k_open_post<NP, BIG, false, false>), g, dim3(kPairBlock), c, d, n, triples, pairs,  \
                   p0, ow, ou, f)
  if (f.big) { AMPH_DISPATCH_NP(n, true, L) } else { AMPH_DISPATCH_NP(n, false, L) }
#undef L
  return hipGetLastError();
}

hipError_t launch_to_gfp(const uint4* in, size_t words, uint4* out, const Fp& f,
                         const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  const unsigned g = grid_for(words, c);
  if (f.big) AMPH_LAUNCH((k_to_gfp<true>), dim3(g), dim3(c.block), c, in, words, out, f);
  else AMPH_LAUNCH((k_to_gfp<false>), dim3(g), dim3(c.block), c, in, words, out, f);
  return hipGetLastError();
}

hipError_t launch_from_gfp(const uint4* in, size_t words, uint4* out, const Fp& f,
                           const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  AMPH_LAUNCH(k_from_gfp, dim3(grid_for(words, c)), dim3(c.block), c, in, words, out, f);
  return hipGetLastError();
}

hipError_t launch_mask_words(const uint4* secrets, const uint4* masks, size_t words, uint4* out,
                             const Fp& f, const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  const unsigned g = grid_for(words, c);
  if (f.big) AMPH_LAUNCH((k_mask_words<true>), dim3(g), dim3(c.block), c, secrets, masks, words, out, f);
  else AMPH_LAUNCH((k_mask_words<false>), dim3(g), dim3(c.block), c, secrets, masks, words, out, f);
  return hipGetLastError();
}

hipError_t launch_synth_odos(const OutSet& out, int n, size_t words, uint64_t seed,
                             uint4* plain_y, long long fault, int permille, const Fp& f,
                             const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  const unsigned g = grid_for(words, c);
  if (f.big) AMPH_LAUNCH((k_synth<true>), dim3(g), dim3(c.block), c, out, n, words, seed, plain_y, fault, permille, f);
  else AMPH_LAUNCH((k_synth<false>), dim3(g), dim3(c.block), c, out, n, words, seed, plain_y, fault, permille, f);
  return hipGetLastError();
}

hipError_t launch_stream_probe(const OdoSet& odo, int n, size_t words, const uint4* secrets,
                               uint4* out, const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  const unsigned g = grid_for(words, c);
#define L(NP, BIG) AMPH_LAUNCH((k_stream_probe<NP>), dim3(g), dim3(c.block), c, odo, n, words, secrets, out)
  AMPH_DISPATCH_NP(n, false, L)
#undef L
  return hipGetLastError();
}

namespace {
// Small host calls (capi.hip run_small): the verdict words the kernels
// atomicMin'd into device memory go to the page-locked staging arena with
// plain vector stores, and are reset to kNoFail for the next call.
__global__ void k_take_words(unsigned long long* dev, unsigned long long* host, int n) {
  const int i = threadIdx.x;
  if (i < n) {
    host[i] = dev[i];
    dev[i] = kNoFail;
  }
}
}  // namespace

namespace {
// Device-mode party session (capi.hip amph_party_finish_b64_dev): if any
// partner text's verdict word reports a failure, the five base64 fields are
// made unusable -- their first unit becomes "!!!!", which no base64 decoder
// accepts -- so a response sent without checking the verdicts cannot carry
// values computed from a rejected text.
__global__ void k_poison_b64(PoisonB64 a) {
  bool bad = false;
  for (int i = 0; i < a.n_bad; ++i) bad |= *a.bad[i] != kNoFail;
  const int t = threadIdx.x;
  if (bad && t < 20) a.field[t / 4][t % 4] = '!';
}
}  // namespace

hipError_t launch_poison_b64(const PoisonB64& a, hipStream_t s) {
  if (a.n_bad <= 0 || a.chars < 4) return hipSuccess;
  hipLaunchKernelGGL(k_poison_b64, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_take_words(unsigned long long* dev, unsigned long long* host, int n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_take_words, dim3(1), dim3(64), 0, s, dev, host, n);
  return hipGetLastError();
}

// Ragged-party tail (capi.hip, ragged_*): the verdict of a one-word call over
// word `base` min-combined into the whole call's first-fail word.
__global__ void k_ff_merge(unsigned long long* ff, const unsigned long long* tail, unsigned long long base) {
  if (threadIdx.x == 0) {
    const unsigned long long t = *tail;
    if (t != kNoFail) atomicMin(ff, base + t);
  }
}

hipError_t launch_ff_merge(unsigned long long* ff, const unsigned long long* tail, size_t base,
                           hipStream_t s) {
  hipLaunchKernelGGL(k_ff_merge, dim3(1), dim3(64), 0, s, ff, tail, (unsigned long long)base);
  return hipGetLastError();
}

hipError_t launch_synth_words(uint4* out, size_t count, uint64_t seed, const Fp& f,
                              const LaunchCfg& c) {
  if (count == 0) return hipSuccess;
  const unsigned g = grid_for(count, c);
  if (f.big) AMPH_LAUNCH((k_synth_words<true>), dim3(g), dim3(c.block), c, out, count, seed, f);
  else AMPH_LAUNCH((k_synth_words<false>), dim3(g), dim3(c.block), c, out, count, seed, f);
  return hipGetLastError();
}

}  // namespace amph

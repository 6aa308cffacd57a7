// Beaver open exchange wire codec (gfx950) -- SURVEY.md 8f rank 4.
//
// Each party sends its unreduced signed diffs (d_k, e_k) to every partner as
// MultiplicationExchangeObject.interimValues, a JSON array of FactorPair
// objects whose fields are BigIntegers written as plain JSON numbers by
// Jackson (amphora-common/.../MultiplicationExchangeObject.java:20-39,
// FactorPair.java:16-25; built in OutputDeliveryService.java:186-200, read
// back by recombineDiffs :231-272):
//
//     [{"a":10,"b":25},{"a":-39,"b":24},...]
//
// Encode (diffs -> compact array text, byte-identical to Jackson's default
// output): a pass that sums each workgroup's entry lengths, a scan of those
// sums, and a write pass that places its entries with a workgroup scan,
// formats them into LDS and stores the contiguous run with aligned 16-byte
// stores.
//
// Decode (array text -> diffs): values are numbered by the colon before them
// ("k":NUM).  Every lane counts the colons in its bytes; the counts are
// scanned per workgroup, and the value after each colon is parsed at its
// global number index.  Each number's key ("a" / "b"),
// the object it sits in (member 0 after '{', member 1 after ','), the other
// member's key and the closing '}' are checked locally, so the pairing is
// validated without a second pass; the first malformed byte's offset is
// reported.  Whitespace between tokens is accepted, as in any JSON reader.
//
// Decimal conversion: 128-bit magnitude <-> five base-10^9 chunks (nine
// 64-by-32-bit divisions by a constant in all, to_chunks), chunks <-> digits.
#include <hip/hip_ext.h>

#include "kernels.hpp"

namespace amph {

#define AMPH_LAUNCH(K, G, B, C, ...) \
  hipExtLaunchKernelGGL(K, G, B, 0, (C).stream, (C).ev_start, (C).ev_stop, 0, __VA_ARGS__)

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Encoded text and fast-path decoded magnitudes leave through nontemporal
// stores (AMPH_CODEC_NT=0 for A/B).
#ifndef AMPH_CODEC_NT
#define AMPH_CODEC_NT 1
#endif
__device__ __forceinline__ void xst16(uint4* p, uint4 v) {
  if constexpr (AMPH_CODEC_NT) __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(p));
  else *p = v;
}

constexpr int kXBlock = 256;      // pairs per workgroup (encode)
constexpr int kXEntry = 92;       // max entry: {"a":-<39 digits>,"b":-<39 digits>},
constexpr int kDecBytes = 32;     // text bytes per lane (decode)
constexpr uint64_t kE9 = 1000000000ull;

__device__ __forceinline__ int ndigits32(uint32_t x) {  // x < 10^9; 0 -> 1
  int n = 1;
#pragma unroll
  for (uint32_t t = 10; t <= 100000000u; t *= 10) n += x >= t;
  return n;
}

// One base-2^32 long-division step by 10^9: (rem, x) -> quotient, rem updated.
__device__ __forceinline__ uint32_t div_step_e9(uint64_t& rem, uint32_t x) {
  const uint64_t cur = (rem << 32) | x;
  const uint64_t q = cur / kE9;  // < 2^32: rem < 10^9
  rem = cur - q * kE9;
  return (uint32_t)q;
}

// 128-bit magnitude -> base-10^9 chunks (little end first); returns the
// decimal digit count (1 for zero).  Any x < 2^128 leaves x / 10^9 < 2^98.1,
// x / 10^18 < 2^68.2, x / 10^27 < 2^38.3 and x / 10^36 < 2^8.4, so after
// each round the leading limb is known to be below 10^9 (it becomes the
// next round's starting remainder with no division) and one more limb is
// zero: 9 64-bit divisions + 1 32-bit one instead of 5 rounds x 4.
__device__ __forceinline__ int to_chunks(const uint4& m, uint32_t (&ch)[5]) {
  uint64_t rem = 0;
  const uint32_t a3 = m.w / (uint32_t)kE9;  // < 5
  rem = m.w - a3 * (uint32_t)kE9;
  const uint32_t a2 = div_step_e9(rem, m.z), a1 = div_step_e9(rem, m.y);
  const uint32_t a0 = div_step_e9(rem, m.x);
  ch[0] = (uint32_t)rem;
  rem = a3;  // x / 10^9 = (a3, a2, a1, a0) < 2^98.1
  const uint32_t b2 = div_step_e9(rem, a2), b1 = div_step_e9(rem, a1);
  const uint32_t b0 = div_step_e9(rem, a0);
  ch[1] = (uint32_t)rem;
  rem = b2;  // x / 10^18 = (b2, b1, b0) < 2^68.2
  const uint32_t c1 = div_step_e9(rem, b1), c0 = div_step_e9(rem, b0);
  ch[2] = (uint32_t)rem;
  rem = c1;  // x / 10^27 = (c1, c0) < 2^38.3
  const uint32_t d0 = div_step_e9(rem, c0);
  ch[3] = (uint32_t)rem;
  ch[4] = d0;  // x / 10^36 < 2^8.4
  int top = 0;
#pragma unroll
  for (int k = 1; k < 5; ++k) top = ch[k] ? k : top;
  return 9 * top + ndigits32(ch[top]);
}

__device__ __forceinline__ bool is_zero(const uint4& m) { return (m.x | m.y | m.z | m.w) == 0; }

// 10^0 .. 10^38 as 128-bit little-endian limbs (10^38 < 2^128 < 10^39)
__device__ const uint32_t kPow10[39][4] = {
    {0x00000001u, 0x00000000u, 0x00000000u, 0x00000000u},
    {0x0000000au, 0x00000000u, 0x00000000u, 0x00000000u},
    {0x00000064u, 0x00000000u, 0x00000000u, 0x00000000u},
    {0x000003e8u, 0x00000000u, 0x00000000u, 0x00000000u},
    {0x00002710u, 0x00000000u, 0x00000000u, 0x00000000u},
    {0x000186a0u, 0x00000000u, 0x00000000u, 0x00000000u},
    {0x000f4240u, 0x00000000u, 0x00000000u, 0x00000000u},
    {0x00989680u, 0x00000000u, 0x00000000u, 0x00000000u},
    {0x05f5e100u, 0x00000000u, 0x00000000u, 0x00000000u},
    {0x3b9aca00u, 0x00000000u, 0x00000000u, 0x00000000u},
    {0x540be400u, 0x00000002u, 0x00000000u, 0x00000000u},
    {0x4876e800u, 0x00000017u, 0x00000000u, 0x00000000u},
    {0xd4a51000u, 0x000000e8u, 0x00000000u, 0x00000000u},
    {0x4e72a000u, 0x00000918u, 0x00000000u, 0x00000000u},
    {0x107a4000u, 0x00005af3u, 0x00000000u, 0x00000000u},
    {0xa4c68000u, 0x00038d7eu, 0x00000000u, 0x00000000u},
    {0x6fc10000u, 0x002386f2u, 0x00000000u, 0x00000000u},
    {0x5d8a0000u, 0x01634578u, 0x00000000u, 0x00000000u},
    {0xa7640000u, 0x0de0b6b3u, 0x00000000u, 0x00000000u},
    {0x89e80000u, 0x8ac72304u, 0x00000000u, 0x00000000u},
    {0x63100000u, 0x6bc75e2du, 0x00000005u, 0x00000000u},
    {0xdea00000u, 0x35c9adc5u, 0x00000036u, 0x00000000u},
    {0xb2400000u, 0x19e0c9bau, 0x0000021eu, 0x00000000u},
    {0xf6800000u, 0x02c7e14au, 0x0000152du, 0x00000000u},
    {0xa1000000u, 0x1bceccedu, 0x0000d3c2u, 0x00000000u},
    {0x4a000000u, 0x16140148u, 0x00084595u, 0x00000000u},
    {0xe4000000u, 0xdcc80cd2u, 0x0052b7d2u, 0x00000000u},
    {0xe8000000u, 0x9fd0803cu, 0x033b2e3cu, 0x00000000u},
    {0x10000000u, 0x3e250261u, 0x204fce5eu, 0x00000000u},
    {0xa0000000u, 0x6d7217cau, 0x431e0faeu, 0x00000001u},
    {0x40000000u, 0x4674edeau, 0x9f2c9cd0u, 0x0000000cu},
    {0x80000000u, 0xc0914b26u, 0x37be2022u, 0x0000007eu},
    {0x00000000u, 0x85acef81u, 0x2d6d415bu, 0x000004eeu},
    {0x00000000u, 0x38c15b0au, 0xc6448d93u, 0x0000314du},
    {0x00000000u, 0x378d8e64u, 0xbead87c0u, 0x0001ed09u},
    {0x00000000u, 0x2b878fe8u, 0x72c74d82u, 0x00134261u},
    {0x00000000u, 0xb34b9f10u, 0x7bc90715u, 0x00c097ceu},
    {0x00000000u, 0x00f436a0u, 0xd5da46d9u, 0x0785ee10u},
    {0x00000000u, 0x098a2240u, 0x5a86c47au, 0x4b3b4ca8u}};

__device__ __forceinline__ bool ge128(const uint4& a, const uint32_t (&b)[4]) {
  uint32_t br;
  __builtin_subc(a.x, b[0], 0u, &br);
  __builtin_subc(a.y, b[1], br, &br);
  __builtin_subc(a.z, b[2], br, &br);
  __builtin_subc(a.w, b[3], br, &br);
  return br == 0;
}

// Decimal digit count of a 128-bit magnitude (1 for zero) without the
// base-10^9 split: t = floor(bits * log10(2)) (bits * 1233 >> 12 is exact
// for bits <= 128) is the count or one less, decided by one compare with 10^t.
__device__ __forceinline__ int ndigits128(const uint4& m) {
  const int bits = m.w ? 128 - __clz(m.w) : m.z ? 96 - __clz(m.z) : m.y ? 64 - __clz(m.y)
                                                                   : 32 - __clz(m.x);
  const int t = (bits * 1233) >> 12;
  const int n = t + (ge128(m, kPow10[t]) ? 1 : 0);
  return n ? n : 1;
}


__device__ __forceinline__ char* put_str(char* o, const char* s) {
  while (*s) *o++ = *s++;
  return o;
}

// x < 10^4 -> its 4 ASCII digits, first digit in the lowest byte
// (x / 100 as x * 5243 >> 19, exact below 43699; then both 2-digit halves
// split by 10 at once in 16-bit fields: y * 103 >> 10 = y / 10 for y < 179)
__device__ __forceinline__ uint32_t ascii4(uint32_t x) {
  const uint32_t a = (x * 5243u) >> 19, b = x - 100u * a;
  const uint32_t p = a | (b << 16);
  const uint32_t q = ((p * 103u) >> 10) & 0x000F000Fu;
  return 0x30303030u | q | ((p - 10u * q) << 8);
}

// nd decimal digits of the chunks ch (to_chunks) at o; returns o + nd.
__device__ __forceinline__ char* put_digits(char* o, const uint32_t (&ch)[5], int nd) {
  // chunk k (base 10^9, little end first) holds text positions
  // [nd - 9 (k + 1), nd - 9 k); its 9 digits come from one division by 10^8,
  // one by 10^4 and two 4-digit SWAR conversions instead of 9 divisions by 10
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int base = nd - 9 * (k + 1);
    if (base + 9 <= 0) break;
    const uint32_t c = ch[k], top = c / 100000000u, r = c - top * 100000000u;
    const uint32_t hi = r / 10000u;
    const uint32_t w0 = ascii4(hi), w1 = ascii4(r - hi * 10000u);
    if (base >= 0) {  // a whole chunk: 1 byte + two (unaligned) 4-byte LDS stores
      o[base] = (char)(0x30u + top);
      __builtin_memcpy(o + base + 1, &w0, 4);
      __builtin_memcpy(o + base + 5, &w1, 4);
      continue;
    }
    const uint32_t dig[9] = {0x30u + top,      w0 & 0xFFu,         (w0 >> 8) & 0xFFu,
                             (w0 >> 16) & 0xFFu, w0 >> 24,          w1 & 0xFFu,
                             (w1 >> 8) & 0xFFu,  (w1 >> 16) & 0xFFu, w1 >> 24};
#pragma unroll
    for (int j = 0; j < 9; ++j)
      if (base + j >= 0) o[base + j] = (char)dig[j];
  }
  return o + nd;
}

// ---- workgroup scans ----------------------------------------------------------------
// Inclusive wave scan of 32-bit values with DPP: row_shr 1/2/4/8 scans each
// 16-lane row, row_bcast 15/31 carries the row totals (6 VALU with DPP
// operands where a __shfl_up ladder costs ~40 VALU and six ds_bpermute).
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

// Exclusive workgroup scan of 32-bit values (the decode's per-lane colon
// counts: <= 32 per lane, <= 8192 per workgroup).
__device__ __forceinline__ uint32_t block_excl_scan32(uint32_t v, uint32_t* total) {
  __shared__ uint32_t wsum32[17];
  const int lane = __lane_id(), wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint32_t inc = wave_incl_scan32(v);
  if (lane == 63) wsum32[wave] = inc;
  __syncthreads();
  if (wave == 0) {
    const uint32_t s = lane < nw ? wsum32[lane] : 0;
    const uint32_t si = wave_incl_scan32(s);
    if (lane < nw) wsum32[lane] = si - s;  // exclusive wave offsets
    if (lane == nw - 1) wsum32[16] = si;
  }
  __syncthreads();
  const uint32_t r = wsum32[wave] + inc - v;
  *total = wsum32[16];
  __syncthreads();
  return r;
}

// ---- hierarchical counts: per-unit bases without scan passes -----------------
// Unit s's count in l0[s] (a decode span's values, an encode block's text
// bytes); l1[s >> 6] = the sum of its 64-unit group (written by the one
// workgroup that counts the group); l2[s >> 12] = the sum of 4096 units (64
// groups; agent-scope atomic adds onto words zeroed by a launch before).  The
// exclusive prefix of unit s is then three masked loads per lane of ONE wave
// and a wave reduction -- l2 below s's 4096-block, l1 of the groups before s
// in it, l0 of the units before s in its group -- issued beside the unit's
// own loads.  This replaced a three-launch scan of the counts (k_scan_reduce
// / single / apply, ~5 us each, mostly launch latency).
struct Hier {
  uint64_t* l0;
  uint64_t* l1;
  uint64_t* l2;
};
constexpr int kGroupSpans = 64;  // units per l1 group = per counting workgroup

// Counts live in bits 0..39 of the words; the decode's single pass marks
// each publication in bits 40..63 (kOne per contributor, see k_xdec_one).
constexpr uint64_t kOne = 1ull << 40, kCountMask = kOne - 1;

// call with a whole wave; every lane returns the prefix
__device__ __forceinline__ uint64_t hier_prefix(const Hier& h, size_t s) {
  const size_t lane = __lane_id();
  uint64_t v = 0;
  for (size_t k = lane; k < (s >> 12); k += 64) v += h.l2[k] & kCountMask;
  const size_t g0 = (s >> 12) << 6, g1 = s >> 6;
  if (g0 + lane < g1) v += h.l1[g0 + lane] & kCountMask;
  const size_t s0 = (s >> 6) << 6;
  if (s0 + lane < s) v += h.l0[s0 + lane] & kCountMask;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// every unit's count: one wave
__device__ __forceinline__ uint64_t hier_total(const Hier& h, size_t n) {
  uint64_t v = 0;
  for (size_t k = __lane_id(); k < ((n + 4095) >> 12); k += 64) v += h.l2[k] & kCountMask;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(256) void k_hier_zero(uint64_t* w, size_t n, unsigned int* flags, int nflags) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) w[i] = 0;
  if (blockIdx.x == 0 && (int)threadIdx.x < nflags) flags[threadIdx.x] = 0;
}

// Encode pass 1: the text length of each 256-pair block's run of entries
// (l0[b] = sum of the entry lengths of pairs [256 b, 256 b + 256)) and the
// l1 / l2 sums of the hierarchy; digit counts from the bit length
// (ndigits128), not the base-10^9 split.  One workgroup per 64 blocks: 16
// rounds of one pair per lane, 4 blocks of 256 pairs per 1024-lane round --
// wave sums by shuffles, then 4 lanes add their block's 4 wave sums.
__global__ __launch_bounds__(4 * kXBlock) void k_xenc_bsum(const uint4* mag, const uint8_t* neg,
                                                       size_t npairs, size_t nb, Hier h) {
  __shared__ uint32_t ws[16];
  uint32_t gsum = 0;  // lanes 0..3: their blocks' lengths over the rounds
  for (int round = 0; round < kGroupSpans / 4; ++round) {
    const size_t b4 = (size_t)blockIdx.x * kGroupSpans + 4 * round;  // this round's first block
    if (b4 >= nb) break;
    const size_t k = b4 * kXBlock + threadIdx.x;
    uint32_t len = 0;
    if (k < npairs) {  // {"a":A,"b":B} (+ ',' unless last)
      const uint4 d = mag[2 * k], e = mag[2 * k + 1];
      len = 11 + ndigits128(d) + (neg[2 * k] != 0 && !is_zero(d)) + ndigits128(e) +
            (neg[2 * k + 1] != 0 && !is_zero(e)) + (k + 1 < npairs);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) len += __shfl_xor(len, o, 64);
    if (__lane_id() == 0) ws[threadIdx.x >> 6] = len;
    __syncthreads();
    const size_t sub = b4 + threadIdx.x;
    if (threadIdx.x < 4 && sub < nb) {
      const uint32_t b = ws[4 * threadIdx.x] + ws[4 * threadIdx.x + 1] + ws[4 * threadIdx.x + 2] +
                         ws[4 * threadIdx.x + 3];
      h.l0[sub] = b;
      gsum += b;
    }
    __syncthreads();
  }
  if (threadIdx.x < 64) {
    uint32_t g = threadIdx.x < 4 ? gsum : 0;
    g += __shfl_xor(g, 1, 64);
    g += __shfl_xor(g, 2, 64);
    if (threadIdx.x == 0) {
      h.l1[blockIdx.x] = g;
      atomicAdd((unsigned long long*)&h.l2[blockIdx.x >> 6], (unsigned long long)g);
    }
  }
}

// Encode pass 3 (after the scan of bs): each lane converts its two numbers,
// the workgroup scans the entry lengths to place them, and the entries are
// formatted into LDS and stored as one contiguous run.  The run sits in LDS
// at the same offset mod 16 as its destination (sh), so every 16-byte unit
// wholly inside it moves as one aligned ds_read_b128 + global 16-byte store;
// the up to 15 bytes at either end go out singly.
__global__ __launch_bounds__(kXBlock) void k_xenc_write(const uint4* mag, const uint8_t* neg,
                                                    size_t npairs, Hier h,
                                                    size_t nblocks, char* out,
                                                    unsigned long long* out_len) {
  __shared__ uint4 bufv[(kXBlock * kXEntry + 8) / 16 + 2];
  __shared__ uint64_t sbase, stotal;
  if (threadIdx.x < 64) {  // this block's text offset (and block 0: the whole text's length)
    const uint64_t b = hier_prefix(h, blockIdx.x);
    const uint64_t t = blockIdx.x == 0 ? hier_total(h, nblocks) : 0;
    if (threadIdx.x == 0) {
      sbase = b;
      stotal = t;
    }
  }
  char* buf = reinterpret_cast<char*>(bufv);
  const size_t k = (size_t)blockIdx.x * kXBlock + threadIdx.x;
  uint32_t cd[5], ce[5];
  int nd = 0, ne = 0;
  bool sd = false, se = false;
  uint32_t len = 0, total;  // <= 92 per entry, <= 23 552 per workgroup
  if (k < npairs) {
    const uint4 d = mag[2 * k], e = mag[2 * k + 1];
    nd = to_chunks(d, cd);
    ne = to_chunks(e, ce);
    sd = neg[2 * k] != 0 && !is_zero(d);  // BigInteger has no negative zero
    se = neg[2 * k + 1] != 0 && !is_zero(e);
    len = 11 + nd + sd + ne + se + (k + 1 < npairs);
  }
  const uint32_t loc = block_excl_scan32(len, &total);  // its barriers publish sbase / stotal
  const uint64_t base = sbase;
  char* dst = out + 1 + base;  // out[0] = '['
  const size_t sh = (uintptr_t)dst & 15;
  if (k < npairs) {
    char* o = buf + sh + loc;
    o = put_str(o, "{\"a\":");
    if (sd) *o++ = '-';
    o = put_digits(o, cd, nd);
    o = put_str(o, ",\"b\":");
    if (se) *o++ = '-';
    o = put_digits(o, ce, ne);
    *o++ = '}';
    if (k + 1 < npairs) *o = ',';
  }
  __syncthreads();
  char* dal = dst - sh;  // 16-aligned; bytes [sh, sh + total) of it are this run
  const size_t endb = sh + total;
  const size_t ulo = sh ? 1 : 0, uhi = endb / 16;  // whole 16-byte units [ulo, uhi)
  if (uhi <= ulo) {
    if (sh + threadIdx.x < endb) dal[sh + threadIdx.x] = buf[sh + threadIdx.x];
  } else {
    if (sh + threadIdx.x < 16 * ulo) dal[sh + threadIdx.x] = buf[sh + threadIdx.x];
    for (size_t u = ulo + threadIdx.x; u < uhi; u += kXBlock)
      xst16(reinterpret_cast<uint4*>(dal) + u, bufv[u]);
    if (16 * uhi + threadIdx.x < endb) dal[16 * uhi + threadIdx.x] = buf[16 * uhi + threadIdx.x];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    out[0] = '[';
    out[1 + stotal] = ']';
    if (out_len) *out_len = stotal + 2;
  }
}

// ---- decode -----------------------------------------------------------------------
// The text is addressed in "virtual" coordinates: v = byte offset from the
// 16-byte-aligned address at or below the text, so every 16-byte chunk load
// is aligned; virtual bytes before the text (v < mis) and after it (v >= L)
// read as ' ' (JSON whitespace).  A chunk that holds a real byte lies in the
// same 16-byte granule as that byte, so it never crosses a page.
struct Text {
  const uint8_t* al;  // aligned base
  size_t mis, L;      // L = mis + len
  __device__ __forceinline__ uint32_t operator[](size_t v) const {
    return v - mis < L - mis ? al[v] : (uint32_t)' ';
  }
  __device__ __forceinline__ uint4 chunk(long long v) const {  // 16-aligned v
    if (v + 16 <= (long long)mis || v >= (long long)L) return make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
    uint4 c = *reinterpret_cast<const uint4*>(al + v);
    if (v < (long long)mis || v + 16 > (long long)L) {
      uint32_t w[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const long long x = v + j;
        if (x < (long long)mis || x >= (long long)L)
          w[j >> 2] = (w[j >> 2] & ~(0xFFu << (8 * (j & 3)))) | (0x20u << (8 * (j & 3)));
      }
      c = make_uint4(w[0], w[1], w[2], w[3]);
    }
    return c;
  }
};

__device__ __forceinline__ bool is_digit(uint32_t c) { return c - '0' < 10u; }
__device__ __forceinline__ bool is_ws(uint32_t c) {
  return c == ' ' || c == '\n' || c == '\r' || c == '\t';
}

// SWAR byte classes on 4 text bytes: bit 7 of byte j set iff byte j is in the class.
__device__ __forceinline__ uint32_t swar_digit(uint32_t w) {
  const uint32_t lo = w & 0x7F7F7F7Fu;
  return (lo + 0x50505050u) & ~(lo + 0x46464646u) & ~w & 0x80808080u;  // 0x30 <= b <= 0x39
}
// Colons in 4 text bytes: bit 7 of byte j set iff byte j is ':' (exact
// zero-byte test of w ^ "::::").  Every number of a FactorPair list follows
// exactly one colon ("k":NUM), so the decoder numbers the values by their
// colons: counting them is 5 VALU ops per 4 bytes where the number-start
// classes of the number tokens took 19, and a colon that is not followed by a number, or a number
// without one, breaks the grammar checks around its neighbours.
__device__ __forceinline__ uint32_t swar_colon(uint32_t w) {
  const uint32_t x = w ^ 0x3A3A3A3Au;
  return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}
// One bit per byte: swar_colon leaves 0x80 in each ':' byte, and one
// v_dot4_u32_u8 per dword with byte weights (1,2,4,8) or (16,32,64,128)
// gathers two dwords' flags into bits 7..14 of their sum (12 VALU per 8 bytes
// where shifting and OR-ing the flags together took ~20).
__device__ __forceinline__ uint32_t colons32(const uint32_t (&w)[8]) {
  uint32_t m = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t hi = __builtin_amdgcn_udot4(swar_colon(w[2 * q + 1]), 0x80402010u, 0u, false);
    const uint32_t a = __builtin_amdgcn_udot4(swar_colon(w[2 * q]), 0x08040201u, hi, false);
    m |= (a >> 7) << (8 * q);
  }
  return m;
}

constexpr int kDecBlock = 256;  // threads per workgroup (512: parse 574 us, 256: 486, 128: 527 at 8 Mi pairs)
constexpr size_t kDecSpan = (size_t)kDecBlock * kDecBytes;  // 8 KiB of text per workgroup
constexpr int kWinPad = 256;                           // window context either side
constexpr int kWin = (int)kDecSpan + 2 * kWinPad;      // staged bytes

// Flags of one decode, zeroed with the counts before the pass (k_hier_zero):
// [0] a workgroup gave up waiting for its predecessors' counts, [1] k_xdec_one
// met a value outside the compact layout.  Either sends the whole text through
// the general pass.
constexpr int kCntWaves = 4;  // (tools/ubench/ubench_xcount.hip's count kernel shape)

// The workgroup's 8 KiB span plus kWinPad bytes either side, staged in LDS;
// bytes outside it (long whitespace runs) come from global memory.
struct Window {
  Text t;
  const uint8_t* lds;
  size_t w0;  // virtual offset of lds[0] (may be "negative": wraps, never in range then)
  __device__ __forceinline__ uint32_t operator[](size_t x) const {
    return x - w0 < (size_t)kWin ? (uint32_t)lds[x - w0] : t[x];
  }
  // 4 bytes starting at x (little-endian)
  __device__ __forceinline__ uint32_t word(size_t x) const {
    const size_t o = x - w0;
    if (o < (size_t)kWin) {  // the window has one spare dword past kWin
      const uint32_t* l32 = reinterpret_cast<const uint32_t*>(lds);
      return __builtin_amdgcn_alignbyte(l32[(o >> 2) + 1], l32[o >> 2], (uint32_t)(o & 3));
    }
    return t[x] | (t[x + 1] << 8) | (t[x + 2] << 16) | (t[x + 3] << 24);
  }
};

template <class T>
__device__ __forceinline__ size_t skip_ws_back(const T& t, size_t q) {  // q: index+1
  while (q > 0 && is_ws(t[q - 1])) --q;
  return q;
}

// Backward from just before a number start x: ws ':' ws '"' key '"' ws.
// Returns the key char (or 0), *q = index+1 of the byte before the key.
template <class T>
__device__ __forceinline__ uint32_t key_before(const T& t, size_t x, size_t* q) {
  size_t p = skip_ws_back(t, x);
  if (p == 0 || t[p - 1] != ':') return 0;
  p = skip_ws_back(t, p - 1);
  if (p < 3 || t[p - 1] != '"' || t[p - 3] != '"') return 0;
  const uint32_t k = t[p - 2];
  if (k != 'a' && k != 'b') return 0;
  *q = skip_ws_back(t, p - 3);
  return k;
}

__device__ __forceinline__ void fold(uint32_t (&v)[4], uint32_t mul, uint32_t add, bool& ovf) {
  uint64_t carry = add;  // v = v * mul + add
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint64_t s = (uint64_t)v[i] * mul + carry;
    v[i] = (uint32_t)s;
    carry = s >> 32;
  }
  ovf |= carry != 0;
}

// 8 ASCII digits (little-endian bytes, first digit lowest) -> value < 10^8:
// v_dot4_u32_u8 forms the four 2-digit pairs straight from the ASCII bytes
// (each offset by 11 * '0' = 528), three 24-bit multiply-adds join them and
// one subtraction removes the offsets (8 VALU where the 16-bit-field SWAR
// took ~15).
__device__ __forceinline__ uint32_t digits8(uint32_t lo, uint32_t hi) {
  const uint32_t a = __builtin_amdgcn_udot4(lo, 0x0000010Au, 0u, false);  // 10 d0 + d1 + 528
  const uint32_t b = __builtin_amdgcn_udot4(lo, 0x010A0000u, 0u, false);  // 10 d2 + d3 + 528
  const uint32_t c = __builtin_amdgcn_udot4(hi, 0x0000010Au, 0u, false);
  const uint32_t d = __builtin_amdgcn_udot4(hi, 0x010A0000u, 0u, false);
  const uint32_t ab = __umul24(a, 100u) + b, cd = __umul24(c, 100u) + d;  // <= 63327
  return __umul24(ab, 10000u) + cd - 528u * 1010101u;
}
__device__ __forceinline__ uint32_t pow10_small(uint32_t k) {  // k <= 7
  return __umul24(__umul24((k & 1u) ? 10u : 1u, (k & 2u) ? 100u : 1u), (k & 4u) ? 10000u : 1u);
}

// Length of the digit run at the start of the 44 bytes d[0..10] (44 if all
// are digits): SWAR non-digit flags (0x80 per byte), packed one bit per byte
// by v_dot4_u32_u8 as in colons32, and one 64-bit count of trailing zeros
// (where a compare-and-select chain over the 11 dwords took twice the VALU).
__device__ __forceinline__ uint32_t digit_run(const uint32_t (&d)[11]) {
  uint64_t mask = 1ull << 44;
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    uint32_t nd2[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = 2 * q + h;
      const uint32_t x = (j < 11 ? d[j] : 0u) ^ 0x30303030u;  // digits -> 0..9
      nd2[h] = (((x & 0x7F7F7F7Fu) + 0x76767676u) | x) & 0x80808080u;
    }
    const uint32_t a = __builtin_amdgcn_udot4(nd2[0], 0x08040201u,
                                              __builtin_amdgcn_udot4(nd2[1], 0x80402010u, 0u, false), false);
    mask |= (uint64_t)(a >> 7) << (8 * q);
  }
  return (uint32_t)__builtin_ctzll(mask);
}

// Fast path for the layout Jackson writes (no whitespace):
//   member 0 (not the first pair):  <digit> '}' ',' '{' '"' k '"' ':' NUM ','
//   member 1:                <digit> ',' '"' k '"' ':' NUM '}'
// with every byte read from the LDS window as whole dwords (independent
// ds_read_b32 + v_alignbyte, no byte-by-byte walk): the digit run is found
// with SWAR over 44 bytes held in registers, and the value is folded in
// base 10^8 from the same registers: full 8-digit chunks, then the partial
// last chunk right-aligned behind '0's.  Returns false for anything else
// (whitespace, the first or last pair, a leading zero, more than 39 digits,
// an overflow, a malformed neighbour):
// the general path then parses the number and reports any error, so both
// paths accept exactly the same texts.  o = the start's offset in the window
// (>= kWinPad, so every read below stays inside it).
struct FastNum {
  uint32_t v[4];
  uint32_t dend;   // window offset one past the last digit
  uint32_t key;    // 'a' / 'b'
  bool minus;
};

__device__ __forceinline__ uint32_t lds_dword(const uint32_t* l32, uint32_t o) {
  return __builtin_amdgcn_alignbyte(l32[(o >> 2) + 1], l32[o >> 2], o & 3u);
}

// The number at window offset o: '-'? then 1..39 digits without a leading
// zero, value < 2^128, followed by what after_ok(one past its last digit)
// accepts (sets r.v, r.minus, r.dend; ok: the caller's own checks so far).
// The digit run is found with SWAR over 44 bytes held in registers; the
// value is folded in base 10^8 from the same registers: full 8-digit
// chunks, then the nd % 8 leading digits of the next chunk right-aligned
// behind '0's.
template <class AfterOk>
__device__ __forceinline__ bool fast_parse(const uint32_t* l32, uint32_t o, bool ok, FastNum& r,
                                           AfterOk after_ok) {
  const uint32_t first = lds_dword(l32, o);
  r.minus = (first & 0xFFu) == (uint32_t)'-';
  const uint32_t ds = o + (r.minus ? 1u : 0u);
  uint32_t d[11];
#pragma unroll
  for (int j = 0; j < 11; ++j) d[j] = lds_dword(l32, ds + 4 * j);
  const uint32_t nd = digit_run(d);
  ok = ok && nd >= 1 && nd <= 39 && !((d[0] & 0xFFu) == (uint32_t)'0' && nd > 1);
  if (!ok) return false;
  r.dend = ds + nd;
  if (!after_ok(r.dend)) return false;
  const uint32_t full = nd >> 3, rem = nd & 7u;
  bool ovf = false;
  if (full == 4) {  // 32..39 digits (a random 128-bit value): two 16-digit halves
    const uint64_t p0 = (uint64_t)digits8(d[0], d[1]) * 100000000u + digits8(d[2], d[3]);
    const uint64_t p1 = (uint64_t)digits8(d[4], d[5]) * 100000000u + digits8(d[6], d[7]);
    const unsigned __int128 t = (unsigned __int128)p0 * 10000000000000000ull + p1;  // < 10^32
    r.v[0] = (uint32_t)t;
    r.v[1] = (uint32_t)(t >> 32);
    r.v[2] = (uint32_t)(t >> 64);
    r.v[3] = (uint32_t)(t >> 96);
  } else {
    r.v[0] = r.v[1] = r.v[2] = r.v[3] = 0;
#pragma unroll
    for (uint32_t m = 0; m < 4; ++m)
      if (m < full) fold(r.v, 100000000u, digits8(d[2 * m], d[2 * m + 1]), ovf);
  }
  if (rem) {
    uint32_t lo = d[0], hi = d[1];
#pragma unroll
    for (uint32_t m = 1; m < 5; ++m)
      if (m == full) { lo = d[2 * m]; hi = d[2 * m + 1]; }
    const uint64_t x = ((uint64_t)hi << 32) | lo;
    const uint32_t sh = 8 * (8 - rem);  // 8..56
    const uint64_t y = (x << sh) | (0x3030303030303030ull >> (64 - sh));
    fold(r.v, pow10_small(rem), digits8((uint32_t)y, (uint32_t)(y >> 32)), ovf);
  }
  return !ovf;
}

// The general pass's fast path (checks the context BEFORE the number; the
// digit scan and conversion as fast_parse, kept separate: inlined through
// fast_parse's lambda it cost the general kernel 20 bytes of scratch).
__device__ __forceinline__ bool fast_number(const uint32_t* l32, uint32_t o, bool member0,
                                            FastNum& r) {
  const uint32_t pre0 = lds_dword(l32, o - 8), pre1 = lds_dword(l32, o - 4);
  // bytes o-4 .. o-1 = '"' k '"' ':'
  r.key = (pre1 >> 8) & 0xFFu;
  bool ok = (pre1 & 0xFFFF00FFu) == 0x3A220022u && (r.key == 'a' || r.key == 'b');
  if (member0)  // bytes o-8 .. o-5 = <digit> '}' ',' '{'
    ok = ok && (pre0 & 0xFFFFFF00u) == 0x7B2C7D00u && is_digit(pre0 & 0xFFu);
  else  // bytes o-6 .. o-5 = <digit> ',' (member 0's digits end right at the ',')
    ok = ok && (pre0 >> 24) == (uint32_t)',' && is_digit((pre0 >> 16) & 0xFFu);
  const uint32_t first = lds_dword(l32, o);
  r.minus = (first & 0xFFu) == (uint32_t)'-';
  const uint32_t ds = o + (r.minus ? 1u : 0u);
  uint32_t d[11];
#pragma unroll
  for (int j = 0; j < 11; ++j) d[j] = lds_dword(l32, ds + 4 * j);
  const uint32_t nd = digit_run(d);
  ok = ok && nd >= 1 && nd <= 39 && !((d[0] & 0xFFu) == (uint32_t)'0' && nd > 1);
  if (!ok) return false;
  r.dend = ds + nd;
  const uint32_t after = lds_dword(l32, r.dend) & 0xFFu;
  if (after != (member0 ? (uint32_t)',' : (uint32_t)'}')) return false;
  // full 8-digit chunks straight from the registers, then the rem = nd % 8
  // leading digits of the next chunk right-aligned behind '0's
  const uint32_t full = nd >> 3, rem = nd & 7u;
  bool ovf = false;
  if (full == 4) {  // 32..39 digits (a random 128-bit value): two 16-digit halves
    const uint64_t p0 = (uint64_t)digits8(d[0], d[1]) * 100000000u + digits8(d[2], d[3]);
    const uint64_t p1 = (uint64_t)digits8(d[4], d[5]) * 100000000u + digits8(d[6], d[7]);
    const unsigned __int128 t = (unsigned __int128)p0 * 10000000000000000ull + p1;  // < 10^32
    r.v[0] = (uint32_t)t;
    r.v[1] = (uint32_t)(t >> 32);
    r.v[2] = (uint32_t)(t >> 64);
    r.v[3] = (uint32_t)(t >> 96);
  } else {
    r.v[0] = r.v[1] = r.v[2] = r.v[3] = 0;
#pragma unroll
    for (uint32_t m = 0; m < 4; ++m)
      if (m < full) fold(r.v, 100000000u, digits8(d[2 * m], d[2 * m + 1]), ovf);
  }
  if (rem) {
    uint32_t lo = d[0], hi = d[1];
#pragma unroll
    for (uint32_t m = 1; m < 5; ++m)
      if (m == full) { lo = d[2 * m]; hi = d[2 * m + 1]; }
    const uint64_t x = ((uint64_t)hi << 32) | lo;
    const uint32_t sh = 8 * (8 - rem);  // 8..56
    const uint64_t y = (x << sh) | (0x3030303030303030ull >> (64 - sh));
    fold(r.v, pow10_small(rem), digits8((uint32_t)y, (uint32_t)(y >> 32)), ovf);
  }
  return !ovf;
}

// Value g's SEGMENT in the compact layout, from the byte after its colon to
// the next value's colon:
//   NUM ',' '"' K '"' ':'            member 0 (K the other key)
//   NUM '}' ',' '{' '"' K '"' ':'    member 1
//   NUM '}' ']' <end of text>        the last value
// plus its own key ('"' k '"' before the colon; value 0: the text starts
// '[' '{' '"' k '"' ':').  The segments of all values tile the text from
// its first byte to its last, so when every value's segment holds, the
// whole array is well-formed; no neighbour's record is needed.
// xo: absolute text offset of window offset o; len: the text length.
__device__ __forceinline__ bool fast_segment(const uint32_t* l32, uint32_t o, uint64_t g,
                                             size_t nvals, size_t xo, size_t len, FastNum& r) {
  const uint32_t pre = lds_dword(l32, o - 4);
  r.key = (pre >> 8) & 0xFFu;
  bool ok = (pre & 0xFFFF00FFu) == 0x3A220022u && (r.key == 'a' || r.key == 'b');
  if (g == 0) ok = ok && xo == 6 && (lds_dword(l32, o - 6) & 0xFFFFu) == 0x7B5Bu;  // "[{"
  const uint32_t key = r.key;
  return fast_parse(l32, o, ok, r, [=](uint32_t dend) {
    const uint32_t a0 = lds_dword(l32, dend), a1 = lds_dword(l32, dend + 4);
    if ((g & 1) == 0) {
      const uint32_t k = (a0 >> 16) & 0xFFu;
      return (a0 & 0xFF00FFFFu) == 0x2200222Cu && (k == 'a' || k == 'b') && k != key &&
             (a1 & 0xFFu) == (uint32_t)':';
    }
    if (g + 1 == nvals) return (a0 & 0xFFFFu) == 0x5D7Du && xo + (dend - o) + 2 == len;  // "}]"
    const uint32_t k = a1 & 0xFFu;
    return a0 == 0x227B2C7Du && (a1 & 0x00FFFF00u) == 0x003A2200u && (k == 'a' || k == 'b');
  });
}

// fast_segment without the value's global index (k_xdec_one parses before
// its span's first index is known): the member comes from the byte before the
// key's quote ('{' member 0, ',' member 1 -- that byte ends the previous
// value's segment, which checks it), and the parts of the check that depend
// on the index are returned for k_xdec_one to apply once it knows it:
//   SEG_OK     every index-independent check held (the member's own form);
//   SEG_M1     member 1 (the index must be odd);
//   SEG_FIRST  the value opens the text ("[{" and the 6th byte: needed if g == 0);
//   SEG_LAST   member 1 closing the text ("}]" and the end: needed if g + 1 == nvals);
//   SEG_MID    member 1 followed by the next pair ("},{"K":": needed otherwise).
enum : uint32_t { SEG_OK = 1, SEG_M1 = 2, SEG_FIRST = 4, SEG_LAST = 8, SEG_MID = 16 };

__device__ __forceinline__ uint32_t fast_value(const uint32_t* l32, uint32_t o, size_t xo, size_t len,
                                               FastNum& r) {
  const uint32_t pre = lds_dword(l32, o - 5);  // bytes o-5 .. o-2: '{'|',' '"' k '"'
  r.key = (pre >> 16) & 0xFFu;
  const uint32_t lead = pre & 0xFFu;
  const bool m1 = lead == (uint32_t)',';
  bool ok = (pre & 0xFF00FF00u) == 0x22002200u && (r.key == 'a' || r.key == 'b') &&
            (lead == (uint32_t)'{' || m1) && (lds_dword(l32, o - 1) & 0xFFu) == (uint32_t)':';
  uint32_t flags = m1 ? SEG_M1 : 0;
  if (xo == 6 && (lds_dword(l32, o - 6) & 0xFFFFu) == 0x7B5Bu) flags |= SEG_FIRST;  // "[{"
  const uint32_t key = r.key;
  ok = fast_parse(l32, o, ok, r, [&](uint32_t dend) {
    const uint32_t a0 = lds_dword(l32, dend), a1 = lds_dword(l32, dend + 4);
    if (!m1) {  // NUM ',' '"' K '"' ':', K the other key
      const uint32_t k = (a0 >> 16) & 0xFFu;
      return (a0 & 0xFF00FFFFu) == 0x2200222Cu && (k == 'a' || k == 'b') && k != key &&
             (a1 & 0xFFu) == (uint32_t)':';
    }
    if ((a0 & 0xFFFFu) == 0x5D7Du && xo + (dend - o) + 2 == len) flags |= SEG_LAST;  // "}]" + end
    const uint32_t k = a1 & 0xFFu;
    if (a0 == 0x227B2C7Du && (a1 & 0x00FFFF00u) == 0x003A2200u && (k == 'a' || k == 'b')) flags |= SEG_MID;
    return (flags & (SEG_LAST | SEG_MID)) != 0;
  });
  return ok ? flags | SEG_OK : flags;
}

__device__ __forceinline__ bool segment_holds(uint32_t f, uint64_t g, size_t nvals) {
  if (!(f & SEG_OK) || g >= nvals || ((f & SEG_M1) != 0) != ((g & 1) != 0)) return false;
  if (g == 0 && !(f & SEG_FIRST)) return false;
  if (f & SEG_M1) return (f & (g + 1 == nvals ? SEG_LAST : SEG_MID)) != 0;
  return true;
}

// Pass 3, general (k_xdec_slow, one workgroup per span; its workgroups
// return at once unless k_xdec_one found a value outside the compact
// layout): each
// workgroup finds its colons again (from LDS), scans them to
// global number indices and lists their positions in LDS; then its
// lanes take ONE NUMBER EACH, consecutive numbers on consecutive lanes (so a
// wave's trip counts match), read the digits four at a time (SWAR) and check
// the grammar around the number:
//   member 0: '[' ws | '}' ws ',' ws (after the previous pair's digits), then
//             '{' ws "k" ws ':' ws NUM ws ','
//   member 1: ',' ws "k" ws ':' ws NUM ws '}'  (last pair: ws ']' ws EOF)
// Phase 1 does each number's own checks and records in LDS where its digits
// end, its key, and (member 1) where the text before its ',' ends; phase 2
// ties each member 1 to the member 0 before it (same ',', other key), so
// together they cover every byte of a well-formed array.  A well-formed text
// has at most kMaxStarts numbers per 8 KiB span ({"a":1,"b":2}, = 14 bytes per 2);
// a colon beyond that is reported as malformed.
constexpr int kMaxStarts = 1280;

// Launched with a small grid (kSlowGrid workgroups), each workgroup taking
// spans blockIdx.x, + gridDim.x, ...: when k_xdec_one held, every workgroup
// returns at once, and 1024 of them cost ~2 us where one per span (92 k for
// 752 MB) cost 21 us of dispatch.
constexpr unsigned kSlowGrid = 1024;

__global__ __launch_bounds__(kDecBlock) void k_xdec_slow(Text text, Hier h, size_t nb,
                                                     size_t nvals, uint4* mag, uint8_t* neg,
                                                     unsigned long long* bad,
                                                     const unsigned int* flags) {
  if (flags[0] == 0 && flags[1] == 0) return;  // k_xdec_one held
  __shared__ uint4 win4[kWin / 16 + 1];
  __shared__ uint16_t pos[kMaxStarts];   // start, relative to b0
  __shared__ uint16_t endp[kMaxStarts];  // one past the last digit, relative to w0
  __shared__ uint16_t comma[kMaxStarts]; // member 1: one past the last byte before its ',', rel. w0
  __shared__ uint8_t keyc[kMaxStarts];   // 'a' / 'b', 0 if the number failed its own checks
  __shared__ uint64_t sbase;
  for (size_t span = blockIdx.x; span < nb; span += gridDim.x) {
  const size_t b0 = span * kDecSpan;
  const long long w0 = (long long)b0 - kWinPad;
  for (int c = threadIdx.x; c < kWin / 16 + 1; c += kDecBlock) win4[c] = text.chunk(w0 + 16LL * c);
  if (threadIdx.x < 64) {
    const uint64_t b = hier_prefix(h, span);
    if (threadIdx.x == 0) sbase = b;
  }
  __syncthreads();
  const uint8_t* win = reinterpret_cast<const uint8_t*>(win4);
  const Window t{text, win, (size_t)w0};
  const int lo = kWinPad + kDecBytes * threadIdx.x;  // this lane's 32 bytes in the window
  const uint4 c0 = win4[lo / 16], c1 = win4[lo / 16 + 1];
  const uint32_t w[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  uint32_t m = colons32(w);  // this lane's colons: one value each
  uint32_t total;
  const uint32_t first = block_excl_scan32(__popc(m), &total);
  for (int k = (int)first; m; m &= m - 1, ++k) {
    const int at = kDecBytes * threadIdx.x + __ffs(m) - 1;
    if (k < kMaxStarts) pos[k] = (uint16_t)at;
    else if (k == kMaxStarts) atomicMin(bad, (unsigned long long)(b0 + at - text.mis));
  }
  __syncthreads();
  const uint32_t nloc = min(total, (uint32_t)kMaxStarts);
  const uint64_t gbase = sbase;
  // phase 1: own checks + value
  const uint32_t* l32 = reinterpret_cast<const uint32_t*>(win4);
  for (uint32_t idx = threadIdx.x; idx < nloc; idx += kDecBlock) {
    // the value's first byte: right after its colon, or after whitespace
    size_t x = b0 + pos[idx] + 1;
    const uint64_t g = gbase + idx;
    const bool first_m = (g & 1) == 0;
    if (g > 0 && g + 1 < nvals && !is_ws(win[x - (size_t)w0])) {
      FastNum fn;
      const uint32_t o = (uint32_t)(x - (size_t)w0);
      if (fast_number(l32, o, first_m, fn)) {
        endp[idx] = (uint16_t)fn.dend;
        // one past the digit before this member's ',' (member 1) or before the '}'
        // that closes the previous pair (member 0)
        comma[idx] = (uint16_t)(first_m ? o - 7 : o - 5);
        keyc[idx] = (uint8_t)fn.key;
        const size_t slot = (g & ~(uint64_t)1) + (fn.key == 'b');
        mag[slot] = make_uint4(fn.v[0], fn.v[1], fn.v[2], fn.v[3]);
        neg[slot] = fn.minus && (fn.v[0] | fn.v[1] | fn.v[2] | fn.v[3]) != 0;
        continue;
      }
    }
    while (x < text.L && is_ws(t[x])) ++x;
    size_t q = 0;
    const uint32_t key = key_before(t, x, &q);
    bool ok = key != 0 && g < nvals && q > 0;
    size_t cm = 0;
    if (ok && first_m) {  // '{' ws then '[' ws BOF (first pair) or '}' ws ',' ws after a digit
      ok = t[q - 1] == '{';
      const size_t r = skip_ws_back(t, q - 1);
      if (g == 0) {
        ok = ok && r > 0 && t[r - 1] == '[' && skip_ws_back(t, r - 1) == 0;
      } else {
        ok = ok && r > 0 && t[r - 1] == ',';
        const size_t r2 = ok ? skip_ws_back(t, r - 1) : 0;
        ok = ok && r2 > 0 && t[r2 - 1] == '}';
        const size_t r3 = ok ? skip_ws_back(t, r2 - 1) : 0;
        ok = ok && r3 > 0 && is_digit(t[r3 - 1]);
        cm = r3;
      }
    } else if (ok) {  // ',' ws before the key
      ok = t[q - 1] == ',';
      cm = skip_ws_back(t, q - 1);
    }
    // the number: optional '-', 1..39 digits without a leading zero, value < 2^128
    size_t p = x;
    const bool minus = t[p] == '-';
    p += minus;
    const bool lead0 = t[p] == '0';
    uint32_t v[4] = {0, 0, 0, 0};
    int nd = 0;
    bool ovf = false;
    for (;;) {
      const uint32_t b = t.word(p);
      const uint32_t nondig = ~swar_digit(b) & 0x80808080u;
      const int k = nondig ? (__builtin_ctz(nondig) >> 3) : 4;
      if (k > 0) {  // the k leading digits as a k-digit value
        uint32_t d = (b - 0x30303030u) << (8 * (4 - k));
        d = d * 10u + (d >> 8);
        fold(v, k == 4 ? 10000u : k == 3 ? 1000u : k == 2 ? 100u : 10u, (d & 0xFFu) * 100u + ((d >> 16) & 0xFFu), ovf);
        nd += k;
        p += k;
      }
      if (k < 4 || nd > 39) break;
    }
    ok = ok && nd > 0 && nd <= 39 && !ovf && !(lead0 && nd > 1);
    const size_t dend = p;
    if (ok) {  // the token ends the member: ws then ',' (member 0) or '}' (member 1)
      while (p < text.L && is_ws(t[p])) ++p;
      ok = p < text.L && t[p] == (first_m ? ',' : '}');
      if (ok && g + 1 == nvals) {  // the last pair closes the array: '}' ws ']' ws EOF
        ++p;
        while (p < text.L && is_ws(t[p])) ++p;
        ok = p < text.L && t[p] == ']';
        ++p;
        while (ok && p < text.L && is_ws(t[p])) ++p;
        ok = ok && p == text.L;
      }
    }
    endp[idx] = (uint16_t)(dend - (size_t)w0);
    comma[idx] = (uint16_t)(cm - (size_t)w0);
    keyc[idx] = ok ? (uint8_t)key : 0;
    if (!ok) {
      atomicMin(bad, (unsigned long long)(x - text.mis));
      continue;
    }
    const size_t slot = (g & ~(uint64_t)1) + (key == 'b');
    mag[slot] = make_uint4(v[0], v[1], v[2], v[3]);
    neg[slot] = minus && (v[0] | v[1] | v[2] | v[3]) != 0;
  }
  __syncthreads();
  // phase 2: every value follows the one before it: member 1's ',' and
  // member 0's '}' sit right after the previous value's digits (ws aside),
  // and member 1's key is not its member 0's
  for (uint32_t idx = threadIdx.x; idx < nloc; idx += kDecBlock) {
    const uint64_t g = gbase + idx;
    const uint32_t key = keyc[idx];
    if (g == 0 || key == 0) continue;
    const bool m1 = (g & 1) != 0;
    bool ok;
    if (idx > 0) {
      ok = comma[idx] == endp[idx - 1] && keyc[idx - 1] != 0 && (!m1 || keyc[idx - 1] != key);
    } else {  // the previous value sits in the previous span: walk back over its digits
      size_t x = b0 + pos[idx] + 1;
      while (x < text.L && is_ws(t[x])) ++x;
      size_t q = 0;
      key_before(t, x, &q);
      size_t r = skip_ws_back(t, q - 1);  // member 1: the ','; member 0: the '{'
      if (!m1) {  // '{' ws ',' ws '}' ws <digit> (checked in phase 1)
        r = skip_ws_back(t, r - 1);
        r = skip_ws_back(t, r - 1);
      }
      while (r > 0 && is_digit(t[r - 1])) --r;
      if (r > 0 && t[r - 1] == '-') --r;
      size_t q0 = 0;
      const uint32_t k0 = key_before(t, r, &q0);
      ok = k0 != 0 && (!m1 || (k0 != key && q0 > 0 && t[q0 - 1] == '{'));
    }
    if (!ok) {
      size_t x = b0 + pos[idx] + 1;
      while (x < text.L && is_ws(t[x])) ++x;
      atomicMin(bad, (unsigned long long)(x - text.mis));
    }
  }
  __syncthreads();  // the next span reuses the LDS arrays
  }
}

// THE decode pass, one read of the text (k_xdec_one; one workgroup per
// 8 KiB span).  Stage the span + kWinPad either side in LDS, list its colons
// (one per value: "k":NUM), PUBLISH the colon count -- one agent-scope atomic
// add each to l0[span], l1[span >> 6] and l2[span >> 12], count + kOne, onto
// words zeroed by the launch before -- then parse one value per lane into
// registers against its compact-layout SEGMENT (fast_segment), and only then
// learn the span's first value index from the published counts of every span
// before it (published_prefix: ONE wave, three polls per lane, retried
// until every needed word carries all its contributors) and store.  A span
// waits only for spans dispatched before it to reach their publication, which
// each does right after its colon listing, so no chain of prefixes forms (a
// decoupled look-back that waited for its predecessor's INCLUSIVE prefix moved
// its frontier 64 spans per memory round trip across the eight XCDs and
// measured 1.5-2.8x slower in round 2).  This replaced a separate count pass
// that read the whole text once more (112 us of 405 for 752 MB).  Any value
// outside the compact layout (whitespace, a malformed byte, value 0 or the last
// value not in the plain form, more colons than a span can hold), or a wait
// that gives up (kLookPolls), raises a flag and k_xdec_slow parses the whole
// text with the general grammar and reports errors; Jackson's compact output
// never takes it.
constexpr int kLookPolls = 1 << 14;  // ~1 us each: a bound, never reached with in-order dispatch

// A poll reads the word by an atomic add of 0 (done at the memory side, like
// the publishing adds), not by an sc1 load: the hand-off table of
// MI355X_MICROARCH.md lists 8-byte sc1 loads as unmeasured for this pattern.
__device__ __forceinline__ uint64_t ld_sc1(uint64_t* p) {
  return __hip_atomic_fetch_add(p, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// whole wave: the exclusive value prefix of span s once every span before it
// has published its count; false if that takes more than kLookPolls polls
__device__ __forceinline__ bool published_prefix(const Hier& h, size_t s, uint64_t* prefix) {
  const size_t lane = __lane_id();
  const size_t b2 = s >> 12, g0 = b2 << 6, g1 = s >> 6, s0 = g1 << 6;
  for (int poll = 0; poll < kLookPolls; ++poll) {
    uint64_t v = 0;
    bool ready = true;
    for (size_t k = lane; k < b2; k += 64) {  // whole 4096-span blocks before s's
      const uint64_t x = ld_sc1(&h.l2[k]);
      v += x & kCountMask;
      ready &= (x >> 40) == 4096;
    }
    if (g0 + lane < g1) {  // whole 64-span groups before s's, in its block
      const uint64_t x = ld_sc1(&h.l1[g0 + lane]);
      v += x & kCountMask;
      ready &= (x >> 40) == 64;
    }
    if (s0 + lane < s) {  // spans before s in its group
      const uint64_t x = ld_sc1(&h.l0[s0 + lane]);
      v += x & kCountMask;
      ready &= (x >> 40) == 1;
    }
    if (__ballot(!ready) == 0) {
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
      *prefix = v;
      return true;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  return false;
}

__global__ __launch_bounds__(kDecBlock) void k_xdec_one(Text text, Hier h, size_t nb, size_t nvals,
                                                    uint4* mag, uint8_t* neg, unsigned int* flags) {
  __shared__ uint4 win4[kWin / 16 + 1];
  __shared__ uint16_t pos[kMaxStarts];  // colon, relative to b0
  __shared__ uint64_t sbase;
  __shared__ int sok;
  const size_t span = blockIdx.x;
  const size_t b0 = span * kDecSpan;
  const long long w0 = (long long)b0 - kWinPad;
  if (w0 >= (long long)text.mis && w0 + 16LL * (kWin / 16 + 1) <= (long long)text.L) {
    // a window wholly inside the text: its 545 chunks as three plain 16-byte
    // loads per lane, all issued before any is written (the third clamped:
    // lanes past the window reload its last chunk and skip the write)
    static_assert(kWin / 16 + 1 <= 3 * kDecBlock && kWin / 16 + 1 > 2 * kDecBlock, "three chunks per lane");
    const u32x4* a = reinterpret_cast<const u32x4*>(text.al + w0);
    const int c2 = min((int)threadIdx.x + 2 * kDecBlock, kWin / 16);
    const u32x4 v0 = __builtin_nontemporal_load(a + threadIdx.x),
                v1 = __builtin_nontemporal_load(a + threadIdx.x + kDecBlock), v2 = __builtin_nontemporal_load(a + c2);
    win4[threadIdx.x] = make_uint4(v0.x, v0.y, v0.z, v0.w);
    win4[threadIdx.x + kDecBlock] = make_uint4(v1.x, v1.y, v1.z, v1.w);
    if ((int)threadIdx.x + 2 * kDecBlock <= kWin / 16) win4[c2] = make_uint4(v2.x, v2.y, v2.z, v2.w);
  } else {
    for (int c = threadIdx.x; c < kWin / 16 + 1; c += kDecBlock) win4[c] = text.chunk(w0 + 16LL * c);
  }
  __syncthreads();
  const int lo = kWinPad + kDecBytes * threadIdx.x;
  const uint4 c0 = win4[lo / 16], c1 = win4[lo / 16 + 1];
  const uint32_t w[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  uint32_t m = colons32(w);
  uint32_t total;
  const uint32_t first = block_excl_scan32(__popc(m), &total);
  if (threadIdx.x == 0) {  // publish this span's count (colons: one per value)
    atomicAdd((unsigned long long*)&h.l0[span], (unsigned long long)(total + kOne));
    atomicAdd((unsigned long long*)&h.l1[span >> 6], (unsigned long long)(total + kOne));
    atomicAdd((unsigned long long*)&h.l2[span >> 12], (unsigned long long)(total + kOne));
  }
  for (int k = (int)first; m && k < kMaxStarts; m &= m - 1, ++k)
    pos[k] = (uint16_t)(kDecBytes * threadIdx.x + __ffs(m) - 1);
  __syncthreads();
  bool fail = total > (uint32_t)kMaxStarts;
  const uint32_t nloc = min(total, (uint32_t)kMaxStarts);
  const uint32_t* l32 = reinterpret_cast<const uint32_t*>(win4);
  const size_t len = text.L - text.mis;
  // the span's first value index: wave 0 learns it after its own values are
  // parsed (the wait overlaps the other waves' parse and the CU's other
  // workgroups); a span with more values than lanes learns it first
  auto learn_base = [&]() {
    if (threadIdx.x < 64) {
      uint64_t b = 0;
      const bool ok = published_prefix(h, span, &b);
      if (threadIdx.x == 0) {
        sbase = b;
        sok = ok;
      }
    }
    __syncthreads();
  };
  if (nloc <= (uint32_t)kDecBlock) {
    const uint32_t idx = threadIdx.x;
    FastNum fn;
    uint32_t f = 0;
    if (idx < nloc) {
      const uint32_t at = pos[idx];
      f = fast_value(l32, at + 1 + kWinPad, b0 + at + 1 - text.mis, len, fn);
    }
    learn_base();
    if (!sok) {
      fail = true;
    } else if (idx < nloc) {
      const uint64_t g = sbase + idx;
      if (segment_holds(f, g, nvals)) {
        const size_t slot = (g & ~(uint64_t)1) + (fn.key == 'b');
        xst16(mag + slot, make_uint4(fn.v[0], fn.v[1], fn.v[2], fn.v[3]));
        neg[slot] = fn.minus && (fn.v[0] | fn.v[1] | fn.v[2] | fn.v[3]) != 0;
      } else {
        fail = true;
      }
    }
  } else {
    learn_base();
    if (!sok) fail = true;
    for (uint32_t idx = threadIdx.x; idx < nloc && sok; idx += kDecBlock) {
      const uint32_t at = pos[idx];
      const uint64_t g = sbase + idx;
      FastNum fn;
      const uint32_t f = fast_value(l32, at + 1 + kWinPad, b0 + at + 1 - text.mis, len, fn);
      if (segment_holds(f, g, nvals)) {
        const size_t slot = (g & ~(uint64_t)1) + (fn.key == 'b');
        xst16(mag + slot, make_uint4(fn.v[0], fn.v[1], fn.v[2], fn.v[3]));
        neg[slot] = fn.minus && (fn.v[0] | fn.v[1] | fn.v[2] | fn.v[3]) != 0;
      } else {
        fail = true;
      }
    }
  }
  if (__ballot(fail) != 0 && __lane_id() == 0) atomicOr(&flags[sok ? 1 : 0], 1u);
}

// The array holds exactly nvals numbers and is bracketed; an empty array
// holds nothing but whitespace (with numbers, the lanes above check the rest).
__global__ __launch_bounds__(256) void k_xdec_check(Text t, Hier h, size_t nb,
                                                    size_t nvals, unsigned long long* bad) {
  __shared__ size_t az[2];
  __shared__ uint64_t stotal;
  if (threadIdx.x < 64) {  // every span's count
    const uint64_t v = hier_total(h, nb);
    if (threadIdx.x == 0) stotal = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    size_t a = t.mis;
    while (a < t.L && is_ws(t[a])) ++a;
    size_t z = t.L;
    while (z > t.mis && is_ws(t[z - 1])) --z;
    if (a >= t.L || t[a] != '[') atomicMin(bad, (unsigned long long)(a - t.mis));
    else if (z <= a + 1 || t[z - 1] != ']') atomicMin(bad, (unsigned long long)(z > t.mis ? z - 1 - t.mis : 0));
    else if (stotal != nvals) atomicMin(bad, (unsigned long long)(t.L - t.mis));
    az[0] = a + 1;
    az[1] = z > t.mis ? z - 1 : t.mis;
  }
  __syncthreads();
  if (nvals == 0)
    for (size_t i = az[0] + threadIdx.x; i < az[1]; i += blockDim.x)
      if (!is_ws(t[i])) atomicMin(bad, (unsigned long long)(i - t.mis));
}

unsigned blocks_of(size_t n, size_t per) { return (unsigned)((n + per - 1) / per); }

}  // namespace

size_t xenc_scratch_bytes(size_t npairs) {  // block lengths, the l1 / l2 sums, one flag word
  const size_t nb = blocks_of(npairs, kXBlock);
  return 8 * (nb + blocks_of(nb, kGroupSpans) + blocks_of(nb, (size_t)kGroupSpans * 64) + 1) + 8;
}

size_t xenc_max_bytes(size_t npairs) { return (size_t)kXEntry * npairs + 2; }

// Three launches: zero the l2 sums, per-block text lengths + the hierarchy
// (k_xenc_bsum), then k_xenc_write, which recomputes its entries' lengths
// while converting, takes its block's offset from the hierarchy and places
// the entries with a workgroup scan -- no per-pair length or offset array goes
// through HBM.
hipError_t launch_exchange_encode(const uint4* mag, const uint8_t* neg, size_t npairs, char* out,
                                  unsigned long long* out_len, void* scratch, const LaunchCfg& c) {
  const size_t nb = npairs ? blocks_of(npairs, kXBlock) : 0;
  uint64_t* p = static_cast<uint64_t*>(scratch);
  const size_t n1 = blocks_of(nb, kGroupSpans), n2 = blocks_of(nb, (size_t)kGroupSpans * 64);
  const Hier h{p, p + nb, p + nb + n1};
  LaunchCfg c0 = c, cm = c, c1 = c;
  c0.ev_stop = nullptr;
  cm.ev_start = cm.ev_stop = nullptr;
  c1.ev_start = nullptr;
  AMPH_LAUNCH(k_hier_zero, dim3(1), dim3(256), c0, h.l2, n2 ? n2 : (size_t)1, (unsigned int*)nullptr, 0);
  if (nb > 0)
    AMPH_LAUNCH(k_xenc_bsum, dim3((unsigned)n1), dim3(4 * kXBlock), cm, mag, neg, npairs, nb, h);
  AMPH_LAUNCH(k_xenc_write, dim3(nb ? (unsigned)nb : 1u), dim3(kXBlock), c1, mag, neg, npairs, h, nb, out,
              out_len);
  return hipGetLastError();
}

namespace {
struct XdecScratch {
  Hier h;
  unsigned int* flags;
};
XdecScratch xdec_layout(void* scratch, size_t nb) {
  uint64_t* p = static_cast<uint64_t*>(scratch);
  const size_t n1 = blocks_of(nb, kGroupSpans), n2 = blocks_of(nb, (size_t)kGroupSpans * 64);
  XdecScratch x;
  x.h = Hier{p, p + nb, p + nb + n1};
  x.flags = reinterpret_cast<unsigned int*>(p + nb + n1 + n2);
  return x;
}
}  // namespace

size_t xdec_scratch_bytes(size_t len) {  // span counts, the l1 / l2 sums, the two flags
  const size_t nb = blocks_of(len + 16, kDecSpan);
  return 8 * (nb + blocks_of(nb, kGroupSpans) + blocks_of(nb, (size_t)kGroupSpans * 64) + 1);
}

// zero the counts and flags, the single pass, the general pass (returns at
// once unless the single pass could not hold), the array check: four launches.
hipError_t launch_exchange_decode(const char* text, size_t len, size_t npairs, uint4* mag,
                                  uint8_t* neg, unsigned long long* bad, void* scratch,
                                  const LaunchCfg& c) {
  const size_t mis = (uintptr_t)text & 15;
  const Text t{reinterpret_cast<const uint8_t*>(text) - mis, mis, mis + len};
  const size_t nb = blocks_of(t.L ? t.L : 1, kDecSpan);
  const XdecScratch x = xdec_layout(scratch, nb);
  const size_t nwords = nb + blocks_of(nb, kGroupSpans) + blocks_of(nb, (size_t)kGroupSpans * 64);
  LaunchCfg c0 = c, cm = c, c1 = c;
  c0.ev_stop = nullptr;
  cm.ev_start = cm.ev_stop = nullptr;
  c1.ev_start = nullptr;
  AMPH_LAUNCH(k_hier_zero, dim3(std::min<unsigned>(blocks_of(nwords, 256), 256u)), dim3(256), c0, x.h.l0, nwords,
              x.flags, 2);
  AMPH_LAUNCH(k_xdec_one, dim3((unsigned)nb), dim3(kDecBlock), cm, t, x.h, nb, 2 * npairs, mag, neg, x.flags);
  AMPH_LAUNCH(k_xdec_slow, dim3((unsigned)std::min<size_t>(nb, kSlowGrid)), dim3(kDecBlock), cm, t, x.h, nb,
              2 * npairs, mag, neg, bad, (const unsigned int*)x.flags);
  AMPH_LAUNCH(k_xdec_check, dim3(1), dim3(256), c1, t, x.h, nb, 2 * npairs, bad);
  return hipGetLastError();
}

}  // namespace amph

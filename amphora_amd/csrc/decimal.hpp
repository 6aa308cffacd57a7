// Decimal digit counts of 128-bit magnitudes, shared by the exchange codec
// (exchange.hip: the encoder's entry lengths) and K_ODO_PRE (kernels.hip: the
// same lengths computed where the diffs are made, for the party session).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace amph {
namespace {

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



// Length of one FactorPair entry of the exchange text as Jackson writes it:
// {"a":D,"b":E} plus the ',' that follows every entry but the last
// (BigInteger has no negative zero).
__device__ __forceinline__ uint32_t xentry_len(const uint4& d, bool dneg, const uint4& e, bool eneg, bool last) {
  return 11 + ndigits128(d) + (dneg && !is_zero(d)) + ndigits128(e) + (eneg && !is_zero(e)) + (last ? 0 : 1);
}

}  // namespace
}  // namespace amph

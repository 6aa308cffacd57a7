// Base64 group coding shared by the wire codec (codec.hip) and the fused
// wire-format kernels (wire.hip): Jackson's Base64Variants.MIME_NO_LINEFEEDS
// alphabet, 4 characters <-> 3 bytes, branch-free SWAR / v_perm table lookups.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace amph {

// Four 6-bit values (one per byte, first char lowest) -> their 4 chars.
// idx = (v >= 26) + (v >= 52) + (v >= 62) + (v >= 63) picks the offset
// to ASCII from a v_perm byte table ('A', 'a' - 26, '0' - 52, '+' - 62,
// '/' - 63).  The offsets are kept mod 128 (0x41 0x47 0x7C 0x6D 0x70): v + off
// <= 63 + 0x7C stays below 256, so one plain add has no carry between bytes
// and its low 7 bits are the character (the mod-256 table needed a
// 5-instruction carry-free add).
// The four threshold flags (bit 7 of v + 128 - t) are summed with three
// v_lerp_u8 (per-byte (a + b) / 2, no carry between bytes): the average of
// the pairwise averages is idx * 32.
__device__ __forceinline__ uint32_t enc_chars(uint32_t v) {
  const uint32_t f26 = (v + 0x66666666u) & 0x80808080u, f52 = (v + 0x4C4C4C4Cu) & 0x80808080u;
  const uint32_t f62 = (v + 0x42424242u) & 0x80808080u, f63 = (v + 0x41414141u) & 0x80808080u;
  const uint32_t idx = __builtin_amdgcn_lerp(__builtin_amdgcn_lerp(f26, f52, 0u),
                                             __builtin_amdgcn_lerp(f62, f63, 0u), 0u) >> 5;
  const uint32_t off = __builtin_amdgcn_perm(0x00000070u, 0x6D7C4741u, idx);
  return (v + off) & 0x7F7F7F7Fu;
}

// 24-bit group (first char in the top 6 bits) -> its 4 chars, packed
// little-endian.
__device__ __forceinline__ uint32_t enc4(uint32_t g) {
  return enc_chars(((g >> 18) & 0x3Fu) | ((g >> 4) & 0x3F00u) | ((g << 10) & 0x3F0000u) |
                   ((g << 24) & 0x3F000000u));
}

// Bytes [3Q, 3Q + 3) of the little-endian byte stream w[0..N) (zero past its
// end) -> their 4 chars, for callers that hold the bytes as dwords.  The four
// 6-bit values come out of two v_perm (the group's bytes b0 b1 b2 arranged as
// 16-bit lanes b0 | b1:b2 and b0:b1 | b2, zero bytes by selector 0x0C) and two
// packed 16-bit shifts with a shift count per lane (>> {2, 6}, << {4, 8}):
// 6 instructions where gathering the bytes into a 24-bit group and
// spreading it took ~12.
typedef unsigned short b64_u16x2 __attribute__((ext_vector_type(2)));
template <int Q, int N>
__device__ __forceinline__ uint32_t enc_group_w(const uint32_t (&w)[N]) {
  constexpr int B = 3 * Q, i = B / 4;
  constexpr uint32_t b0 = B % 4, b1 = b0 + 1, b2 = b0 + 2;  // byte positions in (hi : lo)
  static_assert(i < N, "group past the stream");
  uint32_t hi = 0u;
  if constexpr (i + 1 < N) hi = w[i + 1];
  const uint32_t lo = w[i];
  const uint32_t s1 = __builtin_amdgcn_perm(hi, lo, b0 | 0x0C00u | (b2 << 16) | (b1 << 24));  // b0 0 | b2 b1
  const uint32_t s2 = __builtin_amdgcn_perm(hi, lo, b1 | (b0 << 8) | (b2 << 16) | 0x0C000000u);  // b1 b0 | b2 0
  const b64_u16x2 a = __builtin_bit_cast(b64_u16x2, s1) >> (b64_u16x2){2, 6};
  const b64_u16x2 c = __builtin_bit_cast(b64_u16x2, s2) << (b64_u16x2){4, 8};
  return enc_chars((__builtin_bit_cast(uint32_t, a) & 0x003F003Fu) | (__builtin_bit_cast(uint32_t, c) & 0x3F003F00u));
}

// A 12-byte unit (3 dwords) -> its 16 chars (4 dwords)
__device__ __forceinline__ void enc_unit12(const uint32_t (&w)[3], uint32_t (&g)[4]) {
  g[0] = enc_group_w<0>(w);
  g[1] = enc_group_w<1>(w);
  g[2] = enc_group_w<2>(w);
  g[3] = enc_group_w<3>(w);
}

// 3 bytes (big-endian group) -> 4 chars packed little-endian in a uint32
__device__ __forceinline__ uint32_t enc_group(uint32_t b0, uint32_t b1, uint32_t b2) {
  return enc4((b0 << 16) | (b1 << 8) | b2);
}


// 4 base64 chars (little-endian bytes, first char lowest) -> their four
// 6-bit values (one per byte, same order) and a validity mask (bit 7 of byte
// j set iff char j is in the alphabet, exact per character whatever its
// neighbours hold: the class is masked to 4 bits before the +0x7F, and the
// value add is carry-free).  Table lookups with v_perm_b32 (8-entry byte
// tables): class = HI[c >> 4] & LO[c & 15], valid iff nonzero, with the bits
//   1 '+' '/' (high nibble 2, low B / F)   2 digits (high 3, low 0-9)
//   4 'A'-'O' 'a'-'o' (high 4 / 6, low 1-15)   8 'P'-'Z' 'p'-'z' (high 5 / 7, low 0-A)
// and '/' marked by 3 in bits 4-5 (HI[2] = 0x31, LO[15] = 0x35), so the -3 it
// needs after the ROLL add is (cls >> 4) & 3.  The exact locator of the fast
// paths' rare bad units (dec_unit16); the fast paths use dec4_values6.
__device__ __forceinline__ uint32_t dec4_values(uint32_t w, uint32_t& valid) {
  const uint32_t lo = w & 0x0F0F0F0Fu, l7 = lo & 0x07070707u, h7 = (w >> 4) & 0x07070707u;
  const uint32_t la = __builtin_amdgcn_perm(0x0E0E0E0Eu, 0x0E0E0E0Au, l7);
  const uint32_t lb = __builtin_amdgcn_perm(0x35040404u, 0x050C0E0Eu, l7);
  const uint32_t cl = __builtin_amdgcn_perm(lb, la, 0x03020100u | ((lo & 0x08080808u) >> 1));
  const uint32_t cls = __builtin_amdgcn_perm(0x08040804u, 0x02310000u, h7) & cl;
  valid = ((cls & 0x0F0F0F0Fu) + 0x7F7F7F7Fu) & ~w;  // bit 7: in the alphabet (and ASCII)
  const uint32_t roll = __builtin_amdgcn_perm(0xB9B9BFBFu, 0x04130000u, h7);
  const uint32_t v = ((w & 0x7F7F7F7Fu) + (roll & 0x7F7F7F7Fu)) ^ ((w ^ roll) & 0x80808080u);
  return v - ((cls >> 4) & 0x03030303u);  // no borrow: '/' + ROLL = 66 per byte
}

// The fused wire kernels' form of dec4_values (they are integer-VALU-bound:
// DESIGN.md §4a'), 19 instructions per 4 characters instead of ~25:
// * the value path keeps only the low 6 bits of each byte: c + ROLL6[.]
//   (the roll table mod 64) stays below 256 for an ASCII c, so one plain
//   32-bit add has no carry between bytes, and its low 6 bits are the value;
//   one AND clears bits 6-7 for the packing dot products;
// * '/' needs its own roll (16; '+' 19): the class tables give '/' -- and only
//   '/' -- bit 1 of its class byte (HI[2] and LO[15] are the only entries
//   holding it), and the roll lookup's selector is h ^ (class & 2), which
//   sends '/' to slot 0 (h = 0 is a control character, so slot 0 is free);
// * validity is class + 0x7F per byte (class bytes are <= 0x1C: no carry,
//   bit 7 set iff the class is nonzero), ANDed with ~c into the running mask.
// Classes: bit 0 '+' '/' (h 2), bit 1 '/', bit 2 h 4 / 6, bit 3 h 5 / 7,
// bit 4 digits (h 3); LO[l] holds the groups whose row allows nibble l.
// Non-ASCII or invalid characters may corrupt their neighbours' values (a
// carry out of the byte) -- the unit is reported invalid then.
//
// DecTabs: the low dwords of its four v_perm tables.  A v_perm takes one SGPR or
// literal operand, so the second table dword has to be in a VGPR; given as
// compile-time constants the compiler re-materialises them with a v_mov per
// unit, dec_tabs_vgpr() makes them opaque values held in four VGPRs instead.
struct DecTabs {
  uint32_t la, lb, hi, roll;
};
#define AMPH_DEC_TABS {0x1C1C1C18u, 0x050C1C1Cu, 0x10030000u, 0x04130010u}
__device__ __forceinline__ DecTabs dec_tabs_vgpr() {
  DecTabs t AMPH_DEC_TABS;
  asm volatile("" : "+v"(t.la), "+v"(t.lb), "+v"(t.hi), "+v"(t.roll));
  return t;
}

__device__ __forceinline__ uint32_t dec4_values6(uint32_t w, uint32_t& okacc, const DecTabs& t) {
  const uint32_t l7 = w & 0x07070707u, h7 = (w >> 4) & 0x07070707u;
  const uint32_t la = __builtin_amdgcn_perm(0x1C1C1C1Cu, t.la, l7);  // LO[0..7]
  const uint32_t lb = __builtin_amdgcn_perm(0x07040404u, t.lb, l7);  // LO[8..15]
  const uint32_t cl = __builtin_amdgcn_perm(lb, la, ((w >> 1) & 0x04040404u) | 0x03020100u);
  const uint32_t cls = __builtin_amdgcn_perm(0x08040804u, t.hi, h7) & cl;
  okacc &= (cls + 0x7F7F7F7Fu) & ~w;
  const uint32_t roll6 = __builtin_amdgcn_perm(0x39393F3Fu, t.roll, h7 ^ (cls & 0x02020202u));
  return (w + roll6) & 0x3F3F3F3Fu;
}

// One full 16-character unit (4 groups, no padding) -> its 12 bytes as 3
// little-endian dwords.  Each group's 24 bits come from two v_dot4_u32_u8
// (64 v0 + v1, 64 v2 + v3) and one shift-or, the 12 bytes from three
// v_perm_b32 straight out of the four groups.  The unit's validity is ANDed
// into ok (bit 7 of every byte stays set iff every character seen so far is
// in the alphabet), so a caller tests once per unit (or per many units) and
// locates a bad character only then.
__device__ __forceinline__ void dec_unit16_ok(const uint4 v, uint32_t (&o)[3], uint32_t& ok,
                                              const DecTabs& t = DecTabs AMPH_DEC_TABS) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t g[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t x = dec4_values6(w[q], ok, t);
    g[q] = (__builtin_amdgcn_udot4(x, 0x00000140u, 0u, false) << 12) |
           __builtin_amdgcn_udot4(x, 0x01400000u, 0u, false);
  }
  // bytes in text order: g0[23:16] g0[15:8] g0[7:0] g1[23:16] | g1[15:8] ...
  o[0] = __builtin_amdgcn_perm(g[1], g[0], 0x06000102u);
  o[1] = __builtin_amdgcn_perm(g[2], g[1], 0x05060001u);
  o[2] = __builtin_amdgcn_perm(g[3], g[2], 0x04050600u);
}

// dec_unit16_ok for one unit; returns the offset of the first invalid
// character in it, or 0xFFFFFFFF (located with the exact dec4_values, whose
// validity mask is per character whatever the neighbours hold).
__device__ __forceinline__ uint32_t dec_unit16(const uint4 v, uint32_t (&o)[3]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t ok = 0x80808080u;
  dec_unit16_ok(v, o, ok);
  if (ok == 0x80808080u) return 0xFFFFFFFFu;
  // a bad character somewhere (rare): find the first, group by group
  uint32_t firstbad = 0xFFFFFFFFu;
#pragma unroll
  for (int q = 3; q >= 0; --q) {
    uint32_t val;
    (void)dec4_values(w[q], val);
    const uint32_t inv = ~val & 0x80808080u;
    if (inv) firstbad = 4 * q + (__builtin_ctz(inv) >> 3);
  }
  return firstbad;
}

// A 16-byte word -> its 24-character record (5 full groups, then 1 byte and
// "=="), as 6 little-endian dwords.
__device__ __forceinline__ void enc_word24(const uint4 v, uint32_t (&g)[6]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  g[0] = enc_group_w<0>(w);
  g[1] = enc_group_w<1>(w);
  g[2] = enc_group_w<2>(w);
  g[3] = enc_group_w<3>(w);
  g[4] = enc_group_w<4>(w);
  g[5] = (enc_group_w<5>(w) & 0xFFFFu) | ((uint32_t)'=' << 16) | ((uint32_t)'=' << 24);
}


// ---- base64 decode through an LDS table (wire kernels' fast path) -------------
// kB64Val[c] = the 6-bit value of base64 character c, 0x80 for any other byte.
struct B64ValTable {
  uint8_t v[256];
  constexpr B64ValTable() : v() {
    for (int c = 0; c < 256; ++c) v[c] = 0x80;
    for (int c = 'A'; c <= 'Z'; ++c) v[c] = (uint8_t)(c - 'A');
    for (int c = 'a'; c <= 'z'; ++c) v[c] = (uint8_t)(c - 'a' + 26);
    for (int c = '0'; c <= '9'; ++c) v[c] = (uint8_t)(c - '0' + 52);
    v['+'] = 62;
    v['/'] = 63;
  }
};
__device__ constexpr B64ValTable kB64Val{};
// One byte per entry: the 256-byte table spans the 64 LDS banks once, so two
// lookups either share a dword (a broadcast) or sit in different banks.  A 4-byte
// stride (one bank per character) measured slower: profiles/r05_wire_lut_ab.txt.
constexpr int kLutBytes = 256;

// Fill the workgroup's LDS copy, any block size (the caller synchronises).
__device__ __forceinline__ void b64_lut_fill(uint8_t* lut) {
  for (uint32_t c = threadIdx.x; c < 256; c += blockDim.x) lut[c] = kB64Val.v[c];
}

// One 16-character unit through the table: 16 lookups, each group's 24 bits
// as (v0 << 18) | (v1 << 12) | (v2 << 6) | v3, the 12 bytes by three
// v_perm_b32 as dec_unit16_ok; the OR of the 16 table values accumulates into
// bad (bit 7 set iff a character outside the alphabet was seen).
__device__ __forceinline__ void dec_unit16_lut(const uint4 v, uint32_t (&o)[3], uint32_t& bad, const uint8_t* lut) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t g[4], acc = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t a = lut[w[q] & 0xFFu], b = lut[(w[q] >> 8) & 0xFFu];
    const uint32_t c = lut[(w[q] >> 16) & 0xFFu], d = lut[w[q] >> 24];
    acc |= a | b | c | d;
    g[q] = (((((a << 6) | b) << 6) | c) << 6) | d;
  }
  bad |= acc;
  o[0] = __builtin_amdgcn_perm(g[1], g[0], 0x06000102u);
  o[1] = __builtin_amdgcn_perm(g[2], g[1], 0x05060001u);
  o[2] = __builtin_amdgcn_perm(g[3], g[2], 0x04050600u);
}

}  // namespace amph

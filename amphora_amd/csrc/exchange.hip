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
// Decimal conversion: 128-bit magnitude <-> five base-10^8 chunks (a
// multiply-accumulate over the limbs with four carry divisions by a constant,
// to_chunks), chunks <-> digits.
#include <hip/hip_ext.h>

#include <algorithm>

#include "kernels.hpp"
#include "decimal.hpp"

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
constexpr int kScanBlock = 1024;  // elements per workgroup of the scan passes
constexpr int kDecBytes = 32;     // text bytes per lane (decode)

__device__ __forceinline__ int ndigits32(uint32_t x) {  // x < 10^9; 0 -> 1 (to_chunks' top chunk: < 10^8)
  int n = 1;
#pragma unroll
  for (uint32_t t = 10; t <= 100000000u; t *= 10) n += x >= t;
  return n;
}

__device__ __forceinline__ uint64_t mad_u64(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }

// 128-bit magnitude -> base-10^8 chunks (little end first); returns the
// decimal digit count (1 for zero).  Multiply-accumulate form: with the limbs
// x_i of x = sum x_i 2^(32 i) and the base-10^8 digits of 2^32, 2^64, 2^96
//   2^32 = 42 | 94967296,  2^64 = 1844 | 67440737 | 09551616,
//   2^96 = 79228 | 16251426 | 43375935 | 43950336,
// column k of the base-10^8 product sum is D_k = carry + sum x_i c_(i,k):
// nine v_mad_u64_u32 and four carry divisions by 10^8 in all.  Bounds
// (x_i < 2^32): D_0 < 6.4e17, D_1 < 4.8e17, D_2 < 7.0e16, D_3 < 3.5e14, each
// < 2^64; the last carry (< 3.5e6) is chunk 4 (x < 2^128: <= 7 digits).
// Base 10^8 rather than 10^9: a chunk is exactly two 4-digit halves, so the
// formatter has no separate leading digit per chunk (k_xenc_write -1.5 %,
// profiles/r05_xenc_base1e8_ab.txt; the base-10^9 form: r05_xenc_mac_ab.txt).
__device__ __forceinline__ int to_chunks(const uint4& m, uint32_t (&ch)[5]) {
  constexpr uint64_t kE8 = 100000000ull;
  uint64_t D = mad_u64(m.w, 43950336u, mad_u64(m.z, 9551616u, mad_u64(m.y, 94967296u, m.x)));
  uint64_t q = D / kE8;
  ch[0] = (uint32_t)(D - q * kE8);
  D = mad_u64(m.w, 43375935u, mad_u64(m.z, 67440737u, mad_u64(m.y, 42u, q)));
  q = D / kE8;
  ch[1] = (uint32_t)(D - q * kE8);
  D = mad_u64(m.w, 16251426u, mad_u64(m.z, 1844u, q));
  q = D / kE8;
  ch[2] = (uint32_t)(D - q * kE8);
  D = mad_u64(m.w, 79228u, q);
  q = D / kE8;
  ch[3] = (uint32_t)(D - q * kE8);
  ch[4] = (uint32_t)q;
  int top = 0;
#pragma unroll
  for (int k = 1; k < 5; ++k) top = ch[k] ? k : top;
  return 8 * top + ndigits32(ch[top]);
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

// 8 bytes (lo, then hi) ORed into the zeroed LDS text at p, any alignment,
// as three aligned ds_or_b32: a misaligned 8-byte LDS store costs ~8x an
// aligned dword op (tools/ubench/ubench_lds_align.hip).
__device__ __forceinline__ void or_bytes8(char* p, uint32_t lo, uint32_t hi) {
  const uint32_t mis = (uint32_t)(uintptr_t)p & 3u, sh = 8u * mis;
  uint32_t* d = reinterpret_cast<uint32_t*>(p - mis);  // (pointer arithmetic: stays an LDS pointer)
  const uint64_t x = (uint64_t)lo << sh, y = (uint64_t)hi << sh;
  atomicOr(d, (uint32_t)x);
  atomicOr(d + 1, (uint32_t)(x >> 32) | (uint32_t)y);
  atomicOr(d + 2, (uint32_t)(y >> 32));
}

// nd decimal digits of the chunks ch (to_chunks, base 10^8) at o; returns o + nd.
__device__ __forceinline__ char* put_digits(char* o, const uint32_t (&ch)[5], int nd) {
  // chunk k (little end first) holds text positions [nd - 8 (k + 1), nd - 8 k):
  // one division by 10^4 and two 4-digit SWAR conversions
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int base = nd - 8 * (k + 1);
    if (base + 8 <= 0) break;
    const uint32_t c = ch[k], hi = c / 10000u;
    const uint32_t w0 = ascii4(hi), w1 = ascii4(c - hi * 10000u);
    if (base >= 0) {  // a whole chunk: 8 bytes ORed into the zeroed run
      or_bytes8(o + base, w0, w1);
      continue;
    }
    const uint32_t dig[8] = {w0 & 0xFFu, (w0 >> 8) & 0xFFu, (w0 >> 16) & 0xFFu, w0 >> 24,
                             w1 & 0xFFu, (w1 >> 8) & 0xFFu, (w1 >> 16) & 0xFFu, w1 >> 24};
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (base + j >= 0) o[base + j] = (char)dig[j];
  }
  return o + nd;
}

// ---- device-wide exclusive scan of u64 (three passes) ----------------------------
// Decode count words: colon count in bits 0..39, spans with whitespace (count
// pass) or outside the compact layout (k_xdec_span) from bit 40
constexpr uint64_t kWsBit = 1ull << 40, kCountMask = kWsBit - 1;
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
  const int lane = __lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// Exclusive scan over the workgroup (blockDim multiple of 64, <= 1024);
// returns this lane's exclusive prefix, *total = the workgroup sum.
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t* total) {
  __shared__ uint64_t wsum[17];  // 16 wave offsets + the total
  const int lane = __lane_id(), wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint64_t inc = wave_incl_scan(v);
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  if (wave == 0) {
    const uint64_t s = lane < nw ? wsum[lane] : 0;
    const uint64_t si = wave_incl_scan(s);
    if (lane < nw) wsum[lane] = si - s;  // exclusive wave offsets
    if (lane == nw - 1) wsum[16] = si;
  }
  __syncthreads();
  const uint64_t r = wsum[wave] + inc - v;
  *total = wsum[16];
  __syncthreads();
  return r;
}

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

// The decode's span form: with x the spans' colon counts, map[b] = the span
// holding value kXMapValues * b (b < nmap), written by the lane that scans
// that span.
__device__ __forceinline__ void span_map(uint4* map, size_t nmap, size_t span, uint64_t e, uint64_t c) {
  if (!map) return;
  e &= kCountMask;
  c &= kCountMask;
  for (size_t b = (e + kXMapValues - 1) / kXMapValues; b < nmap && b * kXMapValues < e + c; ++b)
    map[b].x = (uint32_t)span;  // (k_xdec_slow<SpanBases> completes the window)
}

__global__ __launch_bounds__(kScanBlock) void k_scan_reduce(const uint64_t* x, size_t n,
                                                        uint64_t* bsum) {
  const size_t i = (size_t)blockIdx.x * kScanBlock + threadIdx.x;
  uint64_t total;
  block_excl_scan(i < n ? x[i] : 0, &total);
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// One workgroup: in-place exclusive scan of n values, x[n] = total (map as
// k_scan_apply's).
__global__ __launch_bounds__(kScanBlock) void k_scan_single(uint64_t* x, size_t n, uint4* map,
                                                        size_t nmap) {
  uint64_t carry = 0;
  for (size_t base = 0; base < n; base += kScanBlock) {
    const size_t i = base + threadIdx.x;
    const uint64_t v = i < n ? x[i] : 0;
    uint64_t total;
    const uint64_t e = block_excl_scan(v, &total);
    if (i < n) {
      x[i] = carry + e;
      span_map(map, nmap, i, carry + e, v);
    }
    carry += total;
  }
  if (threadIdx.x == 0) x[n] = carry;
}

// x[i] <- exclusive prefix; x[n] <- total (+ the map).  bsum holds the
// per-workgroup sums (k_scan_reduce); wave 0 adds those before its own
// workgroup (and the last workgroup all of them), so no launch scans them in
// between (a single-workgroup scan launch cost ~5 us).
__global__ __launch_bounds__(kScanBlock) void k_scan_apply(uint64_t* x, size_t n,
                                                       const uint64_t* bsum, size_t nb,
                                                       uint4* map, size_t nmap) {
  __shared__ uint64_t sbase[2];
  const size_t i = (size_t)blockIdx.x * kScanBlock + threadIdx.x;
  const uint64_t v = i < n ? x[i] : 0;
  if (threadIdx.x < 64) {
    const bool last = blockIdx.x + 1 == gridDim.x;
    uint64_t b = 0, t = 0;
    for (size_t k = threadIdx.x; k < nb; k += 64) {
      const uint64_t y = bsum[k];
      if (k < blockIdx.x) b += y;
      if (last) t += y;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      b += __shfl_xor(b, o, 64);
      t += __shfl_xor(t, o, 64);
    }
    if (threadIdx.x == 0) {
      sbase[0] = b;
      sbase[1] = t;
    }
  }
  uint64_t total;
  const uint64_t e = block_excl_scan(v, &total);  // (its barriers publish sbase)
  const uint64_t base = sbase[0];
  if (i < n) {
    x[i] = base + e;
    span_map(map, nmap, i, base + e, v);
  }
  if (blockIdx.x + 1 == gridDim.x && threadIdx.x == 0) x[n] = sbase[1];
}

// Encode pass 1: the text length of each workgroup's run of entries
// (bs[g] = sum of the entry lengths of pairs [256 g, 256 g + 256)); digit
// counts from the bit length (ndigits128), not the base-10^8 split.
__global__ __launch_bounds__(4 * kXBlock) void k_xenc_bsum(const uint4* mag, const uint8_t* neg,
                                                       size_t npairs, size_t nb, uint64_t* bs) {
  // one pair per lane, 4 sub-blocks of 256 pairs per 1024-lane workgroup:
  // wave sums by shuffles, then 4 lanes add their sub-block's 4 wave sums.
  // The powers of ten ndigits128 compares with sit in LDS (a global table
  // made its lookup a second dependent memory round trip per number).
  __shared__ uint32_t ws[16];
  __shared__ uint4 p10[39];
  if (threadIdx.x < 39)
    p10[threadIdx.x] = make_uint4(kPow10[threadIdx.x][0], kPow10[threadIdx.x][1], kPow10[threadIdx.x][2],
                                  kPow10[threadIdx.x][3]);
  const size_t k = (size_t)blockIdx.x * (4 * kXBlock) + threadIdx.x;
  uint4 d = make_uint4(0, 0, 0, 0), e = d;
  uint32_t ng = 0;
  if (k < npairs) {
    d = mag[2 * k];
    e = mag[2 * k + 1];
    ng = reinterpret_cast<const uint16_t*>(neg)[k];
  }
  __syncthreads();
  uint32_t len = 0;
  if (k < npairs) {  // {"a":A,"b":B} (+ ',' unless last)
    auto nd = [&](const uint4& m) {
      const int bits = m.w ? 128 - __clz(m.w) : m.z ? 96 - __clz(m.z) : m.y ? 64 - __clz(m.y) : 32 - __clz(m.x);
      const int t = (bits * 1233) >> 12;
      const uint4 p = p10[t];
      const uint32_t pa[4] = {p.x, p.y, p.z, p.w};
      const int n = t + (ge128(m, pa) ? 1 : 0);
      return n ? n : 1;
    };
    len = 11 + nd(d) + ((ng & 0xFFu) != 0 && !is_zero(d)) + nd(e) + ((ng >> 8) != 0 && !is_zero(e)) +
          (k + 1 < npairs);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) len += __shfl_xor(len, o, 64);
  if (__lane_id() == 0) ws[threadIdx.x >> 6] = len;
  __syncthreads();
  const size_t sub = 4 * (size_t)blockIdx.x + threadIdx.x;
  if (threadIdx.x < 4 && sub < nb)
    bs[sub] = (uint64_t)ws[4 * threadIdx.x] + ws[4 * threadIdx.x + 1] + ws[4 * threadIdx.x + 2] +
              ws[4 * threadIdx.x + 3];
}

// Encode pass 3 (after the scan of bs): each lane converts its two numbers,
// the workgroup scans the entry lengths to place them, and the entries are
// formatted into LDS and stored as one contiguous run.  The run sits in LDS
// at the same offset mod 16 as its destination (sh), so every 16-byte unit
// wholly inside it moves as one aligned ds_read_b128 + global 16-byte store;
// the up to 15 bytes at either end go out singly.
// bs[bstride * b] = the offset of workgroup b's run, bs[nblocks] the total.
__global__ __launch_bounds__(kXBlock) void k_xenc_write(const uint4* mag, const uint8_t* neg,
                                                    size_t npairs, const uint64_t* bs,
                                                    size_t nblocks, char* out,
                                                    unsigned long long* out_len, int bstride) {
  __shared__ uint4 bufv[(kXBlock * kXEntry + 8) / 16 + 2];
  char* buf = reinterpret_cast<char*>(bufv);
  const size_t k = (size_t)blockIdx.x * kXBlock + threadIdx.x;
  uint32_t cd[5], ce[5];
  int nd = 0, ne = 0;
  bool sd = false, se = false;
  uint32_t len = 0, total;  // <= 92 per entry, <= 23 552 per workgroup
  // the run's digits are ORed in (or_bytes8): zero the buffer (block_excl_scan32's barriers order it)
  for (int q = threadIdx.x; q < (int)(sizeof(bufv) / 16); q += kXBlock) bufv[q] = make_uint4(0, 0, 0, 0);
  if (k < npairs) {
    const uint4 d = mag[2 * k], e = mag[2 * k + 1];
    const uint32_t ng = reinterpret_cast<const uint16_t*>(neg)[k];  // (loaded beside the magnitudes)
    __builtin_amdgcn_sched_barrier(0);
    nd = to_chunks(d, cd);
    ne = to_chunks(e, ce);
    sd = (ng & 0xFFu) != 0 && !is_zero(d);  // BigInteger has no negative zero
    se = (ng >> 8) != 0 && !is_zero(e);
    len = 11 + nd + sd + ne + se + (k + 1 < npairs);
  }
  const uint32_t loc = block_excl_scan32(len, &total);
  const uint64_t base = bs[(size_t)bstride * blockIdx.x];
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
    out[1 + bs[nblocks]] = ']';
    if (out_len) *out_len = bs[nblocks] + 2;
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

// Pass 1: colons (= numbers) per 8 KiB span, ONE WAVE PER SPAN: 64 lanes x
// eight 16-B loads in flight, lane-interleaved so that every wave
// instruction reads 1 KiB contiguous (nontemporal: the text is read once here
// and once by the parse), a wave reduction, no LDS or barrier; four spans per
// 256-lane workgroup.  96 us per 640 MB text where 128 lanes x 64
// lane-contiguous bytes per span took 162 (tools/ubench/ubench_xcount.hip).
constexpr int kCntWaves = 4;
// Numbers (colons) per 8 KiB span at most: {"a":1,"b":2}, is 14 bytes per 2
constexpr int kMaxStarts = 1280;
constexpr int kListHead = 256;  // colon-list entries per span in the list's dense head

// A 16-byte chunk's colons, one bit per byte (as colons32)
__device__ __forceinline__ uint32_t colons16(const uint4& c) {
  const uint32_t h0 = __builtin_amdgcn_udot4(swar_colon(c.y), 0x80402010u, 0u, false);
  const uint32_t a0 = __builtin_amdgcn_udot4(swar_colon(c.x), 0x08040201u, h0, false);
  const uint32_t h1 = __builtin_amdgcn_udot4(swar_colon(c.w), 0x80402010u, 0u, false);
  const uint32_t a1 = __builtin_amdgcn_udot4(swar_colon(c.z), 0x08040201u, h1, false);
  return (a0 >> 7) | ((a1 >> 7) << 8);
}

__device__ __forceinline__ uint32_t swar_below21(uint32_t w) {  // nonzero iff some byte < 0x21
  return (w - 0x21212121u) & ~w & 0x80808080u;
}

__global__ __launch_bounds__(64 * kCntWaves) void k_xdec_count(Text t, uint64_t* bsum, size_t nb,
                                                             unsigned int* slow, uint16_t* posg) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *slow = 0;  // k_xdec_fast's flag
  const size_t span = (size_t)blockIdx.x * kCntWaves + (threadIdx.x >> 6);
  if (span >= nb) return;
  const uint32_t lane = threadIdx.x & 63;
  const size_t base = span * kDecSpan + (size_t)lane * 16;
  uint4 c[8];
  if (span * kDecSpan >= t.mis && (span + 1) * kDecSpan <= t.L) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(t.al + base + 1024 * k));
      c[k] = make_uint4(v.x, v.y, v.z, v.w);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = t.chunk((long long)(base + 1024 * k));
  }
  uint32_t msk[8], low = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    msk[k] = colons16(c[k]);
    low |= swar_below21(c[k].x) | swar_below21(c[k].y) | swar_below21(c[k].z) | swar_below21(c[k].w);
  }
  // The span's colon list (k_xdec_fast's values, in text order: slab k =
  // bytes 1024k.., lane by lane): per-slab lane prefixes by DPP scans of two
  // slabs' counts per word (<= 1024 each), slab bases by running the totals;
  // listed in LDS, then stored as 16-byte chunks.  At 8 Mi pairs the list
  // (~34 MB) costs this pass ~16 us and saves k_xdec_fast ~34 (its colon
  // scan, workgroup scan and barrier), r05_xdec_colon_list_ab.txt.
  __shared__ uint4 lp4[kCntWaves][kMaxStarts / 8 + 8];  // (+ one dummy slot per lane)
  uint16_t* lp = reinterpret_cast<uint16_t*>(lp4[threadIdx.x >> 6]);
  uint32_t cnt = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t pk = __popc(msk[2 * q]) | (__popc(msk[2 * q + 1]) << 16);
    const uint32_t inc = wave_incl_scan32(pk);
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63), ex = inc - pk;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t i = cnt + ((ex >> (16 * h)) & 0xFFFFu);
      cnt += (tot >> (16 * h)) & 0xFFFFu;
      // the lane's first colon without a branch (none: a dummy slot of its
      // own), the rare rest in a loop taken only when some lane has more
      uint32_t m = msk[2 * q + h];
      const uint32_t at0 = 1024 * (2 * q + h) + 16 * lane - 1;
      lp[m && i < (uint32_t)kMaxStarts ? i : kMaxStarts + lane] = (uint16_t)(at0 + __ffs(m));
      m &= m - 1;
      if (__ballot(m != 0) != 0)
        for (++i; m && i < (uint32_t)kMaxStarts; m &= m - 1, ++i) lp[i] = (uint16_t)(at0 + __ffs(m));
    }
  }
  if (posg) {  // (this wave's own LDS writes: in order, no workgroup barrier)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the first kListHead entries of every span side by side (the spans of a
    // workgroup write one stretch), the rest (short numbers only) after them
    uint4* head = reinterpret_cast<uint4*>(posg + span * kListHead);
    uint4* tail = reinterpret_cast<uint4*>(posg + nb * kListHead + span * (kMaxStarts - kListHead)) - kListHead / 8;
    const uint32_t n16 = (min(cnt, (uint32_t)kMaxStarts) + 7) / 8;
    for (uint32_t u = lane; u < n16; u += 64) (u < kListHead / 8 ? head : tail)[u] = lp4[threadIdx.x >> 6][u];
  }
  // whitespace (or a control byte) in a span wholly inside the text: the
  // compact fast pass cannot hold, so it is skipped (kWsBit, summed by the scan)
  const bool ws = span * kDecSpan >= t.mis && (span + 1) * kDecSpan <= t.L && __ballot(low != 0) != 0;
  if (lane == 0) bsum[span] = cnt | (ws ? kWsBit : 0);
}

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

// Length of the digit run at the start of the 40 bytes d[0..9], capped at
// 40 (a number has at most 39 digits, so a run reaching byte 40 is already a
// rejection): SWAR non-digit flags (0x80 per byte), packed one bit per byte by
// v_dot4_u32_u8 as in colons32, and one 64-bit count of trailing zeros (where
// a compare-and-select chain over the dwords took twice the VALU).
__device__ __forceinline__ uint32_t digit_run(const uint32_t (&d)[10]) {
  uint64_t mask = 1ull << 40;
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    uint32_t nd2[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t x = d[2 * q + h] ^ 0x30303030u;  // digits -> 0..9
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
// with SWAR over 40 bytes held in registers, and the value is folded in
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
// The digit run is found with SWAR over 40 bytes held in registers; the
// value is folded in base 10^8 from the same registers: full 8-digit
// chunks, then the nd % 8 leading digits of the next chunk right-aligned
// behind '0's.
template <class AfterOk>
__device__ __forceinline__ bool fast_parse(const uint32_t* l32, const uint32_t* p10, uint32_t o, bool ok,
                                           FastNum& r, AfterOk after_ok) {
  const uint32_t first = lds_dword(l32, o);
  r.minus = (first & 0xFFu) == (uint32_t)'-';
  const uint32_t ds = o + (r.minus ? 1u : 0u);
  uint32_t d[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) d[j] = lds_dword(l32, ds + 4 * j);
  const uint32_t nd = digit_run(d);
  ok = ok && nd >= 1 && nd <= 39 && !((d[0] & 0xFFu) == (uint32_t)'0' && nd > 1);
  if (!ok) return false;
  r.dend = ds + nd;
  if (!after_ok(r.dend)) return false;
  const uint32_t full = nd >> 3, rem = nd & 7u;
  bool ovf = false;
  uint32_t v[4];  // (a local, not r.v: in a persistent-loop variant r.v was kept in scratch)
  uint32_t lo, hi;  // the chunk whose leading rem digits come last
  if (full == 4) {  // 32..39 digits (a random 128-bit value): two 16-digit halves
    const uint64_t p0 = (uint64_t)digits8(d[0], d[1]) * 100000000u + digits8(d[2], d[3]);
    const uint64_t p1 = (uint64_t)digits8(d[4], d[5]) * 100000000u + digits8(d[6], d[7]);
    const unsigned __int128 t = (unsigned __int128)p0 * 10000000000000000ull + p1;  // < 10^32
    v[0] = (uint32_t)t;
    v[1] = (uint32_t)(t >> 32);
    v[2] = (uint32_t)(t >> 64);
    v[3] = (uint32_t)(t >> 96);
    lo = d[8];  // (the common case: no select chain over the registers)
    hi = d[9];
  } else {
    v[0] = v[1] = v[2] = v[3] = 0;
#pragma unroll
    for (uint32_t m = 0; m < 4; ++m)
      if (m < full) fold(v, 100000000u, digits8(d[2 * m], d[2 * m + 1]), ovf);
    lo = d[0];
    hi = d[1];
#pragma unroll
    for (uint32_t m = 1; m < 4; ++m)
      if (m == full) { lo = d[2 * m]; hi = d[2 * m + 1]; }
  }
  if (rem) {
    const uint64_t x = ((uint64_t)hi << 32) | lo;
    const uint32_t sh = 8 * (8 - rem);  // 8..56
    const uint64_t y = (x << sh) | (0x3030303030303030ull >> (64 - sh));
    fold(v, p10[rem], digits8((uint32_t)y, (uint32_t)(y >> 32)), ovf);
  }
  r.v[0] = v[0];
  r.v[1] = v[1];
  r.v[2] = v[2];
  r.v[3] = v[3];
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
  uint32_t d[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) d[j] = lds_dword(l32, ds + 4 * j);
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
__device__ __forceinline__ bool fast_segment(const uint32_t* l32, const uint32_t* p10, uint32_t o, uint64_t g,
                                             size_t nvals, size_t xo, size_t len, FastNum& r) {
  const uint32_t pre = lds_dword(l32, o - 4);
  r.key = (pre >> 8) & 0xFFu;
  // '"' k '"' ':' before a value was already checked as the end of the
  // previous value's segment (its after_ok); only the text's first value
  // has no previous one
  bool ok = true;
  if (g == 0)
    ok = (pre & 0xFFFF00FFu) == 0x3A220022u && (r.key == 'a' || r.key == 'b') && xo == 6 &&
         (lds_dword(l32, o - 6) & 0xFFFFu) == 0x7B5Bu;  // "[{"
  const uint32_t key = r.key;
  return fast_parse(l32, p10, o, ok, r, [=](uint32_t dend) {
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

// fast_segment without the value's global index (k_xdec_span parses with no
// count pass before it): the member comes from the byte before the key's
// quote ('{' member 0, ',' member 1 -- that byte ends the previous value's
// segment, which checks it).  Returns SEG_OK when the member's own form holds:
// member 0 followed by ',' "K" ':' (K the other key), member 1 by '}' ',' '{'
// "K" ':' (SEG_MID) or by '}' ']' and the end of the text (SEG_LAST); SEG_FIRST
// when the value opens the text ("[{" before its key, 6th byte).  Since every
// value's segment reaches the next value's colon, a text whose values all hold
// alternates member 0 / member 1 from its first value (which must be SEG_FIRST)
// to its last (which can only be SEG_LAST), so no check needs the index; the
// array check adds the count.
enum : uint32_t { SEG_OK = 1, SEG_M1 = 2, SEG_FIRST = 4, SEG_LAST = 8, SEG_MID = 16 };

__device__ __forceinline__ uint32_t fast_value(const uint32_t* l32, const uint32_t* p10, uint32_t o, size_t xo,
                                               size_t len, FastNum& r) {
  const uint32_t pre = lds_dword(l32, o - 5);  // bytes o-5 .. o-2: '{'|',' '"' k '"'
  r.key = (pre >> 16) & 0xFFu;
  const uint32_t lead = pre & 0xFFu;
  const bool m1 = lead == (uint32_t)',';
  // the bytes before the value were checked as the end of the previous
  // value's segment (its after_ok), except for the text's first value: it
  // must be SEG_FIRST, and only it gets the full check here
  bool ok = true;
  uint32_t flags = m1 ? SEG_M1 : 0;
  if (xo == 6) {
    ok = (pre & 0xFF00FF00u) == 0x22002200u && (r.key == 'a' || r.key == 'b') && lead == (uint32_t)'{' &&
         (lds_dword(l32, o - 1) & 0xFFu) == (uint32_t)':';
    if ((lds_dword(l32, o - 6) & 0xFFFFu) == 0x7B5Bu) flags |= SEG_FIRST;  // "[{"
  }
  const uint32_t key = r.key;
  ok = fast_parse(l32, p10, o, ok, r, [&](uint32_t dend) {
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

// The array holds exactly nvals numbers and is bracketed; an empty array
// holds nothing but whitespace (with numbers, the lanes of the decode passes
// check the rest).  Run by workgroup 0 of k_xdec_slow (256 lanes) before it
// decides whether to return: one launch fewer per decode.
__device__ __forceinline__ void array_check(const Text& t, uint64_t total, size_t nvals, unsigned long long* bad) {
  __shared__ size_t az[2];
  if (threadIdx.x == 0) {
    size_t a = t.mis;
    while (a < t.L && is_ws(t[a])) ++a;
    size_t z = t.L;
    while (z > t.mis && is_ws(t[z - 1])) --z;
    if (a >= t.L || t[a] != '[') atomicMin(bad, (unsigned long long)(a - t.mis));
    else if (z <= a + 1 || t[z - 1] != ']') atomicMin(bad, (unsigned long long)(z > t.mis ? z - 1 - t.mis : 0));
    else if (total != nvals) atomicMin(bad, (unsigned long long)(t.L - t.mis));
    az[0] = a + 1;
    az[1] = z > t.mis ? z - 1 : t.mis;
  }
  __syncthreads();
  if (nvals == 0)
    for (size_t i = az[0] + threadIdx.x; i < az[1]; i += blockDim.x)
      if (!is_ws(t[i])) atomicMin(bad, (unsigned long long)(i - t.mis));
}

// Pass 3, general (k_xdec_slow, one workgroup per span; its workgroups
// return at once unless k_xdec_fast found a value outside the compact
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
// a colon beyond that is reported as malformed (kMaxStarts, above).

// Launched on at most kSlowGrid workgroups, each taking spans blockIdx.x,
// + gridDim.x, ...: when the compact pass held, every workgroup returns at
// once, and its dispatch cost is that grid's.  One workgroup per span (92 k
// for 752 MB) cost 21 us of dispatch just to return; 16 k cost ~5 us.  The
// general pass itself (whitespace in the text) then runs 1.38x slower than on
// one workgroup per span (979 vs 710 us on 752 MB; 1 k workgroups: 1285,
// 4 k: 1058; r03 xdec A/B, profiles/r03_xdec_ab.txt).
#ifndef AMPH_XDEC_SLOW_GRID
#define AMPH_XDEC_SLOW_GRID 16384
#endif
constexpr unsigned kSlowGrid = AMPH_XDEC_SLOW_GRID;

// Span bases of the general pass: from the count pass's scan.
struct ScanBases {
  const uint64_t* bscan;
  size_t nb;
  __device__ __forceinline__ bool skip(const unsigned int* slow) const {
    return *slow == 0 && (bscan[nb] & ~kCountMask) == 0;
  }
  __device__ __forceinline__ uint64_t base(size_t span) const { return bscan[span] & kCountMask; }
  __device__ __forceinline__ uint64_t total() const { return bscan[nb] & kCountMask; }
  __device__ __forceinline__ void windows() const {}
};
// After k_xdec_span: the general pass runs when a span's count word carries
// the fail bit, or when the text holds other than nvals values (it then
// reports the first value beyond nvals, as after the count pass).  When the
// span form holds, its workgroups first complete the map's windows (XSpans)
// from the scanned bases.
struct SpanBases {
  const uint64_t* bscan;
  size_t nb, nvals;
  uint4* map;
  __device__ __forceinline__ void windows() const {
    if (bscan[nb] != nvals) return;  // fail bits or a count mismatch: pair order
    auto at = [&](size_t s, uint64_t v0, uint64_t cap) -> uint32_t {
      return (uint32_t)(s <= nb ? min(bscan[s] - v0, cap) : cap);
    };
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t b = (size_t)blockIdx.x * blockDim.x + threadIdx.x; b * kXMapValues < nvals; b += stride) {
      const uint32_t s0 = map[b].x;
      const uint64_t v0 = b * kXMapValues;
      map[b] = make_uint4(s0, (uint32_t)(v0 - bscan[s0]), at(s0 + 1, v0, 0xFFFF) | (at(s0 + 2, v0, 0xFFFF) << 16),
                          at(s0 + 3, v0, 0xFFFFFFFFu));
    }
  }
  __device__ __forceinline__ bool skip(const unsigned int*) const {
    const uint64_t t = bscan[nb];
    return (t & ~kCountMask) == 0 && (t & kCountMask) == nvals;
  }
  __device__ __forceinline__ uint64_t base(size_t span) const { return bscan[span] & kCountMask; }
  __device__ __forceinline__ uint64_t total() const { return bscan[nb] & kCountMask; }
};

template <class Bases>
__global__ __launch_bounds__(kDecBlock) void k_xdec_slow(Text text, Bases bs, size_t nb,
                                                     size_t nvals, uint4* mag, uint8_t* neg,
                                                     unsigned long long* bad,
                                                     const unsigned int* slow) {
  if (blockIdx.x == 0) array_check(text, bs.total(), nvals, bad);
  bs.windows();
  if (bs.skip(slow)) return;  // the compact pass held
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
    const uint64_t b = bs.base(span);
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

// Pass 3 (optimistic): the same staging and colon listing, then one value
// per lane checked against its compact-layout SEGMENT (fast_segment) and
// written; no whitespace walks, no records, no second phase, no general
// path in the kernel (its registers cost occupancy: 100 SGPRs with it, 72
// without).  Any value outside the compact layout (whitespace, a malformed
// byte, value 0 or the last value not in the plain form, more colons than
// expected) raises *slow, and k_xdec_slow then parses the whole text with
// the general grammar and reports errors; Jackson's compact output never
// takes it.
__global__ __launch_bounds__(kDecBlock) void k_xdec_fast(Text text, const uint64_t* bscan, size_t nb,
                                                     size_t nvals, uint4* mag, uint8_t* neg,
                                                     unsigned int* slow, const uint16_t* posg) {
  if ((bscan[nb] & ~kCountMask) != 0) return;  // whitespace somewhere: the general pass does it all
  __shared__ uint4 win4[kWin / 16 + 1];
  __shared__ uint32_t p10[8];  // 10^k, k < 8: the partial chunk's scale (one LDS read per value)
  if (threadIdx.x < 8) p10[threadIdx.x] = pow10_small(threadIdx.x);
  // the count pass's colon list (relative to b0); the first 256 read with the
  // window (entries past the span's count are unused)
  static_assert(kListHead == kDecBlock, "one head entry per lane");
  const uint32_t p0 = posg[(size_t)blockIdx.x * kListHead + threadIdx.x];
  const uint16_t* pl = posg + nb * kListHead + (size_t)blockIdx.x * (kMaxStarts - kListHead) - kListHead;
  const size_t b0 = (size_t)blockIdx.x * kDecSpan;
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
    __builtin_amdgcn_sched_barrier(0);  // (all three in flight first, as in k_xdec_span)
    win4[threadIdx.x] = make_uint4(v0.x, v0.y, v0.z, v0.w);
    win4[threadIdx.x + kDecBlock] = make_uint4(v1.x, v1.y, v1.z, v1.w);
    if ((int)threadIdx.x + 2 * kDecBlock <= kWin / 16) win4[c2] = make_uint4(v2.x, v2.y, v2.z, v2.w);
  } else {
    for (int c = threadIdx.x; c < kWin / 16 + 1; c += kDecBlock) win4[c] = text.chunk(w0 + 16LL * c);
  }
  __syncthreads();
  const uint64_t gbase = bscan[blockIdx.x] & kCountMask;
  const uint32_t total = (uint32_t)((bscan[blockIdx.x + 1] & kCountMask) - gbase);
  bool fail = total > (uint32_t)kMaxStarts;
  const uint32_t nloc = min(total, (uint32_t)kMaxStarts);
  const uint32_t* l32 = reinterpret_cast<const uint32_t*>(win4);
  const size_t len = text.L - text.mis;
  for (uint32_t idx = threadIdx.x; idx < nloc; idx += kDecBlock) {
    const uint32_t at = idx < (uint32_t)kDecBlock ? p0 : pl[idx];
    const uint64_t g = gbase + idx;
    FastNum fn;
    if (g < nvals && fast_segment(l32, p10, at + 1 + kWinPad, g, nvals, b0 + at + 1 - text.mis, len, fn)) {
      const size_t slot = (g & ~(uint64_t)1) + (fn.key == 'b');
      xst16(mag + slot, make_uint4(fn.v[0], fn.v[1], fn.v[2], fn.v[3]));
      neg[slot] = fn.minus && (fn.v[0] | fn.v[1] | fn.v[2] | fn.v[3]) != 0;
    } else {
      fail = true;
    }
  }
  if (__ballot(fail) != 0 && __lane_id() == 0) atomicOr(slow, 1u);
}

// The decode into span form (launch_exchange_decode_spans; the party
// session's partner texts), ONE read of the text with no count pass before
// it (one workgroup per span: a persistent double-buffered variant whose next
// window came in by LDS-DMA during the parse measured 294 vs 257 us,
// profiles/r03s2_xspan_dma_ab.txt): staging and colon listing as k_xdec_fast, then each value checked
// against its compact-layout segment without its global index (fast_value)
// and stored at slot kXSpanSlots * span + its rank among the span's colons,
// its byte = sign (bit 0) | key "b" (bit 1).  cnt[span] = the span's colon
// count, plus kWsBit when a value falls outside the compact layout, the span
// holds more than kXSpanSlots values, or the text's first value is not the
// span-0 value that opens it; the scan of these words gives every span its
// first value index (and the map k_open_post starts from), and any kWsBit sends
// the whole text through k_xdec_slow, which writes pair order instead.
__global__ __launch_bounds__(kDecBlock) void k_xdec_span(Text text, uint64_t* cnt, uint4* smag,
                                                     uint8_t* sneg, unsigned long long* bad) {
  // (the passes after this one report into *bad; null: the caller has reset it)
  if (bad && blockIdx.x == 0 && threadIdx.x == 0) *bad = kNoFail;
  __shared__ uint4 win4[kWin / 16 + 1];
  __shared__ uint16_t pos[kXSpanSlots];  // colon, relative to b0
  __shared__ uint32_t p10[8];  // 10^k, k < 8: the partial chunk's scale (one LDS read per value)
  __shared__ int sfail;
  if (threadIdx.x == 0) sfail = 0;
  if (threadIdx.x < 8) p10[threadIdx.x] = pow10_small(threadIdx.x);
  const size_t span = blockIdx.x, b0 = span * kDecSpan;
  const long long w0 = (long long)b0 - kWinPad;
  if (w0 >= (long long)text.mis && w0 + 16LL * (kWin / 16 + 1) <= (long long)text.L) {
    const u32x4* a = reinterpret_cast<const u32x4*>(text.al + w0);
    const int c2 = min((int)threadIdx.x + 2 * kDecBlock, kWin / 16);
    const u32x4 v0 = __builtin_nontemporal_load(a + threadIdx.x),
                v1 = __builtin_nontemporal_load(a + threadIdx.x + kDecBlock), v2 = __builtin_nontemporal_load(a + c2);
    // all three loads in flight before the first LDS write (the scheduler
    // otherwise sank the third below the first two writes' waits)
    __builtin_amdgcn_sched_barrier(0);
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
  for (int k = (int)first; m && k < kXSpanSlots; m &= m - 1, ++k)
    pos[k] = (uint16_t)(kDecBytes * threadIdx.x + __ffs(m) - 1);
  __syncthreads();
  const size_t len = text.L - text.mis;
  // span 0 holds the text's first colon (virtual offset <= 20) unless the
  // text is not compact
  bool fail = total > (uint32_t)kXSpanSlots || (span == 0 && total == 0 && len > 0);
  const uint32_t nloc = min(total, (uint32_t)kXSpanSlots);
  const uint32_t* l32 = reinterpret_cast<const uint32_t*>(win4);
  uint4* dst = smag + span * kXSpanSlots;
  uint8_t* dneg = sneg + span * kXSpanSlots;
  for (uint32_t idx = threadIdx.x; idx < nloc; idx += kDecBlock) {
    const uint32_t at = pos[idx];
    FastNum fn;
    const uint32_t f = fast_value(l32, p10, at + 1 + kWinPad, b0 + at + 1 - text.mis, len, fn);
    if ((f & SEG_OK) && (span != 0 || idx != 0 || (f & SEG_FIRST))) {
      xst16(dst + idx, make_uint4(fn.v[0], fn.v[1], fn.v[2], fn.v[3]));
      dneg[idx] = (uint8_t)((fn.minus && (fn.v[0] | fn.v[1] | fn.v[2] | fn.v[3]) != 0) | ((fn.key == 'b') << 1));
    } else {
      fail = true;
    }
  }
  if (__ballot(fail) != 0 && __lane_id() == 0) sfail = 1;  // (__syncthreads_or costs 4 KiB of LDS)
  __syncthreads();
  if (threadIdx.x == 0) cnt[span] = total | (sfail ? kWsBit : 0);
}

unsigned blocks_of(size_t n, size_t per) { return (unsigned)((n + per - 1) / per); }

// exclusive scan of x[0..n) in place, x[n] = total; bsum: blocks_of(n)+1 scratch
hipError_t scan_u64(uint64_t* x, size_t n, uint64_t* bsum, LaunchCfg c, uint4* map = nullptr,
                    size_t nmap = 0) {
  const unsigned nb = blocks_of(n, kScanBlock);
  if (nb <= 1) {
    AMPH_LAUNCH(k_scan_single, dim3(1), dim3(kScanBlock), c, x, n, map, nmap);
    return hipGetLastError();
  }
  LaunchCfg c0 = c, c2 = c;
  c0.ev_stop = nullptr;
  c2.ev_start = nullptr;
  AMPH_LAUNCH(k_scan_reduce, dim3(nb), dim3(kScanBlock), c0, x, n, bsum);
  AMPH_LAUNCH(k_scan_apply, dim3(nb), dim3(kScanBlock), c2, x, n, bsum, (size_t)nb, map, nmap);
  return hipGetLastError();
}

}  // namespace

size_t xenc_scratch_bytes(size_t npairs) {
  const size_t nb = blocks_of(npairs, kXBlock);
  return 8 * (nb + 1) + 8 * ((size_t)blocks_of(nb, kScanBlock) + 1);
}

size_t xenc_max_bytes(size_t npairs) { return (size_t)kXEntry * npairs + 2; }

// Three passes: per-workgroup text lengths (k_xenc_bsum), a scan of those
// (one u64 per 256 pairs), then k_xenc_write, which recomputes its entries'
// lengths while converting and places them with a workgroup scan -- no
// per-pair length or offset array goes through HBM.
hipError_t launch_exchange_encode(const uint4* mag, const uint8_t* neg, size_t npairs, char* out,
                                  unsigned long long* out_len, void* scratch, const LaunchCfg& c) {
  const size_t nb = npairs ? blocks_of(npairs, kXBlock) : 0;
  uint64_t* bs = static_cast<uint64_t*>(scratch);
  uint64_t* tmp = bs + nb + 1;
  LaunchCfg c0 = c, cm = c, c1 = c;
  c0.ev_stop = nullptr;
  cm.ev_start = cm.ev_stop = nullptr;
  c1.ev_start = nullptr;
  if (nb > 0) {
    AMPH_LAUNCH(k_xenc_bsum, dim3(blocks_of(nb, 4)), dim3(4 * kXBlock), c0, mag, neg, npairs, nb, bs);
    hipError_t e = scan_u64(bs, nb, tmp, cm);
    if (e != hipSuccess) return e;
  } else {
    AMPH_LAUNCH(k_scan_single, dim3(1), dim3(kScanBlock), c0, bs, (size_t)0, (uint4*)nullptr, (size_t)0);
  }
  AMPH_LAUNCH(k_xenc_write, dim3(nb ? (unsigned)nb : 1u), dim3(kXBlock), c1, mag, neg, npairs, bs,
              nb, out, out_len, 1);
  return hipGetLastError();
}

static_assert(kXBlock == 2 * kXLenPairs, "an encode workgroup spans two K_ODO_PRE length words");
size_t xenc_lens_scratch_bytes(size_t npairs) {
  return 8 * ((size_t)blocks_of(blocks_of(npairs, kXLenPairs), kScanBlock) + 1);
}

// Two passes after K_ODO_PRE's lengths: their scan, then k_xenc_write
hipError_t launch_exchange_encode_lens(const uint4* mag, const uint8_t* neg, size_t npairs, uint64_t* lens,
                                       char* out, unsigned long long* out_len, void* scratch, const LaunchCfg& c) {
  const size_t nl = npairs ? blocks_of(npairs, kXLenPairs) : 0, nb = npairs ? blocks_of(npairs, kXBlock) : 0;
  LaunchCfg c0 = c, c1 = c;
  c0.ev_stop = nullptr;
  c1.ev_start = nullptr;
  hipError_t e = scan_u64(lens, nl, static_cast<uint64_t*>(scratch), c0);
  if (e != hipSuccess) return e;
  AMPH_LAUNCH(k_xenc_write, dim3(nb ? (unsigned)nb : 1u), dim3(kXBlock), c1, mag, neg, npairs, lens, nl, out,
              out_len, 2);
  return hipGetLastError();
}

// (The pair-order decode through the span form -- the one-read span pass into
// scratch, then a gather into pair order -- measured no faster: 383-390 vs
// 382 us at 8 Mi pairs, the gather's ~100 us eating the count pass's 110;
// profiles/r03s2_xdec_pair_via_spans_ab.txt.  The party session keeps the
// span form and reads it in place.)
// span counts, scan partials, the slow-path flag, the spans' colon lists
size_t xdec_scratch_bytes(size_t len) {
  const size_t nb = blocks_of(len + 16, kDecSpan);
  return 8 * (nb + 1) + 8 * ((size_t)blocks_of(nb, kScanBlock) + 1) + 8 + 8 + 2 * (size_t)kMaxStarts * nb;
}

hipError_t launch_exchange_decode(const char* text, size_t len, size_t npairs, uint4* mag,
                                  uint8_t* neg, unsigned long long* bad, void* scratch,
                                  const LaunchCfg& c) {
  const size_t mis = (uintptr_t)text & 15;
  const Text t{reinterpret_cast<const uint8_t*>(text) - mis, mis, mis + len};
  const size_t nb = blocks_of(t.L ? t.L : 1, kDecSpan);
  LaunchCfg c0 = c, cm = c, c1 = c;
  c0.ev_stop = nullptr;
  cm.ev_start = cm.ev_stop = nullptr;
  c1.ev_start = nullptr;
  // count, scan, compact pass, general pass (+ the array check)
  uint64_t* bscan = static_cast<uint64_t*>(scratch);
  uint64_t* bsum = bscan + nb + 1;
  unsigned int* slow = reinterpret_cast<unsigned int*>(bsum + blocks_of(nb, kScanBlock) + 1);
  uint16_t* posg = reinterpret_cast<uint16_t*>(((uintptr_t)(slow + 2) + 15) & ~(uintptr_t)15);  // 16-B aligned
  AMPH_LAUNCH(k_xdec_count, dim3(blocks_of(nb, kCntWaves)), dim3(64 * kCntWaves), c0, t, bscan, nb, slow, posg);
  hipError_t e = scan_u64(bscan, nb, bsum, cm);
  if (e != hipSuccess) return e;
  AMPH_LAUNCH(k_xdec_fast, dim3((unsigned)nb), dim3(kDecBlock), cm, t, bscan, nb, 2 * npairs, mag, neg,
              slow, (const uint16_t*)posg);
  AMPH_LAUNCH(k_xdec_slow<ScanBases>, dim3((unsigned)std::min<size_t>(nb, kSlowGrid)), dim3(kDecBlock), c1, t,
              ScanBases{bscan, nb}, nb, 2 * npairs, mag, neg, bad, (const unsigned int*)slow);
  return hipGetLastError();
}


static_assert(kDecSpan == kXSpanBytes, "span form: one decode workgroup per span");

size_t xspan_spans(size_t len) { return blocks_of(len + 16, kDecSpan); }
size_t xspan_slots(size_t len, size_t npairs) {
  return std::max(xspan_spans(len) * (size_t)kXSpanSlots, 2 * npairs);
}
size_t xspan_map_words(size_t npairs) { return blocks_of(2 * npairs, kXMapValues) + 1; }
size_t xdec_spans_scratch_bytes(size_t len) { return 8 * ((size_t)blocks_of(xspan_spans(len), kScanBlock) + 1); }

// the span pass (which also resets *bad), the scan of its count words (+ the
// map), the general pass (+ the array check and the map's windows; returns at
// once unless a span failed or the count is off): four launches
hipError_t launch_exchange_decode_spans(const char* text, size_t len, size_t npairs, const XSpans& out,
                                        unsigned long long* bad, void* scratch, const LaunchCfg& c) {
  const size_t mis = (uintptr_t)text & 15;
  const Text t{reinterpret_cast<const uint8_t*>(text) - mis, mis, mis + len};
  // out.nb = xspan_spans(len) may exceed the spans the text touches by one
  // (the text's misalignment): that span reads as whitespace and holds nothing
  const size_t nb = out.nb;
  if (nb < blocks_of(t.L ? t.L : 1, kDecSpan)) return hipErrorInvalidValue;
  LaunchCfg c0 = c, cm = c, c1 = c;
  c0.ev_stop = nullptr;
  cm.ev_start = cm.ev_stop = nullptr;
  c1.ev_start = nullptr;
  AMPH_LAUNCH(k_xdec_span, dim3((unsigned)nb), dim3(kDecBlock), c0, t, out.base, out.mag, out.neg, bad);
  hipError_t e = scan_u64(out.base, nb, static_cast<uint64_t*>(scratch), cm, out.map, xspan_map_words(npairs));
  if (e != hipSuccess) return e;
  AMPH_LAUNCH(k_xdec_slow<SpanBases>, dim3((unsigned)std::min<size_t>(nb, kSlowGrid)), dim3(kDecBlock), c1, t,
              (SpanBases{out.base, nb, 2 * npairs, out.map}), nb, 2 * npairs, out.mag, out.neg, bad,
              (const unsigned int*)nullptr);
  return hipGetLastError();
}

}  // namespace amph

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
// output): a length pass, a device-wide exclusive scan of the entry lengths,
// and a write pass that formats each workgroup's entries into LDS and stores
// the contiguous run with aligned 4-byte stores.
//
// Decode (array text -> diffs): every lane classifies 32 bytes; number starts
// are counted per workgroup, scanned, and each start is parsed by the lane
// that found it at its global number index.  Each number's key ("a" / "b"),
// the object it sits in (member 0 after '{', member 1 after ','), the other
// member's key and the closing '}' are checked locally, so the pairing is
// validated without a second pass; the first malformed byte's offset is
// reported.  Whitespace between tokens is accepted, as in any JSON reader.
//
// Decimal conversion: 128-bit magnitude <-> five base-10^9 chunks (four
// 64-by-32-bit divisions by a constant per chunk), chunks <-> digits.
#include <hip/hip_ext.h>

#include "kernels.hpp"

namespace amph {

#define AMPH_LAUNCH(K, G, B, C, ...) \
  hipExtLaunchKernelGGL(K, G, B, 0, (C).stream, (C).ev_start, (C).ev_stop, 0, __VA_ARGS__)

namespace {

constexpr int kXBlock = 256;      // pairs per workgroup (encode)
constexpr int kXEntry = 92;       // max entry: {"a":-<39 digits>,"b":-<39 digits>},
constexpr int kScanBlock = 1024;  // elements per workgroup of the scan passes
constexpr int kDecBytes = 32;     // text bytes per lane (decode)
constexpr int kDecBlock = 256;
constexpr uint64_t kE9 = 1000000000ull;

__device__ __forceinline__ uint32_t divmod_e9(uint32_t (&v)[4]) {
  uint64_t rem = 0;
#pragma unroll
  for (int i = 3; i >= 0; --i) {
    const uint64_t cur = (rem << 32) | v[i];
    const uint64_t q = cur / kE9;  // < 2^32: rem < 10^9
    rem = cur - q * kE9;
    v[i] = (uint32_t)q;
  }
  return (uint32_t)rem;
}

__device__ __forceinline__ int ndigits32(uint32_t x) {  // x < 10^9; 0 -> 1
  int n = 1;
#pragma unroll
  for (uint32_t t = 10; t <= 100000000u; t *= 10) n += x >= t;
  return n;
}

// 128-bit magnitude -> base-10^9 chunks (little end first); returns the
// decimal digit count (1 for zero).
__device__ __forceinline__ int to_chunks(const uint4& m, uint32_t (&ch)[5]) {
  uint32_t v[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
  for (int k = 0; k < 5; ++k) ch[k] = divmod_e9(v);
  int top = 0;
#pragma unroll
  for (int k = 1; k < 5; ++k) top = ch[k] ? k : top;
  return 9 * top + ndigits32(ch[top]);
}

__device__ __forceinline__ bool is_zero(const uint4& m) { return (m.x | m.y | m.z | m.w) == 0; }

// {"a":A,"b":B}  (+ ',' unless last)
__device__ __forceinline__ int entry_len(const uint4& d, bool nd, const uint4& e, bool ne,
                                         bool last) {
  uint32_t ch[5];
  const int ld = to_chunks(d, ch) + (nd && !is_zero(d));
  const int le = to_chunks(e, ch) + (ne && !is_zero(e));
  return 11 + ld + le + (last ? 0 : 1);
}

__device__ __forceinline__ char* put_str(char* o, const char* s) {
  while (*s) *o++ = *s++;
  return o;
}

__device__ __forceinline__ char* put_int(char* o, const uint4& m, bool neg) {
  uint32_t ch[5];
  const int nd = to_chunks(m, ch);
  if (neg && !is_zero(m)) *o++ = '-';  // BigInteger has no negative zero
  int pos = nd;
  // digits from the least significant end
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    uint32_t x = ch[k];
    for (int j = 0; j < 9 && pos > 0; ++j) {
      const uint32_t q = x / 10u;
      o[--pos] = (char)('0' + (x - 10u * q));
      x = q;
    }
  }
  return o + nd;
}

__global__ __launch_bounds__(kMaxBlock) void k_xenc_len(const uint4* mag, const uint8_t* neg,
                                                    size_t npairs, uint64_t* lens) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < npairs; k += stride)
    lens[k] = (uint64_t)entry_len(mag[2 * k], neg[2 * k] != 0, mag[2 * k + 1], neg[2 * k + 1] != 0,
                                  k + 1 == npairs);
}

// ---- device-wide exclusive scan of u64 (three passes) ----------------------------
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

__global__ __launch_bounds__(kScanBlock) void k_scan_reduce(const uint64_t* x, size_t n,
                                                        uint64_t* bsum) {
  const size_t i = (size_t)blockIdx.x * kScanBlock + threadIdx.x;
  uint64_t total;
  block_excl_scan(i < n ? x[i] : 0, &total);
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// One workgroup: in-place exclusive scan of n values, x[n] = total.
__global__ __launch_bounds__(kScanBlock) void k_scan_single(uint64_t* x, size_t n) {
  uint64_t carry = 0;
  for (size_t base = 0; base < n; base += kScanBlock) {
    const size_t i = base + threadIdx.x;
    const uint64_t v = i < n ? x[i] : 0;
    uint64_t total;
    const uint64_t e = block_excl_scan(v, &total);
    if (i < n) x[i] = carry + e;
    carry += total;
  }
  if (threadIdx.x == 0) x[n] = carry;
}

// x[i] <- exclusive prefix (bsum already scanned); x[n] <- total
__global__ __launch_bounds__(kScanBlock) void k_scan_apply(uint64_t* x, size_t n,
                                                       const uint64_t* bsum, size_t nb) {
  const size_t i = (size_t)blockIdx.x * kScanBlock + threadIdx.x;
  uint64_t total;
  const uint64_t e = block_excl_scan(i < n ? x[i] : 0, &total);
  if (i < n) x[i] = bsum[blockIdx.x] + e;
  if (blockIdx.x == 0 && threadIdx.x == 0) x[n] = bsum[nb];
}

// Entries of one workgroup formatted into LDS, then stored as one contiguous
// run: aligned 4-byte words in the middle, single bytes at the two ends.
__global__ __launch_bounds__(kXBlock) void k_xenc_write(const uint4* mag, const uint8_t* neg,
                                                    size_t npairs, const uint64_t* offs,
                                                    char* out, unsigned long long* out_len) {
  __shared__ char buf[kXBlock * kXEntry + 8];
  const size_t k0 = (size_t)blockIdx.x * kXBlock, k = k0 + threadIdx.x;
  const size_t kend = min(k0 + (size_t)kXBlock, npairs);
  const uint64_t base = offs[k0], end = offs[kend];
  if (k < npairs) {
    char* o = buf + (offs[k] - base);
    o = put_str(o, "{\"a\":");
    o = put_int(o, mag[2 * k], neg[2 * k] != 0);
    o = put_str(o, ",\"b\":");
    o = put_int(o, mag[2 * k + 1], neg[2 * k + 1] != 0);
    *o++ = '}';
    if (k + 1 < npairs) *o = ',';
  }
  __syncthreads();
  char* dst = out + 1 + base;  // out[0] = '['
  const size_t n = end - base;
  const size_t head = min(n, (size_t)((4 - ((uintptr_t)dst & 3)) & 3));
  const size_t nw = (n - head) / 4;
  if (threadIdx.x < head) dst[threadIdx.x] = buf[threadIdx.x];
  for (size_t w = threadIdx.x; w < nw; w += kXBlock) {
    const char* s = buf + head + 4 * w;
    const uint32_t v = (uint32_t)(uint8_t)s[0] | ((uint32_t)(uint8_t)s[1] << 8) |
                       ((uint32_t)(uint8_t)s[2] << 16) | ((uint32_t)(uint8_t)s[3] << 24);
    *reinterpret_cast<uint32_t*>(dst + head + 4 * w) = v;
  }
  const size_t t0 = head + 4 * nw;
  if (threadIdx.x < n - t0) dst[t0 + threadIdx.x] = buf[t0 + threadIdx.x];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    out[0] = '[';
    out[1 + offs[npairs]] = ']';
    if (out_len) *out_len = offs[npairs] + 2;
  }
}

// ---- decode -----------------------------------------------------------------------
__device__ __forceinline__ bool is_digit(uint32_t c) { return c - '0' < 10u; }
__device__ __forceinline__ bool is_ws(uint32_t c) {
  return c == ' ' || c == '\n' || c == '\r' || c == '\t';
}
__device__ __forceinline__ bool num_char(uint32_t c) {
  return is_digit(c) || c == '-' || c == '+' || c == '.' || c == 'e' || c == 'E';
}

// Bit j of the result: byte base+j starts a number (a digit or '-' whose
// predecessor is not part of a number token).
__device__ __forceinline__ uint32_t start_mask(const uint8_t* t, size_t len, size_t base) {
  uint8_t b[kDecBytes + 1];
  b[0] = base > 0 ? t[base - 1] : ' ';
  if (base + kDecBytes <= len && (((uintptr_t)(t + base)) & 15) == 0) {
    const uint4* p = reinterpret_cast<const uint4*>(t + base);
#pragma unroll
    for (int q = 0; q < kDecBytes / 16; ++q) {
      const uint4 v = p[q];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 16; ++j) b[1 + 16 * q + j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
    }
  } else {
#pragma unroll
    for (int j = 0; j < kDecBytes; ++j) b[1 + j] = base + j < len ? t[base + j] : ' ';
  }
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < kDecBytes; ++j) {
    const uint32_t c = b[1 + j];
    m |= (uint32_t)((is_digit(c) || c == '-') && !num_char(b[j])) << j;
  }
  return m;
}

__global__ __launch_bounds__(kDecBlock) void k_xdec_count(const uint8_t* t, size_t len,
                                                      uint64_t* bsum) {
  const size_t base = ((size_t)blockIdx.x * kDecBlock + threadIdx.x) * kDecBytes;
  const uint64_t c = base < len ? __popc(start_mask(t, len, base)) : 0;
  uint64_t total;
  block_excl_scan(c, &total);
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// The workgroup's text window (its 8 KiB plus 256 B either side) staged in
// LDS; bytes outside it (long whitespace runs) come from global memory.
struct Window {
  const uint8_t* t;
  const uint8_t* lds;
  size_t w0, w1;
  __device__ __forceinline__ uint32_t operator[](size_t x) const {
    return x - w0 < w1 - w0 ? lds[x - w0] : t[x];
  }
};
constexpr int kWinPad = 256;

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

__global__ __launch_bounds__(kDecBlock) void k_xdec_parse(const uint8_t* text, size_t len,
                                                      const uint64_t* bscan, size_t nvals,
                                                      uint4* mag, uint8_t* neg,
                                                      unsigned long long* bad) {
  __shared__ uint8_t win[kDecBlock * kDecBytes + 2 * kWinPad];
  const size_t b0 = (size_t)blockIdx.x * kDecBlock * kDecBytes;
  const size_t w0 = b0 > (size_t)kWinPad ? b0 - kWinPad : 0;
  const size_t w1 = min(len, b0 + (size_t)kDecBlock * kDecBytes + kWinPad);
  for (size_t i = threadIdx.x; i < w1 - w0; i += kDecBlock) win[i] = text[w0 + i];
  const Window t{text, win, w0, w1};
  const size_t base = b0 + (size_t)threadIdx.x * kDecBytes;
  uint32_t m = base < len ? start_mask(text, len, base) : 0;
  uint64_t total;
  uint64_t g = bscan[blockIdx.x] + block_excl_scan(__popc(m), &total);  // (its barriers also publish win)
  for (; m; m &= m - 1, ++g) {
    const size_t x = base + __ffs(m) - 1;
    size_t q = 0;
    const uint32_t key = key_before(t, x, &q);
    bool ok = key != 0 && g < nvals;
    // member 0 follows '{' (itself after '[' or ','), member 1 follows ','
    const bool first = (g & 1) == 0;
    if (ok) {
      if (first) {
        ok = q > 0 && t[q - 1] == '{';
        if (ok) {
          const size_t r = skip_ws_back(t, q - 1);
          ok = r > 0 && (t[r - 1] == '[' || t[r - 1] == ',');
        }
      } else {
        ok = q > 0 && t[q - 1] == ',';
        if (ok) {  // the other member: number, then its key, then '{'
          size_t r = skip_ws_back(t, q - 1);
          while (r > 0 && is_digit(t[r - 1])) --r;
          if (r > 0 && t[r - 1] == '-') --r;
          size_t q0 = 0;
          const uint32_t k0 = key_before(t, r, &q0);
          ok = k0 != 0 && k0 != key && q0 > 0 && t[q0 - 1] == '{';
        }
      }
    }
    // the number: optional '-', 1..39 digits, value < 2^128
    size_t p = x;
    const bool minus = t[p] == '-';
    p += minus;
    uint32_t v[4] = {0, 0, 0, 0};
    int nd = 0;
    uint32_t chunk = 0, cmul = 1;
    bool ovf = false;
    auto fold = [&](uint32_t mul, uint32_t add) {  // v = v * mul + add
      uint64_t carry = add;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint64_t s = (uint64_t)v[i] * mul + carry;
        v[i] = (uint32_t)s;
        carry = s >> 32;
      }
      ovf |= carry != 0;
    };
    while (p < len && is_digit(t[p]) && nd <= 39) {
      chunk = chunk * 10u + (t[p] - '0');
      cmul *= 10u;
      if (cmul == 1000000000u) {
        fold(cmul, chunk);
        chunk = 0;
        cmul = 1;
      }
      ++p;
      ++nd;
    }
    if (cmul > 1) fold(cmul, chunk);
    ok = ok && nd > 0 && nd <= 39 && !ovf;
    if (ok) {  // the token ends the member: ws then ',' (member 0) or '}' (member 1)
      while (p < len && is_ws(t[p])) ++p;
      ok = p < len && t[p] == (first ? ',' : '}');
    }
    if (!ok) {
      atomicMin(bad, (unsigned long long)x);
      continue;
    }
    const size_t slot = (g & ~(uint64_t)1) + (key == 'b');
    mag[slot] = make_uint4(v[0], v[1], v[2], v[3]);
    neg[slot] = minus && (v[0] | v[1] | v[2] | v[3]) != 0;
  }
}

// the array holds exactly nvals numbers and is bracketed
__global__ void k_xdec_check(const uint8_t* t, size_t len, const uint64_t* bscan, size_t nb,
                             size_t nvals, unsigned long long* bad) {
  size_t a = 0;
  while (a < len && is_ws(t[a])) ++a;
  size_t z = len;
  while (z > 0 && is_ws(t[z - 1])) --z;
  if (a >= len || t[a] != '[') atomicMin(bad, (unsigned long long)a);
  else if (z == 0 || t[z - 1] != ']') atomicMin(bad, (unsigned long long)(z ? z - 1 : 0));
  else if (bscan[nb] != nvals) atomicMin(bad, (unsigned long long)len);
}

unsigned blocks_of(size_t n, size_t per) { return (unsigned)((n + per - 1) / per); }

// exclusive scan of x[0..n) in place, x[n] = total; bsum: blocks_of(n)+1 scratch
hipError_t scan_u64(uint64_t* x, size_t n, uint64_t* bsum, LaunchCfg c) {
  const unsigned nb = blocks_of(n, kScanBlock);
  if (nb <= 1) {
    AMPH_LAUNCH(k_scan_single, dim3(1), dim3(kScanBlock), c, x, n);
    return hipGetLastError();
  }
  LaunchCfg c0 = c, c1 = c, c2 = c;
  c0.ev_stop = nullptr;
  c1.ev_start = c1.ev_stop = nullptr;
  c2.ev_start = nullptr;
  AMPH_LAUNCH(k_scan_reduce, dim3(nb), dim3(kScanBlock), c0, x, n, bsum);
  AMPH_LAUNCH(k_scan_single, dim3(1), dim3(kScanBlock), c1, bsum, (size_t)nb);
  AMPH_LAUNCH(k_scan_apply, dim3(nb), dim3(kScanBlock), c2, x, n, bsum, (size_t)nb);
  return hipGetLastError();
}

}  // namespace

size_t xenc_scratch_bytes(size_t npairs) {
  return 8 * (npairs + 1) + 8 * ((size_t)blocks_of(npairs, kScanBlock) + 1);
}

size_t xenc_max_bytes(size_t npairs) { return (size_t)kXEntry * npairs + 2; }

hipError_t launch_exchange_encode(const uint4* mag, const uint8_t* neg, size_t npairs, char* out,
                                  unsigned long long* out_len, void* scratch, const LaunchCfg& c) {
  uint64_t* offs = static_cast<uint64_t*>(scratch);
  uint64_t* bsum = offs + npairs + 1;
  LaunchCfg c0 = c, cm = c, c1 = c;
  c0.ev_stop = nullptr;
  cm.ev_start = cm.ev_stop = nullptr;
  c1.ev_start = nullptr;
  if (npairs > 0) {
    AMPH_LAUNCH(k_xenc_len, dim3(blocks_of(npairs, kMaxBlock)), dim3(kMaxBlock), c0, mag, neg, npairs, offs);
    hipError_t e = scan_u64(offs, npairs, bsum, cm);
    if (e != hipSuccess) return e;
  } else {
    AMPH_LAUNCH(k_scan_single, dim3(1), dim3(kScanBlock), c0, offs, (size_t)0);
  }
  AMPH_LAUNCH(k_xenc_write, dim3(npairs ? blocks_of(npairs, kXBlock) : 1), dim3(kXBlock), c1, mag, neg,
              npairs, offs, out, out_len);
  return hipGetLastError();
}

size_t xdec_scratch_bytes(size_t len) {
  return 8 * ((size_t)blocks_of(len ? len : 1, (size_t)kDecBlock * kDecBytes) + 1);
}

hipError_t launch_exchange_decode(const char* text, size_t len, size_t npairs, uint4* mag,
                                  uint8_t* neg, unsigned long long* bad, void* scratch,
                                  const LaunchCfg& c) {
  uint64_t* bscan = static_cast<uint64_t*>(scratch);
  const uint8_t* t = reinterpret_cast<const uint8_t*>(text);
  const unsigned nb = blocks_of(len ? len : 1, (size_t)kDecBlock * kDecBytes);
  LaunchCfg c0 = c, cm = c, c1 = c;
  c0.ev_stop = nullptr;
  cm.ev_start = cm.ev_stop = nullptr;
  c1.ev_start = nullptr;
  AMPH_LAUNCH(k_xdec_count, dim3(nb), dim3(kDecBlock), c0, t, len, bscan);
  AMPH_LAUNCH(k_scan_single, dim3(1), dim3(kScanBlock), cm, bscan, (size_t)nb);
  AMPH_LAUNCH(k_xdec_parse, dim3(nb), dim3(kDecBlock), cm, t, len, bscan, 2 * npairs, mag, neg, bad);
  AMPH_LAUNCH(k_xdec_check, dim3(1), dim3(1), c1, t, len, bscan, (size_t)nb, 2 * npairs, bad);
  return hipGetLastError();
}

}  // namespace amph

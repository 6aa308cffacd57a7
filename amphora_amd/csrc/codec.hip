// Base64 wire codec kernels (gfx950) -- the step either side of the path
// (SURVEY.md 8f rank 2): the reference ships every share array as base64 in
// JSON (Jackson's default Base64Variants.MIME_NO_LINEFEEDS: standard
// alphabet, '=' padding, no line breaks; VerifiableSecretTest.java:41-90) and
// each masked word as {"value": base64(16 bytes)} (MaskedInputData.java:44-52).
//
//   k_b64_encode   byte stream -> chars, one 12-byte unit (16 chars) per lane
//   k_b64_decode   chars -> byte stream, one 16-char unit per lane, reports the
//                  first invalid character index
//   k_b64_words    16-byte words -> 24 chars each (per-word base64, "xx..x==")
//   k_b64_unwords  24-char records -> 16-byte words
//
// Pure byte work, HBM-bound; character mapping is branch-free arithmetic.
#include <hip/hip_ext.h>

#include "kernels.hpp"
#include "b64.hpp"

namespace amph {

#define AMPH_LAUNCH(K, G, B, C, ...) \
  hipExtLaunchKernelGGL(K, G, B, 0, (C).stream, (C).ev_start, (C).ev_stop, 0, __VA_ARGS__)

namespace {


// ASCII -> 0..63, or 0xFF if not in the alphabet
__device__ __forceinline__ uint32_t dec6(uint32_t c) {
  uint32_t v = 0xFFu;
  v = (c >= 'A' && c <= 'Z') ? c - 'A' : v;
  v = (c >= 'a' && c <= 'z') ? c - 'a' + 26u : v;
  v = (c >= '0' && c <= '9') ? c - '0' + 52u : v;
  v = c == '+' ? 62u : v;
  v = c == '/' ? 63u : v;
  return v;
}

// Text and decoded bytes leave through nontemporal stores (the result words
// of kernels.hip measured 3-7 % faster that way; AMPH_CODEC_NT=0 for A/B).
#ifndef AMPH_CODEC_NT
#define AMPH_CODEC_NT 1
#endif
typedef unsigned int cu32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16(void* p, uint4 v) {
  if constexpr (AMPH_CODEC_NT) __builtin_nontemporal_store(cu32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<cu32x4*>(p));
  else *reinterpret_cast<uint4*>(p) = v;
}
__device__ __forceinline__ void st4(uint32_t* p, uint32_t v) {
  if constexpr (AMPH_CODEC_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// One 12-byte unit t of a byte stream (the final one may be partial and
// '='-padded; unaligned buffers byte by byte) -> its 16 chars.
__device__ __forceinline__ void encode_unit(const uint8_t* in, size_t nbytes, char* out, size_t t) {
  const size_t base = 12 * t;
  const size_t rem = nbytes - base < 12 ? nbytes - base : 12;
  uint8_t b[12];
  if (rem == 12 && (((uintptr_t)(in + base)) & 3) == 0) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(in + base);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const uint32_t x = __builtin_nontemporal_load(w + q);
      b[4 * q] = x & 0xFF; b[4 * q + 1] = (x >> 8) & 0xFF;
      b[4 * q + 2] = (x >> 16) & 0xFF; b[4 * q + 3] = x >> 24;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 12; ++q) b[q] = (size_t)q < rem ? in[base + q] : 0;
  }
  uint32_t g[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) g[q] = enc_group(b[3 * q], b[3 * q + 1], b[3 * q + 2]);
  char* o = out + 16 * t;
  if (rem == 12 && (((uintptr_t)o) & 15) == 0) {
    st16(o, make_uint4(g[0], g[1], g[2], g[3]));
  } else {
    // final partial unit: ceil(rem / 3) groups, '=' for the missing bytes
    const int groups = (int)((rem + 2) / 3);
    for (int q = 0; q < groups; ++q) {
      const int have = (int)rem - 3 * q;  // bytes present in this group (1..3)
      for (int k = 0; k < 4; ++k) {
        char ch = (char)((g[q] >> (8 * k)) & 0xFF);
        if (k >= 2 && have < k) ch = '=';
        o[4 * q + k] = ch;
      }
    }
  }
}

__global__ __launch_bounds__(kMaxBlock) void k_b64_encode(const uint8_t* in, size_t nbytes,
                                                      char* out) {
  const size_t units = (nbytes + 11) / 12;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < units; t += stride)
    encode_unit(in, nbytes, out, t);
}

// One 16-character unit t of a text (nchars % 4 == 0; the final unit may be
// partial and carry '=' padding when text_end) -> its bytes below out_bytes;
// bad = first invalid index (ibase + offset).
__device__ __forceinline__ void decode_unit(const char* in, size_t nchars, uint8_t* out, size_t out_bytes,
                                            unsigned long long* bad, size_t ibase, int text_end, size_t t) {
  const size_t base = 16 * t;
  const size_t rem = nchars - base < 16 ? nchars - base : 16;
  uint8_t c[16];
  if (rem == 16 && (((uintptr_t)(in + base)) & 15) == 0) {
    const uint4 v = *reinterpret_cast<const uint4*>(in + base);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 16; ++q) c[q] = (w[q >> 2] >> (8 * (q & 3))) & 0xFF;
  } else {
#pragma unroll
    for (int q = 0; q < 16; ++q) c[q] = (size_t)q < rem ? (uint8_t)in[base + q] : 'A';
  }
  uint32_t firstbad = 0xFFFFFFFFu;
  uint8_t o[12];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const size_t pos = base + 4 * q + k;
      // '=' is legal only in the last two positions of the whole text
      const bool pad_ok = text_end && c[4 * q + k] == '=' && pos >= nchars - 2 &&
                          (pos == nchars - 1 || in[nchars - 1] == '=');
      v[k] = pad_ok ? 0u : dec6(c[4 * q + k]);
      if (v[k] == 0xFFu && firstbad == 0xFFFFFFFFu) firstbad = (uint32_t)(4 * q + k);
    }
    const uint32_t g = (v[0] << 18) | (v[1] << 12) | (v[2] << 6) | v[3];
    o[3 * q] = (g >> 16) & 0xFF;
    o[3 * q + 1] = (g >> 8) & 0xFF;
    o[3 * q + 2] = g & 0xFF;
  }
  if (firstbad != 0xFFFFFFFFu && (size_t)firstbad < rem) atomicMin(bad, (unsigned long long)(ibase + base + firstbad));
  const size_t ob = 12 * t;
  uint8_t* op = out + ob;
  if (ob + 12 <= out_bytes && (((uintptr_t)op) & 3) == 0) {
    uint32_t* w = reinterpret_cast<uint32_t*>(op);
#pragma unroll
    for (int q = 0; q < 3; ++q)
      st4(w + q, o[4 * q] | (o[4 * q + 1] << 8) | (o[4 * q + 2] << 16) | ((uint32_t)o[4 * q + 3] << 24));
  } else {
    for (int q = 0; q < 12; ++q)
      if (ob + q < out_bytes) op[q] = o[q];
  }
}

// out_bytes = kB64PadOnDevice (with text_end): the text's last two characters
// size the output here (no host read-back)
__device__ __forceinline__ size_t dev_out_bytes(const char* in, size_t nchars, size_t out_bytes) {
  if (out_bytes != kB64PadOnDevice) return out_bytes;
  const bool p1 = nchars >= 1 && in[nchars - 1] == '=', p2 = p1 && nchars >= 2 && in[nchars - 2] == '=';
  return 3 * nchars / 4 - (size_t)p1 - (size_t)p2;
}

// nchars % 4 == 0; out_bytes = 3 nchars / 4 - padding (or kB64PadOnDevice
// with text_end); bad = first invalid index
__global__ __launch_bounds__(kMaxBlock) void k_b64_decode(const char* in, size_t nchars,
                                                      uint8_t* out, size_t out_bytes,
                                                      unsigned long long* bad, size_t ibase,
                                                      int text_end) {
  out_bytes = dev_out_bytes(in, nchars, out_bytes);
  const size_t units = (nchars + 15) / 16;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < units; t += stride)
    decode_unit(in, nchars, out, out_bytes, bad, ibase, text_end, t);
}

// 16-byte word -> 24 chars ("...==": 5 full groups + 1 byte)
__global__ __launch_bounds__(kMaxBlock) void k_b64_words(const uint4* in, size_t words, char* out) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
    uint32_t g[6];
    enc_word24(in[i], g);
    uint2* o = reinterpret_cast<uint2*>(out + 24 * i);  // 8-byte aligned when out is
    o[0] = make_uint2(g[0], g[1]);
    o[1] = make_uint2(g[2], g[3]);
    o[2] = make_uint2(g[4], g[5]);
  }
}

// 24-char records -> 16-byte words; bad = first invalid record index.
// Characters 0-15 decode as one unit (b64.hpp dec_unit16_ok: the 6-bit
// value path with the tables in VGPRs, ~40 % fewer VALU than dec4 + its
// shift packing), 16-21 as two groups, the final "==" as 'A'.
__global__ __launch_bounds__(kMaxBlock) void k_b64_unwords(const char* in, size_t words, uint4* out,
                                                       unsigned long long* bad, size_t ibase) {
  const DecTabs tabs = dec_tabs_vgpr();
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
    const uint2* p = reinterpret_cast<const uint2*>(in + 24 * i);
    const uint2 x0 = p[0], x1 = p[1], x2 = p[2];
    uint32_t ok = 0x80808080u, o[3];
    dec_unit16_ok(make_uint4(x0.x, x0.y, x1.x, x1.y), o, ok, tabs);
    // the last group's two '=' decode as 'A' (value 0); like java.util.Base64
    // / Jackson, the unused low bits of the last group are ignored
    const uint32_t v4 = dec4_values6(x2.x, ok, tabs), v5 = dec4_values6((x2.y & 0xFFFFu) | 0x41410000u, ok, tabs);
    const uint32_t g4 = (__builtin_amdgcn_udot4(v4, 0x00000140u, 0u, false) << 12) |
                        __builtin_amdgcn_udot4(v4, 0x01400000u, 0u, false);
    const uint32_t g5 = __builtin_amdgcn_udot4(v5, 0x00000140u, 0u, false) << 12;
    out[i] = make_uint4(o[0], o[1], o[2], __builtin_amdgcn_perm(g5, g4, 0x06000102u));
    if (ok != 0x80808080u || (x2.y >> 16) != 0x3D3Du) atomicMin(bad, (unsigned long long)(ibase + i));
  }
}

// Workgroup-staged bulk kernels: a block's contiguous run of input (encode:
// 12 B x 256 units) or output (decode) moves as fully coalesced 16-B
// accesses through LDS, each lane still codes its own 12-byte unit from /
// into LDS (3-dword lane stride: conflict-free).  +46 % encode, +43 % decode
// over the per-lane kernels (tools/ubench/ubench_b64.hip).  Full blocks
// only, 16-B aligned buffers; the final unit (partial / '=' padded) and any
// ragged tail go to the per-lane kernels above.
constexpr int kB64Block = 256;

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldnt4(const uint4* p) {
  const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// The stream's units past the whole blocks (at most kB64Block, the final one
// possibly partial) are the LAST workgroup's, one per lane through the
// per-unit path: one launch per call where a separate tail kernel cost a
// dispatch (~5 us) per call.
__global__ __launch_bounds__(kB64Block) void k_b64_encode_blk(const uint8_t* in, char* out, size_t nbytes) {
  if (blockIdx.x + 1 == gridDim.x) {
    const size_t units = (nbytes + 11) / 12, t = (size_t)blockIdx.x * kB64Block + threadIdx.x;
    if (t < units) encode_unit(in, nbytes, out, t);
    return;
  }
  __shared__ uint32_t lds[3 * kB64Block];
  const size_t u0 = (size_t)blockIdx.x * kB64Block, t = u0 + threadIdx.x;
  const uint4* src = reinterpret_cast<const uint4*>(in + 12 * u0);
  for (int q = threadIdx.x; q < 3 * kB64Block / 4; q += kB64Block) {
    const uint4 v = ldnt4(src + q);
    lds[4 * q] = v.x; lds[4 * q + 1] = v.y; lds[4 * q + 2] = v.z; lds[4 * q + 3] = v.w;
  }
  __syncthreads();
  const uint32_t w[3] = {lds[3 * threadIdx.x], lds[3 * threadIdx.x + 1], lds[3 * threadIdx.x + 2]};
  uint32_t g[4];
  enc_unit12(w, g);
  st16(out + 16 * t, make_uint4(g[0], g[1], g[2], g[3]));  // (nontemporal: 104.3 -> 99.4 us per 256 MiB)
}

// (the last workgroup: the remaining units, as k_b64_encode_blk)
__global__ __launch_bounds__(kB64Block) void k_b64_decode_blk(const char* in, uint8_t* out,
                                                             unsigned long long* bad, size_t nchars,
                                                             size_t out_bytes, int text_end) {
  if (blockIdx.x + 1 == gridDim.x) {
    const size_t units = (nchars + 15) / 16, t = (size_t)blockIdx.x * kB64Block + threadIdx.x;
    if (t < units) decode_unit(in, nchars, out, dev_out_bytes(in, nchars, out_bytes), bad, 0, text_end, t);
    return;
  }
  __shared__ uint32_t lds[3 * kB64Block];
  const size_t u0 = (size_t)blockIdx.x * kB64Block, t = u0 + threadIdx.x;
  const uint4 v = ldnt4(reinterpret_cast<const uint4*>(in) + t);
  uint32_t ok = 0x80808080u, o[3];  // no '=' before the final unit
  dec_unit16_ok(v, o, ok, dec_tabs_vgpr());
  if (ok != 0x80808080u) {  // (rare) locate the first bad character exactly
    uint32_t o2[3];
    atomicMin(bad, (unsigned long long)(16 * t + dec_unit16(v, o2)));
  }
  lds[3 * threadIdx.x] = o[0];
  lds[3 * threadIdx.x + 1] = o[1];
  lds[3 * threadIdx.x + 2] = o[2];
  __syncthreads();
  // nontemporal: in the client pipeline (15 field decodes, then K_RV /
  // K_MASK reads the words) the download took 0.699 -> 0.671-0.686 ms and
  // the consumer kernel 0.20 -> 0.19 ms, interleaved on one box; a loop of
  // this kernel alone over one buffer prefers plain stores (94.5 vs 100.1 us
  // per 256 MiB), the real sequence does not (profiles/r06_codec_store_policy_ab.txt)
  uint4* dst = reinterpret_cast<uint4*>(out + 12 * u0);
  for (int q = threadIdx.x; q < 3 * kB64Block / 4; q += kB64Block)
    st16(dst + q, make_uint4(lds[4 * q], lds[4 * q + 1], lds[4 * q + 2], lds[4 * q + 3]));
}

// Per-word records through LDS: the block's 256 x 24 output chars move as
// 384 coalesced 16-B stores (the per-lane kernel stores 8 B at a 24-B lane
// stride): 3.74 -> 4.86 TB/s at 16 Mi words (round 1; 6.1 -> 6.45 TB/s
// sustained with the stores nontemporal, round 6).
// (words % 256 != 0: the last workgroup codes the remaining words per lane)
__global__ __launch_bounds__(kB64Block) void k_b64_words_blk(const uint4* in, char* out, size_t words) {
  if ((size_t)(blockIdx.x + 1) * kB64Block > words) {
    const size_t i = (size_t)blockIdx.x * kB64Block + threadIdx.x;
    if (i < words) {
      uint32_t g[6];
      enc_word24(in[i], g);
      uint2* o = reinterpret_cast<uint2*>(out + 24 * i);
      o[0] = make_uint2(g[0], g[1]);
      o[1] = make_uint2(g[2], g[3]);
      o[2] = make_uint2(g[4], g[5]);
    }
    return;
  }
  __shared__ uint32_t lds[6 * kB64Block];
  const size_t i0 = (size_t)blockIdx.x * kB64Block, i = i0 + threadIdx.x;
  uint32_t g[6];
  enc_word24(ldnt4(in + i), g);
#pragma unroll
  for (int q = 0; q < 6; ++q) lds[6 * threadIdx.x + q] = g[q];
  __syncthreads();
  // nontemporal 16-byte runs: 110.5 -> 104.1 us per 16 Mi words; each lane's
  // own record as three nontemporal 8-byte stores (what k_mask_b64 now does,
  // wire.hip) took 120.2 here (profiles/r06_codec_store_policy_ab.txt)
  uint4* dst = reinterpret_cast<uint4*>(out + 24 * i0);
  for (int q = threadIdx.x; q < 6 * kB64Block / 4; q += kB64Block)
    st16(dst + q, make_uint4(lds[4 * q], lds[4 * q + 1], lds[4 * q + 2], lds[4 * q + 3]));
}

// Several equal-length byte streams (the five ODO fields of a party session)
// in ONE launch: blockIdx.y = the stream; each workgroup codes 256 12-byte
// units, staged through LDS as k_b64_encode_blk when they are all whole and
// the buffers 16-byte aligned, else unit by unit as k_b64_encode (the streams'
// final unit, '='-padded).  One launch where five k_b64_encode_blk + five
// tail launches queued ten.
struct B64Streams {
  const uint8_t* in[5];
  char* out[5];
};

__global__ __launch_bounds__(kB64Block) void k_b64_encode_multi(B64Streams st, size_t nbytes) {
  __shared__ uint32_t lds[3 * kB64Block];
  const uint8_t* in = st.in[blockIdx.y];
  char* out = st.out[blockIdx.y];
  const size_t units = (nbytes + 11) / 12, u0 = (size_t)blockIdx.x * kB64Block, t = u0 + threadIdx.x;
  const bool whole = 12 * (u0 + kB64Block) <= nbytes && ((((uintptr_t)in | (uintptr_t)out) & 15) == 0);
  if (whole) {
    const uint4* src = reinterpret_cast<const uint4*>(in + 12 * u0);
    for (int q = threadIdx.x; q < 3 * kB64Block / 4; q += kB64Block) {
      const uint4 v = ldnt4(src + q);
      lds[4 * q] = v.x; lds[4 * q + 1] = v.y; lds[4 * q + 2] = v.z; lds[4 * q + 3] = v.w;
    }
    __syncthreads();
    const uint32_t w[3] = {lds[3 * threadIdx.x], lds[3 * threadIdx.x + 1], lds[3 * threadIdx.x + 2]};
    uint32_t g[4];
    enc_unit12(w, g);
    st16(out + 16 * t, make_uint4(g[0], g[1], g[2], g[3]));
    return;
  }
  if (t >= units) return;
  const size_t base = 12 * t, rem = nbytes - base < 12 ? nbytes - base : 12;
  uint8_t b[12];
#pragma unroll
  for (int q = 0; q < 12; ++q) b[q] = (size_t)q < rem ? in[base + q] : 0;
  uint32_t g[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) g[q] = enc_group(b[3 * q], b[3 * q + 1], b[3 * q + 2]);
  char* o = out + 16 * t;
  const int groups = (int)((rem + 2) / 3);
  for (int q = 0; q < groups; ++q) {
    const int have = (int)rem - 3 * q;
    for (int k = 0; k < 4; ++k) {
      char ch = (char)((g[q] >> (8 * k)) & 0xFF);
      if (k >= 2 && have < k) ch = '=';
      o[4 * q + k] = ch;
    }
  }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

unsigned grid_n(size_t n, const LaunchCfg& c) {
  size_t g = (n + c.block - 1) / c.block;
  if (c.grid_cap > 0 && g > (size_t)c.grid_cap) g = (size_t)c.grid_cap;
  if (g > 0x7FFFFFFFu) g = 0x7FFFFFFFu;
  return (unsigned)(g ? g : 1);
}

}  // namespace

// Bulk: full 256-unit blocks that end before the final unit, when both
// buffers are 16-B aligned; the rest: the per-lane kernel on the tail.
hipError_t launch_b64_encode(const uint8_t* in, size_t nbytes, char* out, const LaunchCfg& c) {
  if (nbytes == 0) return hipSuccess;
  const size_t units = (nbytes + 11) / 12;
  const size_t nblk = aligned16(in) && aligned16(out) ? (units - 1) / kB64Block : 0;
  if (nblk) {  // whole blocks + the tail as the last workgroup, one launch
    AMPH_LAUNCH(k_b64_encode_blk, dim3((unsigned)nblk + 1), dim3(kB64Block), c, in, out, nbytes);
    return hipGetLastError();
  }
  AMPH_LAUNCH(k_b64_encode, dim3(grid_n(units, c)), dim3(c.block), c, in, nbytes, out);
  return hipGetLastError();
}

hipError_t launch_b64_encode_multi(const uint8_t* const* in, char* const* out, int n, size_t nbytes,
                                   const LaunchCfg& c) {
  if (nbytes == 0 || n <= 0) return hipSuccess;
  if (n > 5) return hipErrorInvalidValue;
  B64Streams st{};
  for (int k = 0; k < n; ++k) {
    st.in[k] = in[k];
    st.out[k] = out[k];
  }
  const size_t units = (nbytes + 11) / 12;
  AMPH_LAUNCH(k_b64_encode_multi, dim3((unsigned)((units + kB64Block - 1) / kB64Block), (unsigned)n),
              dim3(kB64Block), c, st, nbytes);
  return hipGetLastError();
}

hipError_t launch_b64_decode(const char* in, size_t nchars, uint8_t* out, size_t out_bytes,
                             unsigned long long* bad, const LaunchCfg& c, bool text_end) {
  if (nchars == 0) return hipSuccess;
  const size_t units = (nchars + 15) / 16;
  const size_t nblk = aligned16(in) && aligned16(out) ? (units - 1) / kB64Block : 0;
  if (nblk) {  // whole blocks + the tail as the last workgroup, one launch
    AMPH_LAUNCH(k_b64_decode_blk, dim3((unsigned)nblk + 1), dim3(kB64Block), c, in, out, bad, nchars, out_bytes,
                (int)text_end);
    return hipGetLastError();
  }
  AMPH_LAUNCH(k_b64_decode, dim3(grid_n(units, c)), dim3(c.block), c, in, nchars, out, out_bytes, bad, (size_t)0,
              (int)text_end);
  return hipGetLastError();
}

hipError_t launch_b64_words(const uint4* in, size_t words, char* out, const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  if (aligned16(in) && aligned16(out) && words >= (size_t)kB64Block) {  // one launch, tail included
    AMPH_LAUNCH(k_b64_words_blk, dim3((unsigned)((words + kB64Block - 1) / kB64Block)), dim3(kB64Block), c, in,
                out, words);
    return hipGetLastError();
  }
  AMPH_LAUNCH(k_b64_words, dim3(grid_n(words, c)), dim3(c.block), c, in, words, out);
  return hipGetLastError();
}

hipError_t launch_b64_unwords(const char* in, size_t words, uint4* out, unsigned long long* bad,
                              const LaunchCfg& c) {
  // (an LDS-staged variant of the 24-char record loads measured no faster)
  if (words == 0) return hipSuccess;
  AMPH_LAUNCH(k_b64_unwords, dim3(grid_n(words, c)), dim3(c.block), c, in, words, out, bad, (size_t)0);
  return hipGetLastError();
}

}  // namespace amph

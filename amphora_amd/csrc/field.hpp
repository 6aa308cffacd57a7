// Prime-field arithmetic for one 128-bit word per lane (gfx950).
//
// A word is four 32-bit limbs, little-endian (limb 0 = bits 0..31), held in
// four VGPRs.  All additive work stays in the Montgomery domain the wire
// format already uses: a wire word is [x] = x * R mod p with R = 2^128
// (mp-spdz-integration 0.2.2 toGfp, restated in oracle/amphora_oracle.py).
//
//   [x] + [y] = [x + y]               -> recombine = sum of raw words mod p
//   mont_mul([a], [b]) = [a b]        -> MAC check  [y][r] == [w]
//   mont_mul(x, R^2) = [x]            -> canonical secret to wire form
//   redc([x]) = x                     -> wire form to canonical secret
//
// Multiplication is CIOS Montgomery (Koc et al.) on 32-bit limbs: each
// (64-bit) = a*b + t + carry step lowers to one v_mad_u64_u32 plus a carry
// add.  Add/sub chains use __builtin_addc/__builtin_subc, which lower to
// v_add_co_u32 / v_addc_co_u32 (v_sub_co / v_subb_co).
//
// Bounds used throughout (p odd, p < 2^128):
//   * mont_mul(a, b) with a < 2^128 and b < p returns a value < 2p before the
//     final conditional subtract, so one subtract makes it canonical.
//   * BIG (p > 2^127): every 128-bit word is < 2p, so canon() is one
//     conditional subtract and a + b of canonical values needs a 129th bit.
//   * !BIG: canon(x) = redc(mont_mul(x, R^2)) (rare configuration).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace amph {

struct Fp {
  uint32_t p[4];
  uint32_t r2[4];   // R^2 mod p
  uint32_t n0;      // -p^-1 mod 2^32
  uint32_t big;     // p > 2^127
};

struct W4 {
  uint32_t v[4];
};

__host__ __device__ __forceinline__ W4 w4(uint4 x) { return W4{{x.x, x.y, x.z, x.w}}; }
__host__ __device__ __forceinline__ uint4 u4(const W4& a) {
  return make_uint4(a.v[0], a.v[1], a.v[2], a.v[3]);
}

__host__ __device__ __forceinline__ uint32_t addc(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_addc(a, b, cin, cout);
#else
  uint64_t s = (uint64_t)a + b + cin;
  *cout = (uint32_t)(s >> 32);
  return (uint32_t)s;
#endif
}

__host__ __device__ __forceinline__ uint32_t subc(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_subc(a, b, bin, bout);
#else
  uint64_t d = (uint64_t)a - b - bin;
  *bout = (uint32_t)(d >> 63);
  return (uint32_t)d;
#endif
}

// s = a - p; returns borrow
__host__ __device__ __forceinline__ uint32_t sub_p(const W4& a, const Fp& f, W4& s) {
  uint32_t b;
  s.v[0] = subc(a.v[0], f.p[0], 0, &b);
  s.v[1] = subc(a.v[1], f.p[1], b, &b);
  s.v[2] = subc(a.v[2], f.p[2], b, &b);
  s.v[3] = subc(a.v[3], f.p[3], b, &b);
  return b;
}

__host__ __device__ __forceinline__ W4 sel(bool c, const W4& a, const W4& b) {
  return W4{{c ? a.v[0] : b.v[0], c ? a.v[1] : b.v[1], c ? a.v[2] : b.v[2], c ? a.v[3] : b.v[3]}};
}

__host__ __device__ __forceinline__ bool eq(const W4& a, const W4& b) {
  return ((a.v[0] ^ b.v[0]) | (a.v[1] ^ b.v[1]) | (a.v[2] ^ b.v[2]) | (a.v[3] ^ b.v[3])) == 0;
}

// (hi:a) with hi in {0,1} and value < 2p  ->  canonical
__host__ __device__ __forceinline__ W4 reduce_once(const W4& a, uint32_t hi, const Fp& f) {
  W4 s;
  uint32_t b = sub_p(a, f, s);
  return sel((hi != 0) | (b == 0), s, a);
}

__host__ __device__ __forceinline__ W4 mod_add(const W4& a, const W4& b, const Fp& f) {
  W4 s;
  uint32_t c;
  s.v[0] = addc(a.v[0], b.v[0], 0, &c);
  s.v[1] = addc(a.v[1], b.v[1], c, &c);
  s.v[2] = addc(a.v[2], b.v[2], c, &c);
  s.v[3] = addc(a.v[3], b.v[3], c, &c);
  return reduce_once(s, c, f);
}

__host__ __device__ __forceinline__ W4 mod_sub(const W4& a, const W4& b, const Fp& f) {
  W4 d, e;
  uint32_t bw, c;
  d.v[0] = subc(a.v[0], b.v[0], 0, &bw);
  d.v[1] = subc(a.v[1], b.v[1], bw, &bw);
  d.v[2] = subc(a.v[2], b.v[2], bw, &bw);
  d.v[3] = subc(a.v[3], b.v[3], bw, &bw);
  e.v[0] = addc(d.v[0], f.p[0], 0, &c);
  e.v[1] = addc(d.v[1], f.p[1], c, &c);
  e.v[2] = addc(d.v[2], f.p[2], c, &c);
  e.v[3] = addc(d.v[3], f.p[3], c, &c);
  return sel(bw != 0, e, d);
}

// t = x - y (128-bit, no reduction); returns borrow (x < y)
__host__ __device__ __forceinline__ uint32_t sub128(const W4& x, const W4& y, W4& t) {
  uint32_t b;
  t.v[0] = subc(x.v[0], y.v[0], 0, &b);
  t.v[1] = subc(x.v[1], y.v[1], b, &b);
  t.v[2] = subc(x.v[2], y.v[2], b, &b);
  t.v[3] = subc(x.v[3], y.v[3], b, &b);
  return b;
}

__host__ __device__ __forceinline__ uint64_t mad32(uint32_t a, uint32_t b, uint64_t c) {
  return (uint64_t)a * b + c;
}

// CIOS Montgomery product a * b * 2^-128 mod p.  Requires a < 2^128, b < p
// (or the symmetric case); returns a canonical value.
__host__ __device__ __forceinline__ W4 mont_mul_cios(const W4& a, const W4& b, const Fp& f) {
  uint32_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t bi = b.v[i];
    uint64_t c;
    c = mad32(a.v[0], bi, t0);                       t0 = (uint32_t)c;
    c = mad32(a.v[1], bi, (uint64_t)t1 + (c >> 32)); t1 = (uint32_t)c;
    c = mad32(a.v[2], bi, (uint64_t)t2 + (c >> 32)); t2 = (uint32_t)c;
    c = mad32(a.v[3], bi, (uint64_t)t3 + (c >> 32)); t3 = (uint32_t)c;
    c = (uint64_t)t4 + (c >> 32);                    t4 = (uint32_t)c; t5 = (uint32_t)(c >> 32);
    const uint32_t m = t0 * f.n0;
    c = mad32(m, f.p[0], t0);
    c = mad32(m, f.p[1], (uint64_t)t1 + (c >> 32)); t0 = (uint32_t)c;
    c = mad32(m, f.p[2], (uint64_t)t2 + (c >> 32)); t1 = (uint32_t)c;
    c = mad32(m, f.p[3], (uint64_t)t3 + (c >> 32)); t2 = (uint32_t)c;
    c = (uint64_t)t4 + (c >> 32);                   t3 = (uint32_t)c;
    t4 = t5 + (uint32_t)(c >> 32);
  }
  return reduce_once(W4{{t0, t1, t2, t3}}, t4, f);
}

// acc += a * b on a 96-bit accumulator (lo: 64 bits, hi: 32): one
// v_mad_u64_u32 whose carry-out (vcc) goes straight into the top word.  The
// compiler's own lowering of the same sum builds zero-extended 64-bit addends
// around every mad (v_mov_b32 + 64-bit adds, ~5 instructions per product).
__host__ __device__ __forceinline__ void macc96(uint64_t& lo, uint32_t& hi, uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t out;
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %4\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "=&v"(out), "+v"(hi)
      : "v"(a), "v"(b), "v"(lo)
      : "vcc");
  lo = out;
#else
  const uint64_t p = (uint64_t)a * b, s = p + lo;
  hi += s < p;
  lo = s;
#endif
}

// Product-scanning (FIPS) Montgomery product: column k of a*b and m*p summed
// in the 96-bit accumulator, m_k chosen as the column's low word comes up,
// then shifted out.  Same contract as mont_mul_cios (a < 2^128, b < p; the
// 129-bit result < 2p is reduced once).  ~100 VALU instructions instead of
// ~165 (tools/ubench/ubench_mm.hip).
__host__ __device__ __forceinline__ W4 mont_mul_ps(const W4& a, const W4& b, const Fp& f) {
  uint32_t m[4], r[4];
  uint64_t lo = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
#pragma unroll
    for (int i = 0; i < k; ++i) {
      macc96(lo, hi, a.v[i], b.v[k - i]);
      macc96(lo, hi, m[i], f.p[k - i]);
    }
    macc96(lo, hi, a.v[k], b.v[0]);
    m[k] = (uint32_t)lo * f.n0;
    macc96(lo, hi, m[k], f.p[0]);  // the low word becomes zero
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int k = 4; k < 7; ++k) {
#pragma unroll
    for (int i = k - 3; i < 4; ++i) {
      macc96(lo, hi, a.v[i], b.v[k - i]);
      macc96(lo, hi, m[i], f.p[k - i]);
    }
    r[k - 4] = (uint32_t)lo;
    lo = (lo >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  r[3] = (uint32_t)lo;
  return reduce_once(W4{{r[0], r[1], r[2], r[3]}}, (uint32_t)(lo >> 32), f);
}

// The HBM-bound kernels keep the compiler's CIOS lowering: there the VALU
// work hides under the memory stream anyway, and mont_mul_ps's extra live
// registers took K_RV at 2 parties from 62 to 66 VGPRs (7 waves per SIMD: one
// 1024-lane workgroup per CU instead of two, 35.4 vs 33 us at C2).  The
// VALU-bound wire kernels (k_rv_b64, k_mask_b64) call mont_mul_ps.
__host__ __device__ __forceinline__ W4 mont_mul(const W4& a, const W4& b, const Fp& f) {
  return mont_mul_cios(a, b, f);
}

// Montgomery product for VALU-bound kernels (see above).
__host__ __device__ __forceinline__ W4 mont_mul_v(const W4& a, const W4& b, const Fp& f) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(AMPH_MONT_CIOS)
  return mont_mul_ps(a, b, f);
#else
  return mont_mul_cios(a, b, f);
#endif
}

// Montgomery reduction of a single word: a * 2^-128 mod p (a < 2^128).
// = fromGfp on a wire word.
__host__ __device__ __forceinline__ W4 redc(const W4& a, const Fp& f) {
  uint32_t t0 = a.v[0], t1 = a.v[1], t2 = a.v[2], t3 = a.v[3], t4 = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t m = t0 * f.n0;
    uint64_t c;
    c = mad32(m, f.p[0], t0);
    c = mad32(m, f.p[1], (uint64_t)t1 + (c >> 32)); t0 = (uint32_t)c;
    c = mad32(m, f.p[2], (uint64_t)t2 + (c >> 32)); t1 = (uint32_t)c;
    c = mad32(m, f.p[3], (uint64_t)t3 + (c >> 32)); t2 = (uint32_t)c;
    c = (uint64_t)t4 + (c >> 32);                   t3 = (uint32_t)c;
    t4 = (uint32_t)(c >> 32);
  }
  return reduce_once(W4{{t0, t1, t2, t3}}, t4, f);
}

// REDC(x*y + u*v) = (x*y + u*v) * 2^-128 mod p, canonical, for x, u < p and
// y, v < 2^128: both products summed at full width (t < 2 p 2^128), ONE
// Montgomery reduction (result < 3p), two conditional subtracts.  48 mads
// instead of the 64 of two mont_mul; used for the Beaver cross terms
// D*[b] + E*[a] = (Db + Ea) R.
__host__ __device__ __forceinline__ W4 dot2_redc(const W4& x, const W4& y, const W4& u,
                                                const W4& v, const Fp& f) {
  uint32_t t[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // t = x * y
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c = mad32(x.v[i], y.v[j], (uint64_t)t[i + j] + (c >> 32));
      t[i + j] = (uint32_t)c;
    }
    t[i + 4] = (uint32_t)(c >> 32);
  }
  uint32_t top = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // t += u * v
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c = mad32(u.v[i], v.v[j], (uint64_t)t[i + j] + (c >> 32));
      t[i + j] = (uint32_t)c;
    }
    uint32_t cc;
    t[i + 4] = addc(t[i + 4], (uint32_t)(c >> 32), 0, &cc);
#pragma unroll
    for (int k = i + 5; k < 8; ++k) t[k] = addc(t[k], 0, cc, &cc);
    top += cc;
  }
  t[8] = top;
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // Montgomery reduction of the 258-bit sum
    const uint32_t m = t[i] * f.n0;
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      c = mad32(m, f.p[j], (uint64_t)t[i + j] + (c >> 32));
      t[i + j] = (uint32_t)c;
    }
    uint32_t cc;
    t[i + 4] = addc(t[i + 4], (uint32_t)(c >> 32), 0, &cc);
#pragma unroll
    for (int k = i + 5; k < 9; ++k) t[k] = addc(t[k], 0, cc, &cc);
  }
  W4 r = {{t[4], t[5], t[6], t[7]}};
  uint32_t hi = t[8];
#pragma unroll
  for (int s = 0; s < 2; ++s) {  // (hi:r) < 3p
    W4 d;
    const uint32_t b = sub_p(r, f, d);
    const bool ge = hi >= b;  // (hi:r) >= p: no borrow out of the top limb
    r = sel(ge, d, r);
    hi = ge ? hi - b : hi;
  }
  return r;
}

__host__ __device__ __forceinline__ W4 r2_word(const Fp& f) {
  return W4{{f.r2[0], f.r2[1], f.r2[2], f.r2[3]}};
}

// Any 128-bit word -> canonical representative in [0, p).
template <bool BIG>
__host__ __device__ __forceinline__ W4 canon(const W4& a, const Fp& f) {
  if constexpr (BIG) {
    return reduce_once(a, 0, f);
  } else {
    return redc(mont_mul(a, r2_word(f), f), f);
  }
}

}  // namespace amph

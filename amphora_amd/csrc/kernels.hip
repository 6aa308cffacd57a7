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

namespace amph {

// Every launch goes through hipExtLaunchKernelGGL: with the config's timing
// events set (amph_time_next_launch) the events are stamped by the kernel's
// own dispatch, i.e. they measure the kernel, not the queue gap before it.
#define AMPH_LAUNCH(K, G, B, C, ...) \
  hipExtLaunchKernelGGL(K, G, B, 0, (C).stream, (C).ev_start, (C).ev_stop, 0, __VA_ARGS__)

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Streamed-once inputs: nontemporal 16-byte loads (global_load_dwordx4 nt).
__device__ __forceinline__ uint4 ld(const uint4* p) {
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st(uint4* p, const W4& v) { *p = u4(v); }

// Wave-level reduction of the failing indices to one atomic per wave: the
// lowest set lane holds the smallest index of this iteration.
__device__ __forceinline__ void report_fail(bool bad, size_t i, unsigned long long* ff) {
  const unsigned long long m = __ballot(bad);
  if (m != 0ULL) {
    const int lane = __lane_id();
    if (lane == __ffsll((long long)m) - 1) atomicMin(ff, (unsigned long long)i);
  }
}

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
    if constexpr (WRITE_Y) st(out_y + i, redc(a[0], f));
    report_fail(!ok, ibase + i, ff);
  }
}

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
    st(out + i, mod_sub(mont_mul(w4(s), r2, f), a[0], f));
    report_fail(!ok, i, ff);
  }
}

template <int NP, bool BIG>
__global__ __launch_bounds__(kMaxBlock) void k_recombine(ShareSet sh, int n, size_t words,
                                                     uint4* out, Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride)
    st(out + i, redc(sum_field<NP, BIG>(sh.s, n, i, f), f));
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

template <bool BIG>
__global__ __launch_bounds__(kMaxBlock) void k_conv(const uint4* masked, const uint4* tuples,
                                                size_t words, W4 alpha, int use_zero,
                                                uint4* out, Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
    const uint4 mr = ld(masked + i), vr = ld(tuples + 2 * i), cr = ld(tuples + 2 * i + 1);
    const W4 m = canon<BIG>(w4(mr), f);
    const W4 val = canon<BIG>(w4(vr), f), mac = canon<BIG>(w4(cr), f);
    st(out + 2 * i, use_zero ? val : mod_add(val, m, f));
    st(out + 2 * i + 1, mod_add(mac, mont_mul(m, alpha, f), f));
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

__global__ __launch_bounds__(kMaxBlock) void k_odo_pre(const uint4* share_data, int stride_w,
                                                   const uint4* masks, const uint4* triples,
                                                   size_t words, uint4* oy, uint4* orr, uint4* ov,
                                                   uint4* omag, uint32_t* oneg, Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
    const uint4 yr = ld(share_data + (size_t)stride_w * i);
    const uint4 m1 = ld(masks + 4 * i), m2 = ld(masks + 4 * i + 2);
    const uint4* t0 = triples + 12 * i;  // triple 2i: a = t0[0], b = t0[2]
    const uint4 a0 = ld(t0), b0 = ld(t0 + 2), a1 = ld(t0 + 6), b1 = ld(t0 + 8);
    oy[i] = yr;
    orr[i] = m1;
    ov[i] = m2;
    const W4 Y = redc(w4(yr), f), M1 = redc(w4(m1), f), M2 = redc(w4(m2), f);
    W4 d0, e0, d1, e1;
    const uint32_t s0 = signed_diff(Y, redc(w4(a0), f), d0);
    const uint32_t s1 = signed_diff(M1, redc(w4(b0), f), e0);
    const uint32_t s2 = signed_diff(M2, redc(w4(a1), f), d1);
    const uint32_t s3 = signed_diff(M1, redc(w4(b1), f), e1);
    st(omag + 4 * i + 0, d0);
    st(omag + 4 * i + 1, e0);
    st(omag + 4 * i + 2, d1);
    st(omag + 4 * i + 3, e1);
    oneg[i] = s0 | (s1 << 8) | (s2 << 16) | (s3 << 24);
  }
}

template <int NP, bool BIG>
__global__ __launch_bounds__(kMaxBlock) void k_open(SignedSet d, int n, size_t words, uint4* out,
                                                Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const int np = NP > 0 ? NP : n;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
    W4 acc[4] = {};
    for (int j = 0; j < np; ++j) {
      const uint32_t s = d.neg[j][i];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const W4 m = canon<BIG>(w4(ld(d.mag[j] + 4 * i + c)), f);
        acc[c] = ((s >> (8 * c)) & 0xFF) ? mod_sub(acc[c], m, f) : mod_add(acc[c], m, f);
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) st(out + 4 * i + c, acc[c]);
  }
}

template <bool BIG>
__global__ __launch_bounds__(kMaxBlock) void k_odo_post(const uint4* opened, const uint4* triples,
                                                    size_t words, int p0, uint4* ow, uint4* ou,
                                                    Fp f) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const W4 r2 = r2_word(f);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
    W4 z[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint4* t = triples + 12 * i + 6 * h;
      const W4 a = w4(ld(t)), b = w4(ld(t + 2)), c = w4(ld(t + 4));
      const W4 D = mont_mul(w4(ld(opened + 4 * i + 2 * h)), r2, f);
      const W4 E = mont_mul(w4(ld(opened + 4 * i + 2 * h + 1)), r2, f);
      W4 acc = mod_add(canon<BIG>(c, f), mont_mul(D, b, f), f);
      acc = mod_add(acc, mont_mul(E, a, f), f);
      if (p0) acc = mod_add(acc, mont_mul(D, E, f), f);
      z[h] = acc;
    }
    st(ow + i, z[0]);
    st(ou + i, z[1]);
  }
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
#define AMPH_DISPATCH_NP(n, BIG, LAUNCH) \
  switch (n) {                           \
    case 1: LAUNCH(1, BIG); break;       \
    case 2: LAUNCH(2, BIG); break;       \
    case 3: LAUNCH(3, BIG); break;       \
    case 4: LAUNCH(4, BIG); break;       \
    default: LAUNCH(0, BIG); break;      \
  }

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
  const unsigned g = grid_for(words, c);
  if (f.big) AMPH_LAUNCH((k_conv<true>), dim3(g), dim3(c.block), c, masked, tuples, words, alpha, use_zero, out, f);
  else AMPH_LAUNCH((k_conv<false>), dim3(g), dim3(c.block), c, masked, tuples, words, alpha, use_zero, out, f);
  return hipGetLastError();
}

hipError_t launch_odo_pre(const uint4* share_data, int stride_w, const uint4* masks,
                          const uint4* triples, size_t words, uint4* oy, uint4* orr, uint4* ov,
                          uint4* omag, uint32_t* oneg, const Fp& f, const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  AMPH_LAUNCH(k_odo_pre, dim3(grid_for(words, c)), dim3(c.block), c, share_data,
                     stride_w, masks, triples, words, oy, orr, ov, omag, oneg, f);
  return hipGetLastError();
}

hipError_t launch_open_diffs(const SignedSet& d, int n, size_t words, uint4* out, const Fp& f,
                             const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  const unsigned g = grid_for(words, c);
#define L(NP, BIG) AMPH_LAUNCH((k_open<NP, BIG>), dim3(g), dim3(c.block), c, d, n, words, out, f)
  if (f.big) { AMPH_DISPATCH_NP(n, true, L) } else { AMPH_DISPATCH_NP(n, false, L) }
#undef L
  return hipGetLastError();
}

hipError_t launch_odo_post(const uint4* opened, const uint4* triples, size_t words, int p0,
                           uint4* ow, uint4* ou, const Fp& f, const LaunchCfg& c) {
  if (words == 0) return hipSuccess;
  const unsigned g = grid_for(words, c);
  if (f.big) AMPH_LAUNCH((k_odo_post<true>), dim3(g), dim3(c.block), c, opened, triples, words, p0, ow, ou, f);
  else AMPH_LAUNCH((k_odo_post<false>), dim3(g), dim3(c.block), c, opened, triples, words, p0, ow, ou, f);
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

hipError_t launch_synth_words(uint4* out, size_t count, uint64_t seed, const Fp& f,
                              const LaunchCfg& c) {
  if (count == 0) return hipSuccess;
  const unsigned g = grid_for(count, c);
  if (f.big) AMPH_LAUNCH((k_synth_words<true>), dim3(g), dim3(c.block), c, out, count, seed, f);
  else AMPH_LAUNCH((k_synth_words<false>), dim3(g), dim3(c.block), c, out, count, seed, f);
  return hipGetLastError();
}

}  // namespace amph

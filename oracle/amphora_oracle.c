/*
 * CPU oracle for Amphora's per-word secret-share arithmetic -- C restatement.
 *
 * TEST INFRASTRUCTURE ONLY.  The product library (libamphora_hip.so) never
 * links or calls this file.  It is used by tests/ as the checker at sizes the
 * pure-Python oracle (oracle/amphora_oracle.py) cannot reach quickly, by
 * __graft_entry__.smoke(), and as bench.py's cpu_baseline ("port").
 *
 * It restates the Java BigInteger algorithm of the reference, NOT the
 * Montgomery-domain shortcut the HIP kernels take:
 *   fromGfp(b) = (LEint(b) * rInv) mod p      (schoolbook 128x128 product +
 *   toGfp(x)   = LE16((x * r) mod p)           Knuth algorithm-D division,
 *                                              like BigInteger.multiply/mod)
 * so agreement between the two is an independent check of the kernels.
 *
 * Reference rows (paths relative to /root/reference):
 *   orc_recombine_verify  amphora-java-client/.../client/SecretShareUtil.java:53-141
 *                         + DefaultAmphoraClient.java:476-505
 *   orc_mask_input        DefaultAmphoraClient.java:150-160 + SecretShareUtil.java:65-68
 *   orc_convert_share     amphora-service/.../calculation/SecretShareUtil.java:58-107
 *   orc_odo_pre           amphora-service/.../calculation/OutputDeliveryService.java:75-139,186-200
 *   orc_odo_post          OutputDeliveryService.java:147-152,274-286
 *   orc_recombine_diffs   OutputDeliveryService.java:231-272
 * The third-party codec (mp-spdz-integration 0.2.2, absent) is restated as in
 * oracle/amphora_oracle.py (ENCODING "mont_le").  Requires 2^64 <= p < 2^128.
 *
 * Parallelism mirrors the reference's parallelStream over words: OpenMP
 * static schedule over the word index, `nthreads` threads.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <omp.h>

typedef unsigned __int128 u128;
typedef __int128 s128;
typedef uint64_t u64;

typedef struct orc_field {
  u128 p, r, rinv;
  u64 vn[2]; /* p << s, normalised divisor digits */
  int s;     /* normalisation shift */
} orc_field;

static u128 ld16(const uint8_t* b) {
  u64 lo, hi;
  memcpy(&lo, b, 8);
  memcpy(&hi, b + 8, 8);
  return ((u128)hi << 64) | lo;
}

static void st16(uint8_t* b, u128 x) {
  u64 lo = (u64)x, hi = (u64)(x >> 64);
  memcpy(b, &lo, 8);
  memcpy(b + 8, &hi, 8);
}

/* 256-bit (4 x 64-bit digits, little-endian) mod p: Knuth algorithm D with
 * 64-bit digits (Hacker's Delight divmnu, n = 2). */
static u128 mod256(const orc_field* f, const u64 x[4]) {
  u64 un[5];
  const int s = f->s;
  if (s == 0) {
    un[4] = 0; un[3] = x[3]; un[2] = x[2]; un[1] = x[1]; un[0] = x[0];
  } else {
    un[4] = x[3] >> (64 - s);
    un[3] = (x[3] << s) | (x[2] >> (64 - s));
    un[2] = (x[2] << s) | (x[1] >> (64 - s));
    un[1] = (x[1] << s) | (x[0] >> (64 - s));
    un[0] = x[0] << s;
  }
  const u64 v1 = f->vn[1], v0 = f->vn[0];
  const u128 B = (u128)1 << 64;
  for (int j = 2; j >= 0; --j) {
    u128 num = ((u128)un[j + 2] << 64) | un[j + 1];
    u128 qhat = num / v1;
    u128 rhat = num - qhat * v1;
    while (qhat >= B || qhat * v0 > ((rhat << 64) | un[j])) {
      qhat -= 1;
      rhat += v1;
      if (rhat >= B) break;
    }
    /* multiply and subtract */
    s128 k = 0, t;
    u128 prod = qhat * v0;
    t = (s128)un[j] - k - (s128)(u64)prod;
    un[j] = (u64)t;
    k = (s128)(prod >> 64) - (t >> 64);
    prod = qhat * v1;
    t = (s128)un[j + 1] - k - (s128)(u64)prod;
    un[j + 1] = (u64)t;
    k = (s128)(prod >> 64) - (t >> 64);
    t = (s128)un[j + 2] - k;
    un[j + 2] = (u64)t;
    if (t < 0) { /* add back */
      u128 c = (u128)un[j] + v0;
      un[j] = (u64)c;
      c = (u128)un[j + 1] + v1 + (u64)(c >> 64);
      un[j + 1] = (u64)c;
      un[j + 2] += (u64)(c >> 64);
    }
  }
  u64 r0, r1;
  if (s == 0) { r0 = un[0]; r1 = un[1]; }
  else { r0 = (un[0] >> s) | (un[1] << (64 - s)); r1 = un[1] >> s; }
  return ((u128)r1 << 64) | r0;
}

static void mul128(u128 a, u128 b, u64 out[4]) {
  u64 a0 = (u64)a, a1 = (u64)(a >> 64), b0 = (u64)b, b1 = (u64)(b >> 64);
  u128 p00 = (u128)a0 * b0, p01 = (u128)a0 * b1, p10 = (u128)a1 * b0, p11 = (u128)a1 * b1;
  u128 mid = (p00 >> 64) + (u64)p01 + (u64)p10;
  out[0] = (u64)p00;
  out[1] = (u64)mid;
  u128 hi = (mid >> 64) + (p01 >> 64) + (p10 >> 64) + (u64)p11;
  out[2] = (u64)hi;
  out[3] = (u64)((hi >> 64) + (p11 >> 64));
}

static u128 mulmod(const orc_field* f, u128 a, u128 b) {
  u64 t[4];
  mul128(a, b, t);
  return mod256(f, t);
}

static u128 mod128(const orc_field* f, u128 a) {
  u64 t[4] = {(u64)a, (u64)(a >> 64), 0, 0};
  return mod256(f, t);
}

static u128 addmod(const orc_field* f, u128 a, u128 b) { /* a, b < p */
  u128 s = a + b;
  if (s < a || s >= f->p) s -= f->p;
  return s;
}

static u128 submod(const orc_field* f, u128 a, u128 b) { /* a, b < p */
  return a >= b ? a - b : a + (f->p - b);
}

/* MpSpdzIntegrationUtils.fromGfp / toGfp (restated) */
static u128 from_gfp(const orc_field* f, const uint8_t* b) { return mulmod(f, ld16(b), f->rinv); }
static void to_gfp(const orc_field* f, u128 x, uint8_t* out) { st16(out, mulmod(f, x, f->r)); }

int orc_field_init(orc_field* f, const uint8_t p[16], const uint8_t r[16], const uint8_t rinv[16]) {
  f->p = ld16(p);
  f->r = ld16(r);
  f->rinv = ld16(rinv);
  if ((f->p >> 64) == 0 || (f->p & 1) == 0) return -1;
  u64 hi = (u64)(f->p >> 64);
  int s = __builtin_clzll(hi);
  f->s = s;
  u128 pn = f->p << s;
  f->vn[0] = (u64)pn;
  f->vn[1] = (u64)(pn >> 64);
  if (mulmod(f, f->r, f->rinv) != 1) return -2;
  return 0;
}

/* Heap-allocated field (malloc gives the 16-byte alignment u128 needs). */
orc_field* orc_field_new(const uint8_t p[16], const uint8_t r[16], const uint8_t rinv[16],
                         int* status) {
  orc_field* f = (orc_field*)malloc(sizeof(orc_field));
  *status = f ? orc_field_init(f, p, r, rinv) : -3;
  return f;
}

void orc_field_free(orc_field* f) { free(f); }

/* recombineObject for one field: sum_j fromGfp(share_j[i]) as a BigInteger,
 * then mod p (summingGfpAsBigInteger :53-63). */
static u128 recombine_word(const orc_field* f, int n, const uint8_t* const* sh, size_t i) {
  u64 acc[4] = {0, 0, 0, 0};
  for (int j = 0; j < n; ++j) {
    u128 v = from_gfp(f, sh[j] + 16 * i);
    u128 lo = ((u128)acc[1] << 64) | acc[0];
    u128 s = lo + v;
    acc[2] += (s < lo);
    acc[0] = (u64)s;
    acc[1] = (u64)(s >> 64);
  }
  return mod256(f, acc);
}

void orc_recombine(const orc_field* f, int n, const uint8_t* const* shares, size_t W,
                   uint8_t* out16, int nthreads) {
#pragma omp parallel for schedule(static) num_threads(nthreads)
  for (size_t i = 0; i < W; ++i) st16(out16 + 16 * i, recombine_word(f, n, shares, i));
}

/* verifyOutputDeliveryObjects :476-505 -> canonical secrets; min failing index
 * (or -1).  Field arrays: odo[5][n] = {y, r, v, w, u} x parties. */
static int64_t recombine_verify_core(const orc_field* f, int n, const uint8_t* const* y,
                                     const uint8_t* const* r, const uint8_t* const* v,
                                     const uint8_t* const* w, const uint8_t* const* u, size_t W,
                                     uint8_t* ys16, int nthreads) {
  int64_t first = INT64_MAX;
#pragma omp parallel for schedule(static) num_threads(nthreads) reduction(min : first)
  for (size_t i = 0; i < W; ++i) {
    u128 sy = recombine_word(f, n, y, i), sr = recombine_word(f, n, r, i);
    u128 sv = recombine_word(f, n, v, i), sw = recombine_word(f, n, w, i);
    u128 su = recombine_word(f, n, u, i);
    st16(ys16 + 16 * i, sy);
    u128 aw = mulmod(f, sy, sr), au = mulmod(f, sv, sr);
    if (aw != sw || au != su) {
      if ((int64_t)i < first) first = (int64_t)i;
    }
  }
  return first == INT64_MAX ? -1 : first;
}

int64_t orc_recombine_verify(const orc_field* f, int n, const uint8_t* const* y,
                             const uint8_t* const* r, const uint8_t* const* v,
                             const uint8_t* const* w, const uint8_t* const* u, size_t W,
                             uint8_t* out_y16, int nthreads) {
  return recombine_verify_core(f, n, y, r, v, w, u, W, out_y16, nthreads);
}

/* createSecret :150-160: verify the mask ODOs, then
 * masked_i = toGfp((s_i - m_i) mod p).  secrets16: canonical LE16 ints. */
int64_t orc_mask_input(const orc_field* f, int n, const uint8_t* const* y,
                       const uint8_t* const* r, const uint8_t* const* v,
                       const uint8_t* const* w, const uint8_t* const* u,
                       const uint8_t* secrets16, size_t W, uint8_t* out16, int nthreads) {
  int64_t ff = recombine_verify_core(f, n, y, r, v, w, u, W, out16, nthreads);
#pragma omp parallel for schedule(static) num_threads(nthreads)
  for (size_t i = 0; i < W; ++i) {
    u128 s = mod128(f, ld16(secrets16 + 16 * i));
    to_gfp(f, submod(f, s, ld16(out16 + 16 * i)), out16 + 16 * i);
  }
  return ff;
}

/* convertToSecretShare :58-107.  alpha16: the MAC key as a canonical int.
 * tuples32: value || mac of share 0 per input mask. */
void orc_convert_share(const orc_field* f, const uint8_t* masked16, const uint8_t* tuples32,
                       const uint8_t* alpha16, int use_zero_input, size_t W, uint8_t* out32,
                       int nthreads) {
  const u128 key = mod128(f, ld16(alpha16));
#pragma omp parallel for schedule(static) num_threads(nthreads)
  for (size_t i = 0; i < W; ++i) {
    u128 pub = from_gfp(f, masked16 + 16 * i);
    u128 ind = use_zero_input ? 0 : pub;
    u128 sv = from_gfp(f, tuples32 + 32 * i);
    u128 sm = from_gfp(f, tuples32 + 32 * i + 16);
    to_gfp(f, addmod(f, sv, ind), out32 + 32 * i);
    to_gfp(f, addmod(f, sm, mulmod(f, key, pub)), out32 + 32 * i + 16);
  }
}

/* diff = x - a as a signed BigInteger: magnitude LE16 + negative flag. */
static void put_diff(u128 x, u128 a, uint8_t* mag, uint8_t* neg) {
  if (x >= a) { st16(mag, x - a); *neg = 0; }
  else { st16(mag, a - x); *neg = 1; }
}

/* computeOutputDeliveryObject(SecretShare|byte[]) :75-139 + multiplyShares
 * diffs :186-200.  share_stride = 32 (SecretShare.data, MACs stripped :79-84)
 * or 16 (raw word array, e.g. InputMaskCachingService :81-91).
 * Outputs raw y/r/v copies and, per pair k (k = 2i: (y_i, r_i); k = 2i+1:
 * (v_i, r_i)), d_k = x_k - a_k and e_k = y_k - b_k as sign+magnitude, in the
 * FactorPair order [d_0, e_0, d_1, e_1, ...]. */
void orc_odo_pre(const orc_field* f, const uint8_t* share_data, int share_stride,
                 const uint8_t* masks32, const uint8_t* triples96, size_t W, uint8_t* y16,
                 uint8_t* r16, uint8_t* v16, uint8_t* diff_mag, uint8_t* diff_neg, int nthreads) {
#pragma omp parallel for schedule(static) num_threads(nthreads)
  for (size_t i = 0; i < W; ++i) {
    const uint8_t* ys = share_data + (size_t)share_stride * i;
    const uint8_t* m1 = masks32 + 32 * (2 * i);
    const uint8_t* m2 = masks32 + 32 * (2 * i + 1);
    memcpy(y16 + 16 * i, ys, 16);
    memcpy(r16 + 16 * i, m1, 16);
    memcpy(v16 + 16 * i, m2, 16);
    u128 yb = from_gfp(f, ys), m1b = from_gfp(f, m1), m2b = from_gfp(f, m2);
    const uint8_t* t0 = triples96 + 96 * (2 * i);
    const uint8_t* t1 = triples96 + 96 * (2 * i + 1);
    size_t k0 = 2 * i, k1 = 2 * i + 1;
    put_diff(yb, from_gfp(f, t0), diff_mag + 32 * k0, diff_neg + 2 * k0);
    put_diff(m1b, from_gfp(f, t0 + 32), diff_mag + 32 * k0 + 16, diff_neg + 2 * k0 + 1);
    put_diff(m2b, from_gfp(f, t1), diff_mag + 32 * k1, diff_neg + 2 * k1);
    put_diff(m1b, from_gfp(f, t1 + 32), diff_mag + 32 * k1 + 16, diff_neg + 2 * k1 + 1);
  }
}

/* recombineDiffs :231-272 for canonical output: sum over parties of the
 * signed diffs, mod p.  mags/negs: n party arrays as produced by orc_odo_pre.
 * (With n == 1 Java keeps the raw signed value; its use in
 * multiplySharedSecrets is mod p, so the canonical form is equivalent.) */
void orc_recombine_diffs(const orc_field* f, int n, const uint8_t* const* mags,
                         const uint8_t* const* negs, size_t n_values, uint8_t* out16,
                         int nthreads) {
#pragma omp parallel for schedule(static) num_threads(nthreads)
  for (size_t k = 0; k < n_values; ++k) {
    u128 acc = 0;
    for (int j = 0; j < n; ++j) {
      u128 m = mod128(f, ld16(mags[j] + 16 * k));
      acc = negs[j][k] ? submod(f, acc, m) : addmod(f, acc, m);
    }
    st16(out16 + 16 * k, acc);
  }
}

/* multiplySharedSecrets :274-286 + toGfp of the products :147-152.
 * opened16: canonical [D_0, E_0, D_1, E_1, ...] (2 values per pair). */
void orc_odo_post(const orc_field* f, const uint8_t* opened16, const uint8_t* triples96,
                  int is_player0, size_t W, uint8_t* w16, uint8_t* u16, int nthreads) {
#pragma omp parallel for schedule(static) num_threads(nthreads)
  for (size_t k = 0; k < 2 * W; ++k) {
    const uint8_t* t = triples96 + 96 * k;
    u128 d = mod128(f, ld16(opened16 + 32 * k)), e = mod128(f, ld16(opened16 + 32 * k + 16));
    u128 a = from_gfp(f, t), b = from_gfp(f, t + 32), c = from_gfp(f, t + 64);
    u128 z = addmod(f, addmod(f, c, mulmod(f, d, b)), mulmod(f, e, a));
    if (is_player0) z = addmod(f, z, mulmod(f, d, e));
    to_gfp(f, z, (k & 1) ? u16 + 16 * (k >> 1) : w16 + 16 * (k >> 1));
  }
}

/* ---------------------------------------------------------------------- */
/* Synthetic honest inputs -- used by tests to build inputs at
 * sizes the Python oracle is too slow for.  Counter-based, so the output is
 * independent of the thread count. */
static u64 splitmix64(u64 x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

static u128 rand_fe(const orc_field* f, u64 seed, u64 ctr) {
  u64 a = splitmix64(seed ^ splitmix64(2 * ctr)), b = splitmix64(seed ^ splitmix64(2 * ctr + 1));
  return mod128(f, ((u128)a << 64) | b);
}

/* Honest ODOs for n parties: per word y, r, v uniform, w = y r, u = v r;
 * each additively shared (n-1 uniform shares, last = x - sum) and toGfp'd.
 * odo[field][party] with field order y, r, v, w, u.  If y_plain != NULL the
 * y values are taken from it (canonical LE16) instead of drawn.
 * fault_index >= 0: party (n > 1 ? 1 : 0)'s w share at that index gets +1.
 * noncanon_permille: that many of every 1000 raw words (chosen by hash) are
 * written as [x] + p when that still fits in 128 bits. */
void orc_synth_odos(const orc_field* f, u64 seed, int n, size_t W, uint8_t* const* odo,
                    const uint8_t* y_plain, int64_t fault_index, int noncanon_permille,
                    int nthreads) {
#pragma omp parallel for schedule(static) num_threads(nthreads)
  for (size_t i = 0; i < W; ++i) {
    u64 base = (u64)i * 64;
    u128 val[5];
    val[0] = y_plain ? mod128(f, ld16(y_plain + 16 * i)) : rand_fe(f, seed, base + 0);
    val[1] = rand_fe(f, seed, base + 1);
    val[2] = rand_fe(f, seed, base + 2);
    val[3] = mulmod(f, val[0], val[1]);
    val[4] = mulmod(f, val[2], val[1]);
    for (int fl = 0; fl < 5; ++fl) {
      u128 rest = val[fl];
      for (int j = 0; j < n; ++j) {
        u128 sh;
        if (j < n - 1) {
          sh = rand_fe(f, seed, base + 8 + (u64)fl * 8 + (u64)j);
          rest = submod(f, rest, sh);
        } else {
          sh = rest;
        }
        if (fl == 3 && (int64_t)i == fault_index && j == (n > 1 ? 1 : 0)) sh = addmod(f, sh, 1);
        u128 mont = mulmod(f, sh, f->r);
        if (noncanon_permille > 0) {
          u64 h = splitmix64(seed ^ splitmix64(base + 48 + (u64)fl * 8 + (u64)j));
          if ((int)(h % 1000) < noncanon_permille && mont + f->p > mont) mont += f->p;
        }
        st16(odo[fl * n + j] + 16 * i, mont);
      }
    }
  }
}

/* Uniform raw words (canonical field elements in Montgomery LE16 form), for
 * tuple streams and secrets. */
void orc_synth_words(const orc_field* f, u64 seed, size_t count, uint8_t* out16, int mont,
                     int nthreads) {
#pragma omp parallel for schedule(static) num_threads(nthreads)
  for (size_t i = 0; i < count; ++i) {
    u128 x = rand_fe(f, seed, i);
    st16(out16 + 16 * i, mont ? mulmod(f, x, f->r) : x);
  }
}

int orc_max_threads(void) { return omp_get_max_threads(); }

/* Drives the C oracle (test infrastructure) under ASan/UBSan on the CPU:
 * synthetic ODOs for 1..4 parties with faults and non-canonical words,
 * recombine+verify, masking, share conversion and the ODO party steps.
 * Built by tests/test_sanitizers.py; exit 0 = clean and self-consistent. */
#include "../../oracle/amphora_oracle.c"

#include <stdio.h>

static void le(u128 x, uint8_t* o) { memcpy(o, &x, 16); }

int main(void) {
  const u128 P = ((u128)0x958907458f213686ULL << 64) | 0x1bd7554a24340001ULL;
  const u128 RI = ((u128)0x64b363aaebadc239ULL << 64) | 0xc970b543e5633b46ULL;
  const u128 R = (0 - P) % P; /* 2^128 mod p */
  uint8_t p[16], r[16], ri[16];
  le(P, p); le(R, r); le(RI, ri);
  int st = 0;
  orc_field* f = orc_field_new(p, r, ri, &st);
  if (!f || st) { fprintf(stderr, "field init failed\n"); return 1; }
  const size_t W = 3001;
  for (int n = 1; n <= 4; ++n) {
    uint8_t* bufs = malloc(5 * (size_t)n * W * 16);
    uint8_t* ptr[5 * 4];
    for (int i = 0; i < 5 * n; ++i) ptr[i] = bufs + (size_t)i * W * 16;
    orc_synth_odos(f, 7 + n, n, W, ptr, NULL, (int64_t)(W / 2), 50, 2);
    const uint8_t* const* fl[5];
    for (int k = 0; k < 5; ++k) fl[k] = (const uint8_t* const*)(ptr + k * n);
    uint8_t *y = malloc(W * 16), *sec = malloc(W * 16);
    int64_t ff = orc_recombine_verify(f, n, fl[0], fl[1], fl[2], fl[3], fl[4], W, y, 2);
    if (ff != (int64_t)(W / 2)) { fprintf(stderr, "n=%d ff=%lld\n", n, (long long)ff); return 1; }
    orc_synth_words(f, 9, W, sec, 0, 2);
    ff = orc_mask_input(f, n, fl[0], fl[1], fl[2], fl[3], fl[4], sec, W, y, 2);
    if (ff != (int64_t)(W / 2)) { fprintf(stderr, "mask n=%d ff=%lld\n", n, (long long)ff); return 1; }
    free(bufs); free(y); free(sec);
  }
  uint8_t *m = malloc(W * 16), *t = malloc(W * 32), *o = malloc(W * 32), key[16];
  orc_synth_words(f, 1, W, m, 1, 2);
  orc_synth_words(f, 2, 2 * W, t, 1, 2);
  le(12345, key);
  orc_convert_share(f, m, t, key, 0, W, o, 2);
  uint8_t *masks = malloc(2 * W * 32), *tr = malloc(2 * W * 96);
  orc_synth_words(f, 3, 4 * W, masks, 1, 2);
  orc_synth_words(f, 4, 12 * W, tr, 1, 2);
  uint8_t *yy = malloc(W * 16), *rr = malloc(W * 16), *vv = malloc(W * 16);
  uint8_t *mag = malloc(W * 64), *neg = malloc(W * 4), *op = malloc(W * 64);
  orc_odo_pre(f, o, 32, masks, tr, W, yy, rr, vv, mag, neg, 2);
  const uint8_t* mags[1] = {mag};
  const uint8_t* negs[1] = {neg};
  orc_recombine_diffs(f, 1, mags, negs, 4 * W, op, 2);
  uint8_t *w = malloc(W * 16), *u = malloc(W * 16);
  orc_odo_post(f, op, tr, 1, W, w, u, 2);
  uint8_t *w2 = malloc(W * 16), *u2 = malloc(W * 16);
  orc_odo_post(f, op, tr, 1, W, w2, u2, 1);
  if (memcmp(w, w2, W * 16) || memcmp(u, u2, W * 16)) { fprintf(stderr, "odo_post nondeterministic\n"); return 1; }
  free(m); free(t); free(o); free(masks); free(tr); free(yy); free(rr); free(vv); free(mag);
  free(neg); free(op); free(w); free(u); free(w2); free(u2);
  orc_field_free(f);
  puts("oracle sanitize: clean");
  return 0;
}

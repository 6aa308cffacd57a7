/* JNI-independent core of libamphora_jni (see amphora_jni_core.h). */
#include "amphora_jni_core.h"

#include <stdio.h>
#include <string.h>

static __thread char g_msg[1024];
/* AMPH_F_HOST_IO for this thread's next calls (amphj_set_host_io) */
static __thread uint32_t g_io;

void amphj_set_host_io(int on) { g_io = on ? AMPH_F_HOST_IO : 0u; }

static int set_msg(int status, const char* msg) {
  snprintf(g_msg, sizeof g_msg, "%s", msg);
  return status;
}

/* a libamphora_hip failure: keep its detail */
static int abi(int status) {
  if (status != AMPH_OK && status != AMPH_E_VERIFY) set_msg(status, amph_last_error());
  else g_msg[0] = 0;
  return status;
}

const char* amphj_message(void) { return g_msg; }

const char* amphj_exception_class(int status) {
  switch (status) {
    case AMPH_OK: return NULL;
    /* SecretShareUtil.verifySecrets :116-129 */
    case AMPH_E_VERIFY: return "io/carbynestack/amphora/common/exceptions/IntegrityVerificationException";
    /* OutputDeliveryObject.java:90-96, service SecretShareUtil.java:64-66, Jackson input errors */
    case AMPH_E_LEN:
    case AMPH_E_PARAM: return "java/lang/IllegalArgumentException";
    /* recombineObject's Arrays.copyOfRange past a shorter party's end (SecretShareUtil.java:87-88) */
    case AMPH_E_RANGE: return "java/lang/ArrayIndexOutOfBoundsException";
    default: return "java/lang/IllegalStateException"; /* HIP runtime / allocation */
  }
}

static const char kSameLength[] = "The provided shares must be of the same length";

/* n parties x 5 fields: the five arrays of one party have one length (the
 * OutputDeliveryObject constructor's invariant, OutputDeliveryObject.java:
 * 90-96); parties may differ -- recombineObject's semantics (word count from
 * party 0, ragged partners cut / zero-padded / ArrayIndexOutOfBounds) are
 * libamphora_hip's (include/amphora.h amph_odo).  *words = party 0's words. */
static int odo_lengths(int n, const size_t* lens, size_t* words) {
  if (n < 1 || n > AMPH_MAX_PARTIES) return set_msg(AMPH_E_PARAM, "n_parties must be in [1, 16]");
  for (int k = 1; k < 5; ++k)
    for (int j = 0; j < n; ++j)
      if (lens[k * n + j] != lens[j]) return set_msg(AMPH_E_LEN, kSameLength);
  *words = lens[0] / AMPH_WORD_WIDTH;
  return AMPH_OK;
}

/* base64 field texts: the wire entry points take one word count for every
 * text (amph_odo_b64), so all 5 n texts must have one length */
static int text_lengths(int n, const size_t* lens) {
  if (n < 1 || n > AMPH_MAX_PARTIES) return set_msg(AMPH_E_PARAM, "n_parties must be in [1, 16]");
  for (int i = 1; i < 5 * n; ++i)
    if (lens[i] != lens[0]) return set_msg(AMPH_E_LEN, kSameLength);
  return AMPH_OK;
}

static int room(size_t have, size_t need, const char* what) {
  if (have >= need) return AMPH_OK;
  char m[256];
  snprintf(m, sizeof m, "%s holds %zu bytes, %zu needed", what, have, need);
  return set_msg(AMPH_E_LEN, m);
}

int amphj_ctx_create(const uint8_t* p_le, size_t p_len, const uint8_t* r_le, size_t r_len,
                     const uint8_t* rinv_le, size_t rinv_len, const int* devices, int ndev, void** ctx) {
  if (p_len != 16 || r_len != 16 || rinv_len != 16)
    return set_msg(AMPH_E_PARAM, "prime, r and rInv must be 16-byte little-endian integers");
  amph_ctx* c = NULL;
  const int dev0 = 0;
  int st = ndev > 0 ? amph_ctx_create_multi(p_le, r_le, rinv_le, devices, ndev, &c)
                    : amph_ctx_create(p_le, r_le, rinv_le, dev0, &c);
  *ctx = c;
  return abi(st);
}

void amphj_ctx_destroy(void* ctx) { amph_ctx_destroy((amph_ctx*)ctx); }

static void odo_structs(int n, const uint8_t* const* fields, const size_t* lens, amph_odo* odos) {
  for (int j = 0; j < n; ++j) {
    odos[j].secret_shares = fields[0 * n + j];
    odos[j].r_shares = fields[1 * n + j];
    odos[j].v_shares = fields[2 * n + j];
    odos[j].w_shares = fields[3 * n + j];
    odos[j].u_shares = fields[4 * n + j];
    odos[j].nbytes = lens[j]; /* party j's own length */
  }
}

int amphj_recombine_verify(void* ctx, int n, const uint8_t* const* fields, const size_t* lens,
                           uint8_t* out, size_t out_len, int64_t* fail) {
  size_t W;
  *fail = -1;
  const int lst = odo_lengths(n, lens, &W);
  if (lst) return lst;
  if (room(out_len, 16 * W, "the secrets array")) return AMPH_E_LEN;
  amph_odo odos[AMPH_MAX_PARTIES];
  odo_structs(n, fields, lens, odos);
  return abi(amph_recombine_verify((amph_ctx*)ctx, odos, n, out, fail, g_io, NULL));
}

int amphj_mask_input(void* ctx, int n, const uint8_t* const* fields, const size_t* lens,
                     const uint8_t* secrets, size_t secrets_len, uint8_t* out, size_t out_len,
                     int64_t* fail) {
  size_t W;
  *fail = -1;
  const int lst = odo_lengths(n, lens, &W);
  if (lst) return lst;
  const size_t S = secrets_len / 16;
  if (room(out_len, 16 * S, "the masked-input array")) return AMPH_E_LEN;
  amph_odo odos[AMPH_MAX_PARTIES];
  odo_structs(n, fields, lens, odos);
  return abi(amph_mask_input((amph_ctx*)ctx, odos, n, secrets, S, out, fail, g_io, NULL));
}

int amphj_recombine(void* ctx, int n, const uint8_t* const* shares, const size_t* lens, uint8_t* out,
                    size_t out_len) {
  if (n < 1 || n > AMPH_MAX_PARTIES) return set_msg(AMPH_E_PARAM, "n_parties must be in [1, 16]");
  const size_t W = lens[0] / 16;  /* recombineObject: shares.get(0).length / WORD_WIDTH */
  if (room(out_len, 16 * W, "the output array")) return AMPH_E_LEN;
  /* ragged partners: cut / zero-padded / ArrayIndexOutOfBounds, as copyOfRange (:87-88) */
  return abi(amph_recombine_object((amph_ctx*)ctx, shares, n, lens, out, g_io, NULL));
}

int amphj_verify(void* ctx, const uint8_t* const* a, const size_t* lens, int64_t* fail) {
  *fail = -1;
  for (int k = 1; k < 5; ++k)
    if (lens[k] != lens[0]) return set_msg(AMPH_E_LEN, "verifySecrets: lists of unequal size");
  return abi(amph_verify((amph_ctx*)ctx, a[0], a[1], a[2], a[3], a[4], lens[0] / 16, fail, g_io, NULL));
}

int amphj_mask_words(void* ctx, const uint8_t* secrets, size_t s_len, const uint8_t* masks, size_t m_len,
                     uint8_t* out, size_t out_len) {
  const size_t W = s_len / 16;
  if (m_len / 16 != W) return set_msg(AMPH_E_LEN, "one input mask per secret word");
  if (room(out_len, 16 * W, "the output array")) return AMPH_E_LEN;
  return abi(amph_mask_words((amph_ctx*)ctx, secrets, masks, W, out, g_io, NULL));
}

int amphj_mask_word(void* ctx, const uint8_t secret[16], const uint8_t mask[16], uint8_t out[16]) {
  return abi(amph_mask_word_host((amph_ctx*)ctx, secret, mask, out));
}

int amphj_verify_message(void* ctx, const uint8_t* y, const uint8_t* r, const uint8_t* u,
                         const uint8_t* v, const uint8_t* w, char* buf, size_t cap) {
  const int len = amph_verify_message((amph_ctx*)ctx, y, r, u, v, w, buf, cap);
  return len < 0 ? abi(-len) : AMPH_OK;
}

static int text_structs(int n, const char* const* texts, const size_t* lens, amph_odo_b64* odos) {
  const int lst = text_lengths(n, lens);
  if (lst) return lst;
  for (int j = 0; j < n; ++j) {
    odos[j].secret_shares = texts[0 * n + j];
    odos[j].r_shares = texts[1 * n + j];
    odos[j].v_shares = texts[2 * n + j];
    odos[j].w_shares = texts[3 * n + j];
    odos[j].u_shares = texts[4 * n + j];
    odos[j].nchars = lens[0];
  }
  return AMPH_OK;
}

int amphj_recombine_verify_b64(void* ctx, int n, const char* const* texts, const size_t* lens,
                               size_t words, uint8_t* out, size_t out_len, int64_t* fail) {
  *fail = -1;
  amph_odo_b64 odos[AMPH_MAX_PARTIES];
  const int tst = text_structs(n, texts, lens, odos);
  if (tst) return tst;
  if (room(out_len, 16 * words, "the secrets array")) return AMPH_E_LEN;
  int64_t bad = -1;
  return abi(amph_recombine_verify_b64((amph_ctx*)ctx, odos, n, words, out, fail, &bad, 0, NULL));
}

int amphj_mask_input_b64(void* ctx, int n, const char* const* texts, const size_t* lens, size_t words,
                         const uint8_t* secrets, size_t secrets_len, char* records24,
                         size_t records_len, int64_t* fail) {
  *fail = -1;
  amph_odo_b64 odos[AMPH_MAX_PARTIES];
  const int tst = text_structs(n, texts, lens, odos);
  if (tst) return tst;
  const size_t S = secrets_len / 16;
  if (room(records_len, 24 * S, "the record array")) return AMPH_E_LEN;
  int64_t bad = -1;
  return abi(amph_mask_input_b64((amph_ctx*)ctx, odos, n, words, secrets, S, NULL, records24, fail, &bad, 0,
                                 NULL));
}

int amphj_convert_share(void* ctx, const uint8_t* masked, size_t masked_len, const uint8_t* tuples,
                        size_t tuples_len, const uint8_t* mac_key_le, size_t key_len, int use_zero_input_as_data,
                        uint8_t* out, size_t out_len) {
  const size_t W = masked_len / 16;
  /* service SecretShareUtil.java:64-66 (isTrue -> IllegalArgumentException) */
  if (tuples_len / AMPH_INPUT_MASK_TUPLE_SIZE != W)
    return set_msg(AMPH_E_LEN, "Received more input data than available inputMasks.");
  if (key_len != 16) return set_msg(AMPH_E_PARAM, "the MAC key must be a 16-byte little-endian integer");
  if (room(out_len, 32 * W, "the share array")) return AMPH_E_LEN;
  return abi(amph_convert_share((amph_ctx*)ctx, masked, tuples, W, mac_key_le, use_zero_input_as_data, out, g_io, NULL));
}

int amphj_odo_pre(void* ctx, const uint8_t* share, size_t share_len, int stride, const uint8_t* masks,
                  size_t masks_len, const uint8_t* triples, size_t triples_len, uint8_t* y, uint8_t* r,
                  uint8_t* v, size_t out_len, uint8_t* mag, size_t mag_len, uint8_t* neg, size_t neg_len) {
  if (stride != 16 && stride != 32) return set_msg(AMPH_E_PARAM, "share stride must be 16 or 32");
  const size_t W = share_len / (size_t)stride;
  /* castor delivers exactly 2W input masks and 2W triples (OutputDeliveryService.java:103-107,140-146) */
  if (room(masks_len, 2 * W * AMPH_INPUT_MASK_TUPLE_SIZE, "the input-mask stream") ||
      room(triples_len, 2 * W * AMPH_TRIPLE_TUPLE_SIZE, "the triple stream") ||
      room(out_len, 16 * W, "an ODO field array") || room(mag_len, 64 * W, "the diff magnitudes") ||
      room(neg_len, 4 * W, "the diff signs"))
    return AMPH_E_LEN;
  return abi(amph_odo_pre((amph_ctx*)ctx, share, (size_t)stride, masks, triples, W, y, r, v, mag, neg, g_io,
                          NULL));
}

int amphj_open_post(void* ctx, int n, const uint8_t* const* mags, const size_t* mag_lens,
                    const uint8_t* const* negs, const size_t* neg_lens, const uint8_t* triples,
                    size_t triples_len, int is_player0, uint8_t* w, uint8_t* u, size_t out_len) {
  if (n < 1 || n > AMPH_MAX_PARTIES) return set_msg(AMPH_E_PARAM, "n_parties must be in [1, 16]");
  const size_t W = triples_len / (2 * AMPH_TRIPLE_TUPLE_SIZE);
  for (int j = 0; j < n; ++j)
    if (room(mag_lens[j], 64 * W, "a party's diff magnitudes") || room(neg_lens[j], 4 * W, "a party's diff signs"))
      return AMPH_E_LEN;
  if (room(out_len, 16 * W, "an ODO field array")) return AMPH_E_LEN;
  return abi(amph_open_post((amph_ctx*)ctx, mags, negs, n, triples, W, is_player0, w, u, g_io, NULL));
}

size_t amphj_exchange_max_chars(size_t npairs) { return amph_exchange_max_chars(npairs); }

int amphj_exchange_encode(void* ctx, const uint8_t* mag, size_t mag_len, const uint8_t* neg, size_t neg_len,
                          char* out, size_t out_cap, uint64_t* out_len) {
  const size_t P = mag_len / 32;
  if (room(neg_len, 2 * P, "the diff signs")) return AMPH_E_LEN;
  return abi(amph_exchange_encode((amph_ctx*)ctx, mag, neg, P, out, out_cap, out_len, 0, NULL));
}

int amphj_exchange_decode(void* ctx, const char* text, size_t len, size_t npairs, uint8_t* mag, size_t mag_len,
                          uint8_t* neg, size_t neg_len) {
  if (room(mag_len, 32 * npairs, "the diff magnitudes") || room(neg_len, 2 * npairs, "the diff signs"))
    return AMPH_E_LEN;
  int64_t bad = -1;
  return abi(amph_exchange_decode((amph_ctx*)ctx, text, len, npairs, mag, neg, &bad, 0, NULL));
}

/* ---- one request's Output Delivery, device-resident between steps ---------------- */
int amphj_party_begin(void* ctx, const uint8_t* share, size_t share_len, int stride, const uint8_t* masks,
                      size_t masks_len, const uint8_t* triples, size_t triples_len, int n_parties, uint8_t* y,
                      uint8_t* r, uint8_t* v, size_t out_len, void** session) {
  *session = NULL;
  if (stride != 16 && stride != 32) return set_msg(AMPH_E_PARAM, "share stride must be 16 or 32");
  if (n_parties < 1 || n_parties > AMPH_MAX_PARTIES) return set_msg(AMPH_E_PARAM, "n_parties must be in [1, 16]");
  const size_t W = share_len / (size_t)stride;
  /* castor delivers exactly 2W input masks and 2W triples (OutputDeliveryService.java:103-107,140-146) */
  if (room(masks_len, 2 * W * AMPH_INPUT_MASK_TUPLE_SIZE, "the input-mask stream") ||
      room(triples_len, 2 * W * AMPH_TRIPLE_TUPLE_SIZE, "the triple stream"))
    return AMPH_E_LEN;
  if ((y || r || v) && (!y || !r || !v)) return set_msg(AMPH_E_PARAM, "y, r and v are all given or all null");
  if (y && room(out_len, 16 * W, "an ODO field array")) return AMPH_E_LEN;
  amph_party* p = NULL;
  const int st = abi(amph_party_begin((amph_ctx*)ctx, share, (size_t)stride, masks, triples, W, n_parties, y, r, v,
                                      &p));
  *session = p;
  return st;
}

uint64_t amphj_party_text_len(void* session) { return amph_party_text_len((const amph_party*)session); }

int amphj_party_text(void* session, char* out, size_t out_len) {
  if (!session) return set_msg(AMPH_E_PARAM, "null party session");
  return abi(amph_party_text((amph_party*)session, out, out_len));
}

int amphj_party_partner(void* session, int slot, const char* text, size_t len) {
  if (!session) return set_msg(AMPH_E_PARAM, "null party session");
  int64_t bad = -1;
  return abi(amph_party_partner((amph_party*)session, slot, text, len, &bad));
}

int amphj_party_finish(void* session, int is_player0, uint8_t* w, uint8_t* u, size_t out_len) {
  if (!session) return set_msg(AMPH_E_PARAM, "null party session");
  if (room(out_len, 16 * amph_party_words((const amph_party*)session), "an ODO field array")) return AMPH_E_LEN;
  return abi(amph_party_finish((amph_party*)session, is_player0, w, u));
}

int amphj_party_finish_b64(void* session, int is_player0, char* const* fields, const size_t* lens) {
  if (!session) return set_msg(AMPH_E_PARAM, "null party session");
  const size_t nb = 16 * amph_party_words((const amph_party*)session), nc = 4 * ((nb + 2) / 3);
  for (int k = 0; k < 5; ++k)
    if (room(lens[k], nc, "a base64 field array")) return AMPH_E_LEN;
  return abi(amph_party_finish_b64((amph_party*)session, is_player0, fields));
}

void amphj_party_free(void* session) { amph_party_free((amph_party*)session); }

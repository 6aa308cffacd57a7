/*
 * JNI-independent core of libamphora_jni: the length checks, the status ->
 * Java exception mapping and the calls into libamphora_hip, over plain
 * pointers and Java array lengths.  amphora_jni.c pins the Java arrays and
 * calls these; tests/test_jni_core.py drives them through ctypes (no JDK is
 * needed for that), so everything but the pinning is tested here.
 *
 * Each call takes the Java arrays' lengths as well as their data: the C ABI
 * trusts one word count per call, so a Java byte[] shorter than the count
 * implies must be rejected HERE, before any copy reads or writes past it.
 *
 * Return convention: the libamphora_hip status (AMPH_OK, AMPH_E_*); a call
 * that verifies writes the smallest failing word index to *fail (-1 if every
 * word verified).  amphj_message() holds the text of the last failure on the
 * calling thread; amphj_exception_class() names the Java exception a status
 * maps to (the reference's exception types).
 */
#ifndef AMPHORA_JNI_CORE_H_
#define AMPHORA_JNI_CORE_H_

#include <stddef.h>
#include <stdint.h>

#include "amphora.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Region mode for this thread's following calls (amphora_jni.c): the data
 * pointers of recombine_verify, mask_input, recombine, verify, mask_words,
 * convert_share (not its key), odo_pre and open_post are amph_host_array
 * descriptors, passed with AMPH_F_HOST_IO.  Lengths are still the arrays'. */
void amphj_set_host_io(int on);

/* JNI class names ("/"-separated), or NULL for AMPH_OK */
const char* amphj_exception_class(int status);
const char* amphj_message(void);

/* SecretShareUtil.of(prime, r, rInv): LE16 integers; devices NULL / ndev 0 = device 0 */
int amphj_ctx_create(const uint8_t* p_le, size_t p_len, const uint8_t* r_le, size_t r_len,
                     const uint8_t* rinv_le, size_t rinv_len, const int* devices, int ndev, void** ctx);
void amphj_ctx_destroy(void* ctx);

/* ---- client ------------------------------------------------------------- */
/* fields[k * n + j] = party j's field k (secretShares, rShares, vShares,
 * wShares, uShares), lens likewise (Java array lengths in bytes) */
int amphj_recombine_verify(void* ctx, int n, const uint8_t* const* fields, const size_t* lens,
                           uint8_t* out, size_t out_len, int64_t* fail);
int amphj_mask_input(void* ctx, int n, const uint8_t* const* fields, const size_t* lens,
                     const uint8_t* secrets, size_t secrets_len, uint8_t* out, size_t out_len,
                     int64_t* fail);
int amphj_recombine(void* ctx, int n, const uint8_t* const* shares, const size_t* lens, uint8_t* out,
                    size_t out_len);
/* verifySecrets over five canonical LE16 arrays (Java argument order) */
int amphj_verify(void* ctx, const uint8_t* const* ys_rs_us_vs_ws, const size_t* lens, int64_t* fail);
int amphj_mask_words(void* ctx, const uint8_t* secrets, size_t s_len, const uint8_t* masks,
                     size_t m_len, uint8_t* out, size_t out_len);
/* one word on the calling thread (amph_mask_word_host): no device work */
int amphj_mask_word(void* ctx, const uint8_t secret[16], const uint8_t mask[16], uint8_t out[16]);
/* the IntegrityVerificationException text for one word (5 LE16 values) */
int amphj_verify_message(void* ctx, const uint8_t* y, const uint8_t* r, const uint8_t* u,
                         const uint8_t* v, const uint8_t* w, char* buf, size_t cap);
/* straight from the response text: texts / lens as `fields` above (ASCII) */
int amphj_recombine_verify_b64(void* ctx, int n, const char* const* texts, const size_t* lens,
                               size_t words, uint8_t* out, size_t out_len, int64_t* fail);
int amphj_mask_input_b64(void* ctx, int n, const char* const* texts, const size_t* lens, size_t words,
                         const uint8_t* secrets, size_t secrets_len, char* records24,
                         size_t records_len, int64_t* fail);

/* ---- service ------------------------------------------------------------ */
int amphj_convert_share(void* ctx, const uint8_t* masked, size_t masked_len, const uint8_t* tuples,
                        size_t tuples_len, const uint8_t* mac_key_le, size_t key_len, int use_zero_input_as_data,
                        uint8_t* out, size_t out_len);
/* shareData (stride 32 = SecretShare.data, 16 = raw words) -> y, r, v and
 * the signed Beaver diffs (2 pairs per word: magnitudes 64 B, signs 4 B) */
int amphj_odo_pre(void* ctx, const uint8_t* share, size_t share_len, int stride, const uint8_t* masks,
                  size_t masks_len, const uint8_t* triples, size_t triples_len, uint8_t* y, uint8_t* r,
                  uint8_t* v, size_t out_len, uint8_t* mag, size_t mag_len, uint8_t* neg, size_t neg_len);
int amphj_open_post(void* ctx, int n, const uint8_t* const* mags, const size_t* mag_lens,
                    const uint8_t* const* negs, const size_t* neg_lens, const uint8_t* triples,
                    size_t triples_len, int is_player0, uint8_t* w, uint8_t* u, size_t out_len);
/* MultiplicationExchangeObject.interimValues text <-> signed diffs */
size_t amphj_exchange_max_chars(size_t npairs);
int amphj_exchange_encode(void* ctx, const uint8_t* mag, size_t mag_len, const uint8_t* neg,
                          size_t neg_len, char* out, size_t out_cap, uint64_t* out_len);
int amphj_exchange_decode(void* ctx, const char* text, size_t len, size_t npairs, uint8_t* mag,
                          size_t mag_len, uint8_t* neg, size_t neg_len);
/* one request's Output Delivery with device-resident state (amph_party_*):
 * y/r/v may be NULL (then finish_b64 returns them); texts are ASCII bytes */
int amphj_party_begin(void* ctx, const uint8_t* share, size_t share_len, int stride, const uint8_t* masks,
                      size_t masks_len, const uint8_t* triples, size_t triples_len, int n_parties, uint8_t* y,
                      uint8_t* r, uint8_t* v, size_t out_len, void** session);
uint64_t amphj_party_text_len(void* session);
int amphj_party_text(void* session, char* out, size_t out_len);
int amphj_party_partner(void* session, int slot, const char* text, size_t len);
int amphj_party_finish(void* session, int is_player0, uint8_t* w, uint8_t* u, size_t out_len);
/* fields[k] (secretShares, rShares, vShares, wShares, uShares), lens[k] bytes each */
int amphj_party_finish_b64(void* session, int is_player0, char* const* fields, const size_t* lens);
void amphj_party_free(void* session);

#ifdef __cplusplus
}
#endif
#endif /* AMPHORA_JNI_CORE_H_ */

/*
 * libamphora_hip -- C ABI of the MI355X-native Amphora share arithmetic.
 *
 * The drop-in boundary for the reference's per-word BigInteger path
 * (carbynestack/amphora, snapshot 2025-03-21; paths relative to the repo):
 *
 *   amph_ctx_create      <- client SecretShareUtil.of(prime, r, rInv)
 *                           amphora-java-client/.../client/SecretShareUtil.java:48-51;
 *                           service UtilsConfig.java:17-25 (MpSpdzIntegrationUtils.of)
 *   amph_recombine_verify<- DefaultAmphoraClient.verifyOutputDeliveryObjects
 *                           amphora-java-client/.../DefaultAmphoraClient.java:476-505
 *                           (= 5 x SecretShareUtil.recombineObject :70-90
 *                              + SecretShareUtil.verifySecrets :102-141)
 *   amph_mask_input      <- DefaultAmphoraClient.createSecret arithmetic :150-160
 *                           (verifyOutputDeliveryObjects on the Input Mask ODOs
 *                            + SecretShareUtil.maskInput :65-68 per word)
 *   amph_recombine       <- SecretShareUtil.recombineObject :70-90
 *   amph_verify          <- SecretShareUtil.verifySecrets :102-141
 *   amph_convert_share   <- service calculation/SecretShareUtil.convertToSecretShare
 *                           amphora-service/.../calculation/SecretShareUtil.java:58-107
 *   amph_odo_pre         <- OutputDeliveryService.computeOutputDeliveryObject
 *                           amphora-service/.../calculation/OutputDeliveryService.java:75-139
 *                           + multiplyShares diff computation :186-200
 *   amph_open_diffs      <- OutputDeliveryService.recombineDiffs :231-272 (the sum)
 *   amph_odo_post        <- OutputDeliveryService.multiplySharedSecrets :274-286
 *                           + w/u encoding :147-152
 *   amph_open_post       <- recombineDiffs :231-272 + multiplySharedSecrets :274-286
 *                           + w/u encoding :147-152 (the two calls above, fused)
 *   amph_party_*         <- computeOutputDeliveryObject :75-286 for one request with the
 *                           triples, diffs and ODO fields device-resident between steps
 *   amph_mask_words      <- SecretShareUtil.maskInput :65-68 (canonical mask given)
 *   amph_to_gfp / amph_from_gfp <- MpSpdzIntegrationUtils.toGfp / fromGfp (call
 *                           sites: client SecretShareUtil.java:56,67; service
 *                           SecretShareUtil.java:87-104; OutputDeliveryService.java:129-131,150-151)
 *
 * Word format: every field element on the wire is 16 bytes, the
 * mp-spdz-integration 0.2.2 "gfp" encoding toGfp(x) = LE16(x * R mod p),
 * R = 2^128 (see oracle/amphora_oracle.py, ENCODING "mont_le").  Integers
 * crossing the ABI in canonical form (secrets, MAC key, opened diffs) are
 * plain little-endian 16-byte unsigned integers; the host reduces arbitrary
 * BigIntegers mod p before packing.
 *
 * Memory: by default every buffer is a caller-owned HOST pointer; the call is
 * synchronous and retains nothing.  With AMPH_F_DEVICE every buffer
 * (including first_fail) is a DEVICE pointer on the context's device, the call
 * only enqueues work on `stream` (a hipStream_t, NULL = default stream) and
 * returns; first_fail then holds AMPH_NO_FAILURE or the failing index once the
 * stream reaches that point.  Device word arrays (16-byte words, tuples,
 * diff magnitudes) must be 16-byte aligned and first_fail 8-byte aligned
 * (AMPH_E_PARAM otherwise): the kernels move them as 16-byte vectors.
 *
 * Threading: host-pointer calls on one context are serialised by an internal
 * mutex; device-pointer calls use no context state and may run concurrently.
 *
 * Errors: functions return AMPH_OK (0) or a negative/positive status below.
 * AMPH_E_VERIFY = the MAC check failed; *first_fail then holds the smallest
 * failing word index (the Java path throws IntegrityVerificationException for
 * some failing index; see amph_verify_message for the message text).
 */
#ifndef AMPHORA_H_
#define AMPHORA_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AMPH_WORD_WIDTH 16  /* MpSpdzIntegrationUtils.WORD_WIDTH */
#define AMPH_SHARE_WIDTH 32 /* MpSpdzIntegrationUtils.SHARE_WIDTH (value || mac) */
#define AMPH_INPUT_MASK_TUPLE_SIZE 32 /* castor INPUT_MASK_GFP tuple: value || mac */
#define AMPH_TRIPLE_TUPLE_SIZE 96     /* castor MULTIPLICATION_TRIPLE_GFP: a,mac,b,mac,c,mac */
#define AMPH_MAX_PARTIES 16

/* status codes */
#define AMPH_OK 0
#define AMPH_E_VERIFY 1   /* IntegrityVerificationException */
#define AMPH_E_LEN 2      /* IllegalArgumentException (length invariants) */
#define AMPH_E_PARAM 3    /* invalid argument / field parameters */
#define AMPH_E_HIP 4      /* HIP runtime error (see amph_last_error) */
#define AMPH_E_NOMEM 5    /* device or host allocation failed */
#define AMPH_E_RANGE 6    /* ArrayIndexOutOfBoundsException (a ragged party's word
                             starts past its array's end, see amph_odo) */

/* flags */
#define AMPH_F_DEVICE 0x1u /* all buffers are device pointers; async on `stream` */
/* with AMPH_F_DEVICE: do not reset *first_fail before the launch; the kernel
 * min-combines its failing index (local to this call) into the value there.
 * The caller sets it to AMPH_NO_FAILURE once before a run of calls (saves
 * one memset launch per call; used by bench.py and for repeated passes). */
#define AMPH_F_ACCUMULATE 0x2u
/* Host arrays behind callbacks: every word-array argument of the call is a
 * `const amph_host_array*` (cast to the argument's pointer type) instead of
 * host memory, and the library moves the words with the descriptors' read /
 * write callbacks as its batched pipeline consumes and produces them (a JNI
 * layer's Get/SetByteArrayRegion: the Java heap is not pinned across the GPU
 * call -- INTEGRATION.md).  Accepted by the word-array calls that stream
 * through the host pipeline: amph_recombine_verify, amph_mask_input,
 * amph_recombine, amph_recombine_object, amph_verify, amph_mask_words,
 * amph_to_gfp, amph_from_gfp, amph_convert_share, amph_odo_pre,
 * amph_open_diffs, amph_odo_post, amph_open_post; refused (AMPH_E_PARAM) by
 * every other call with flags, and exclusive with AMPH_F_DEVICE.
 * What stays raw host memory under AMPH_F_HOST_IO (read or written on the
 * calling thread, never through a callback):
 *   - the MAC key of amph_convert_share (16 bytes, mac_key_le);
 *   - the containers of per-party arrays: the amph_odo array (its five field
 *     pointers ARE descriptors, nbytes stays a length), and the `shares` /
 *     `mags` / `negs` pointer arrays and amph_recombine_object's `nbytes`
 *     (their entries are descriptors / lengths);
 *   - first_fail, and every scalar.
 * Offsets and sizes are in bytes from the start of the array the descriptor
 * stands for; a call reads only what its word counts and lengths imply (a
 * ragged party's last word only up to its nbytes), so the caller checks
 * array lengths first. */
#define AMPH_F_HOST_IO 0x4u
typedef struct amph_host_array {
  /* copy `bytes` bytes at byte offset `off` of the array into dst (inputs)
   * or from src into it (outputs); return 0, or nonzero to fail the call
   * (AMPH_E_PARAM, after the copies in flight have ended).  Called from the
   * library's staging threads -- several at once, for disjoint ranges --
   * and never after the call has returned. */
  int (*read)(const struct amph_host_array* a, size_t off, size_t bytes, void* dst);
  int (*write)(const struct amph_host_array* a, size_t off, size_t bytes, const void* src);
  void* user;
} amph_host_array;

/* value of a device-side first_fail word when every word verified */
#define AMPH_NO_FAILURE ((int64_t)0x7F7F7F7F7F7F7F7FLL)

typedef struct amph_ctx amph_ctx;

/* One party's OutputDeliveryObject (amphora-common OutputDeliveryObject.java:55-106):
 * five byte[] of equal length nbytes.
 * Parties may differ in length, with recombineObject's semantics (client
 * SecretShareUtil.java:75,87-88): words W = odos[0].nbytes / 16 (a trailing
 * partial word is ignored); party j's word i is Arrays.copyOfRange(field,
 * 16 i, 16 i + 16), so a longer party is cut to W words, a party ending
 * inside word W-1 (16 (W-1) <= nbytes < 16 W) has that word zero-padded
 * (it then nearly always fails its MAC check: AMPH_E_VERIFY at W-1), and a
 * party ending before 16 (W-1) makes a word start past its end:
 * AMPH_E_RANGE (ArrayIndexOutOfBoundsException), nothing written.
 * amph_recombine_verify and amph_mask_input take such ragged parties in
 * every mode; the wire-text calls and amph_stream_probe need equal lengths
 * (AMPH_E_LEN). */
typedef struct amph_odo {
  const uint8_t* secret_shares; /* <y>  */
  const uint8_t* r_shares;      /* <r>  */
  const uint8_t* v_shares;      /* <v>  */
  const uint8_t* w_shares;      /* <w> = <y r> */
  const uint8_t* u_shares;      /* <u> = <v r> */
  size_t nbytes;
} amph_odo;

/* ---- context ---------------------------------------------------------- */
/* p, r = 2^128 mod p, rInv = r^-1 mod p as LE16 integers (SpdzProperties /
 * DefaultAmphoraClientBuilder.prime/r/rInv).  Checks p odd, r == 2^128 mod p
 * and r * rInv == 1 (mod p).  `device` = HIP device ordinal. */
int amph_ctx_create(const uint8_t p_le[16], const uint8_t r_le[16], const uint8_t rinv_le[16],
                    int device, amph_ctx** out);
/* Several GPUs behind one context (SURVEY.md 8b's amph_ctx_create(...,
 * const int* devices, int ndev, ...)): host-pointer calls split their word
 * range into ndev contiguous shards, stream each through its own device
 * concurrently (every shard with its own 3-slot pipeline and staging
 * threads) and report the smallest failing word index over all shards --
 * SURVEY.md 8e's "direct per-GPU HtoD from pinned memory" for host-origin
 * data (C5).  Device-pointer calls (AMPH_F_DEVICE) and the exchange codec
 * run on devices[0].  A device may appear more than once.  ndev == 1 is
 * amph_ctx_create. */
int amph_ctx_create_multi(const uint8_t p_le[16], const uint8_t r_le[16],
                          const uint8_t rinv_le[16], const int* devices, int ndev,
                          amph_ctx** out);
void amph_ctx_destroy(amph_ctx* ctx);
int amph_ctx_device(const amph_ctx* ctx);
/* Number of devices behind the context (1 unless amph_ctx_create_multi). */
int amph_ctx_device_count(const amph_ctx* ctx);
/* Host-path maximum batch size in words (default 4 Mi); 0 keeps the current
 * value.  A call is cut into about 8 batches of at least 32 MiB of traffic
 * each, at most this many words.
 * Host-pointer calls stream their arrays through the GPU batch by batch:
 * pageable caller memory is staged through page-locked buffers by CPU
 * threads (AMPH_HOST_THREADS, default min(8, cores/2)) with HtoD, kernel and
 * DtoH of consecutive batches overlapped on 3 HIP streams. */
int amph_ctx_set_batch_words(amph_ctx* ctx, size_t words);

/* Counters of a context (summed over the devices of a multi-device context),
 * for tests and operators: no reference interface corresponds (the Java
 * path has no device state).
 *   kernel_launches  arithmetic / codec kernels launched so far
 *   pool_buffers / pool_bytes  party-session device buffers kept for reuse
 *     after amph_party_free (at most 16 buffers and AMPH_PARTY_POOL_BYTES
 *     bytes, default 32 GiB, per device; freed, and the allocation retried,
 *     when any device allocation of the context runs out of memory)
 *   device_workers   long-lived per-device threads of a multi-device
 *     context (created with it; run_sharded posts each call's shards to
 *     them instead of starting threads per call)
 *   worker_tasks     shards those workers have run */
typedef struct amph_stats {
  uint64_t kernel_launches;
  uint64_t pool_buffers;
  uint64_t pool_bytes;
  uint64_t device_workers;
  uint64_t worker_tasks;
} amph_stats;
int amph_ctx_stats(amph_ctx* ctx, amph_stats* out);
/* Page-lock a caller buffer (hipHostRegister, portable to every device) so
 * host-pointer calls DMA it directly without the staging copy (e.g. a
 * long-lived direct ByteBuffer). */
int amph_host_register(amph_ctx* ctx, void* ptr, size_t bytes);
int amph_host_unregister(amph_ctx* ctx, void* ptr);

/* Kernel timing: the next kernel launch made by an amph_* call on the
 * calling thread records these hipEvent_t's (created, timing-enabled) at its
 * own dispatch start / end (hipExtLaunchKernel), so hipEventElapsedTime
 * measures the kernel alone.  Either may be NULL.  Used by bench.py. */
int amph_time_next_launch(void* start_event, void* stop_event);
/* Timing-only hipEvent_t for amph_time_next_launch, created with
 * hipEventDisableSystemFence: recording it does no system-scope release, so
 * it does not write back and invalidate L2 between the timed kernel and the
 * next one (measured at 1 Mi words: a stamped launch costs 3.7 us of
 * dispatch with these events, 5.0 us with default ones; tools/step_overhead.py).
 * Not for host synchronisation with the work it follows. */
int amph_timing_event_create(void** event);
int amph_timing_event_destroy(void* event);
/* Record a timing event on a stream (hipEventRecord): bracketing an amph_*
 * call with two of these times it from the end of the work before it. */
int amph_timing_event_record(void* event, void* stream);
/* Milliseconds between two recorded, completed timing events. */
int amph_timing_event_elapsed_ms(void* start_event, void* stop_event, float* ms);

const char* amph_strerror(int status);
/* Detail of the last error on the calling thread (empty string if none). */
const char* amph_last_error(void);
const char* amph_version(void);
/* Identity of the build: 16 hex digits of a SHA-256 over the sources and
 * headers the library is compiled from, the compile flags and the offload
 * arch (tools/build_native.py tree_digest).  Recomputing it from a source
 * tree and comparing proves which tree a tested binary came from. */
const char* amph_build_id(void);

/* ---- client (amphora-java-client) ------------------------------------- */
/* verifyOutputDeliveryObjects: recombine the 5 fields over n_parties ODOs,
 * check w == y r and u == v r for every word, write the canonical secrets y
 * (LE16, words = odos[0].nbytes / 16).  Returns AMPH_E_VERIFY with
 * *first_fail = smallest failing index, else *first_fail = -1 (host mode). */
int amph_recombine_verify(amph_ctx* ctx, const amph_odo* odos, int n_parties,
                          uint8_t* out_secrets, int64_t* first_fail, uint32_t flags,
                          void* stream);

/* createSecret arithmetic: verify the Input Mask ODOs as above and write
 * masked[i] = toGfp((secret_i - mask_i) mod p) for i < n_secrets.
 * secrets: LE16 integers (any 128-bit value; reduced mod p).
 * n_secrets must be <= the ODO word count, else AMPH_E_LEN -- but, as in
 * the reference (DefaultAmphoraClient.java:153 verifies before :160 indexes),
 * only after all the masks verified: a MAC failure there returns
 * AMPH_E_VERIFY with *first_fail set, in both modes (device mode waits for
 * the verdict on this error path). */
int amph_mask_input(amph_ctx* ctx, const amph_odo* mask_odos, int n_parties,
                    const uint8_t* secrets, size_t n_secrets, uint8_t* out_masked,
                    int64_t* first_fail, uint32_t flags, void* stream);

/* recombineObject for one byte[] field: out[i] = sum_j fromGfp(share_j[i]) mod p. */
int amph_recombine(amph_ctx* ctx, const uint8_t* const* shares, int n_parties, size_t nbytes,
                   uint8_t* out, uint32_t flags, void* stream);
/* recombineObject exactly (client SecretShareUtil.java:70-90), parties of
 * their own lengths nbytes[j]: words = nbytes[0] / 16 and the ragged-party
 * rules of amph_odo (zero-padded last word, AMPH_E_RANGE).  Equal lengths
 * are amph_recombine.  Same flags (AMPH_F_DEVICE / AMPH_F_HOST_IO). */
int amph_recombine_object(amph_ctx* ctx, const uint8_t* const* shares, int n_parties,
                          const size_t* nbytes, uint8_t* out, uint32_t flags, void* stream);

/* verifySecrets over canonical LE16 integers (argument order of the Java
 * method: secrets, rs, us, vs, ws).  The host must pass w, u < p (a value
 * outside [0, p) can never equal a reduced product: fail it before calling). */
int amph_verify(amph_ctx* ctx, const uint8_t* secrets, const uint8_t* rs, const uint8_t* us,
                const uint8_t* vs, const uint8_t* ws, size_t words, int64_t* first_fail,
                uint32_t flags, void* stream);

/* Renders the IntegrityVerificationException message of SecretShareUtil.java:116-129
 * for canonical LE16 values (w, y, r, u, v) of the failing word into buf
 * (NUL-terminated, truncated to cap).  Returns the untruncated length. */
int amph_verify_message(amph_ctx* ctx, const uint8_t y[16], const uint8_t r[16],
                        const uint8_t u[16], const uint8_t v[16], const uint8_t w[16], char* buf,
                        size_t cap);

/* maskInput word by word with canonical masks (SecretShareUtil.java:65-68):
 * out[i] = toGfp((secrets[i] - masks[i]) mod p); both LE16 integers. */
int amph_mask_words(amph_ctx* ctx, const uint8_t* secrets, const uint8_t* masks, size_t words,
                    uint8_t* out, uint32_t flags, void* stream);
/* The same for ONE word on the calling thread, with no device work: the
 * reference's per-word maskInput (SecretShareUtil.java:65-68, called once per
 * word by DefaultAmphoraClient.java:155-160) is not worth a kernel launch and
 * a stream synchronisation.  secret / mask are LE16 integers (reduced mod p
 * here); out = LE16((secret - mask) mod p * R mod p).  Batched callers use
 * amph_mask_input (verify + mask on the GPU). */
int amph_mask_word_host(amph_ctx* ctx, const uint8_t secret[16], const uint8_t mask[16], uint8_t out[16]);

/* MpSpdzIntegrationUtils.toGfp / fromGfp over word arrays (mp-spdz-integration
 * 0.2.2, absent; restated): toGfp(x) = LE16(x R mod p) for any LE16 integer x;
 * fromGfp(b) = LEint(b) R^-1 mod p. */
int amph_to_gfp(amph_ctx* ctx, const uint8_t* in, size_t words, uint8_t* out, uint32_t flags,
                void* stream);
int amph_from_gfp(amph_ctx* ctx, const uint8_t* in, size_t words, uint8_t* out, uint32_t flags,
                  void* stream);

/* ---- service (amphora-service) ---------------------------------------- */
/* convertToSecretShare: masked (words x 16) + input mask tuples (words x 32,
 * share 0 value || mac) -> SecretShare.data (words x 32, value || mac).
 * mac_key: the party's MAC key as an LE16 integer (reduced mod p by the
 * caller, as new BigInteger(macKey) mod p); raw host memory even under
 * AMPH_F_HOST_IO (never a descriptor).  use_zero_input_as_data =
 * (playerId != 0) in StorageService.createSecret :104-109. */
int amph_convert_share(amph_ctx* ctx, const uint8_t* masked, const uint8_t* mask_tuples,
                       size_t words, const uint8_t mac_key_le[16], int use_zero_input_as_data,
                       uint8_t* out_share, uint32_t flags, void* stream);

/* computeOutputDeliveryObject front half + Beaver diffs.
 * share_data: words x share_stride bytes (32 = SecretShare.data with MACs,
 * stripped as in :79-84; 16 = raw words as in InputMaskCachingService :81-91).
 * mask_tuples: 2*words input-mask tuples (32 B); triples: 2*words triples (96 B).
 * out_y/out_r/out_v: raw copies (secretShares, rShares, vShares of the ODO).
 * out_diff_mag: 2*words pairs x 2 values x 16 B, FactorPair order
 * [d_0, e_0, d_1, e_1, ...]; out_diff_neg: same order, 1 byte each (1 = negative).
 * Pair 2i = (y_i, r_i), pair 2i+1 = (v_i, r_i); d = x - a, e = y - b,
 * signed and unreduced, exactly as :186-200. */
int amph_odo_pre(amph_ctx* ctx, const uint8_t* share_data, size_t share_stride,
                 const uint8_t* mask_tuples, const uint8_t* triples, size_t words,
                 uint8_t* out_y, uint8_t* out_r, uint8_t* out_v, uint8_t* out_diff_mag,
                 uint8_t* out_diff_neg, uint32_t flags, void* stream);

/* recombineDiffs: opened = sum over n_parties signed diff lists (as written
 * by amph_odo_pre) mod p, canonical LE16, same [D_0, E_0, ...] order.
 * n_pairs = number of FactorPairs (= 2 * words). */
int amph_open_diffs(amph_ctx* ctx, const uint8_t* const* diff_mags,
                    const uint8_t* const* diff_negs, int n_parties, size_t n_pairs,
                    uint8_t* out_opened, uint32_t flags, void* stream);

/* multiplySharedSecrets + toGfp: per pair k, z = c + D b + E a (+ D E if
 * is_player0) mod p; out_w[i] = toGfp(z_2i), out_u[i] = toGfp(z_2i+1).
 * opened: 2*words pairs x 2 canonical LE16 values. */
int amph_odo_post(amph_ctx* ctx, const uint8_t* opened, const uint8_t* triples, size_t words,
                  int is_player0, uint8_t* out_w, uint8_t* out_u, uint32_t flags, void* stream);

/* recombineDiffs + multiplySharedSecrets + toGfp in one pass (the two calls
 * above fused: the opened D, E never leave the GPU's registers).  Per pair k:
 * D, E = sum over n_parties of the signed diffs (amph_open_diffs' inputs),
 * then out_w / out_u exactly as amph_odo_post.  Same outputs, bit for bit, as
 * amph_open_diffs followed by amph_odo_post; 360 instead of 488 HBM bytes per
 * word at 2 parties.  words = n_pairs / 2 = triples / 2. */
int amph_open_post(amph_ctx* ctx, const uint8_t* const* diff_mags, const uint8_t* const* diff_negs,
                   int n_parties, const uint8_t* triples, size_t words, int is_player0,
                   uint8_t* out_w, uint8_t* out_u, uint32_t flags, void* stream);

/* ---- wire codec ----------------------------------
 * Base64 as Jackson writes byte[] (Base64Variants.MIME_NO_LINEFEEDS: standard
 * alphabet, '=' padding, no line breaks): the secretShares/rShares/... fields
 * of VerifiableSecretShare / OutputDeliveryObject JSON
 * (amphora-common/.../VerifiableSecretTest.java:41-90) and the per-word
 * {"value": ...} of MaskedInputData (MaskedInputData.java:44-52).
 * encode: out gets 4 * ceil(nbytes / 3) chars.
 * decode: nchars % 4 == 0 (else AMPH_E_LEN); *out_bytes = decoded length;
 *   an illegal character returns AMPH_E_PARAM with *bad_index = its position
 *   (device mode: bad_index is a device word, AMPH_NO_FAILURE if clean; with
 *   out_bytes non-null the call reads the last 2 chars back to size the
 *   output -- a stream synchronisation; with out_bytes NULL it is fully
 *   asynchronous: the kernel sizes the output itself, out must hold
 *   3 * nchars / 4 bytes and the caller knows the decoded length, e.g.
 *   16 bytes per word of an ODO field).
 * words: one 16-byte word <-> one 24-char record (per-word base64). */
int amph_base64_encode(amph_ctx* ctx, const uint8_t* in, size_t nbytes, char* out, uint32_t flags,
                       void* stream);
int amph_base64_decode(amph_ctx* ctx, const char* in, size_t nchars, uint8_t* out,
                       size_t* out_bytes, int64_t* bad_index, uint32_t flags, void* stream);
int amph_base64_encode_words(amph_ctx* ctx, const uint8_t* words16, size_t words, char* out24,
                             uint32_t flags, void* stream);
int amph_base64_decode_words(amph_ctx* ctx, const char* in24, size_t words, uint8_t* out16,
                             int64_t* bad_index, uint32_t flags, void* stream);

/* ---- K_RV / K_MASK straight from the wire ----------------------------------
 * The client receives every party's ODO as base64 text -- the secretShares,
 * rShares, vShares, wShares, uShares strings of the VerifiableSecretShare
 * (GET /secret-shares/{id}) or OutputDeliveryObject (GET /input-masks) JSON --
 * and uploads each masked word as a 24-character base64 record
 * ({"value":"..."} of MaskedInputData).  These calls run the arithmetic of
 * amph_recombine_verify / amph_mask_input on the text itself: each workgroup
 * decodes its slice of every field into LDS and consumes it there, so the
 * decoded words never round-trip through HBM (replaces Jackson's base64
 * decode of each field + verifyOutputDeliveryObjects, DefaultAmphoraClient.java:
 * 206-217 / 150-170, MaskedInputData.java:44-52 for the records).
 *
 * Every field of every party must be the base64 of exactly 16 * words bytes:
 * nchars = 4 * ceil(16 * words / 3), '=' padding only in the final group
 * (else AMPH_E_LEN).  bad_char: the smallest (5 * party + field) * nchars +
 * offset of a character outside the alphabet (field 0..4 = secretShares,
 * rShares, vShares, wShares, uShares); -1 / the device sentinel when clean.
 * Host mode: AMPH_E_PARAM on a bad character (message names party, field
 * and offset), else AMPH_E_VERIFY as amph_recombine_verify.  Device mode:
 * text pointers 16-byte aligned, first_fail and bad_char device int64s,
 * asynchronous on `stream`. */
typedef struct amph_odo_b64 {
  const char* secret_shares;
  const char* r_shares;
  const char* v_shares;
  const char* w_shares;
  const char* u_shares;
  size_t nchars; /* characters in each of the five strings */
} amph_odo_b64;

int amph_recombine_verify_b64(amph_ctx* ctx, const amph_odo_b64* odos, int n_parties, size_t words,
                              uint8_t* out_secrets, int64_t* first_fail, int64_t* bad_char,
                              uint32_t flags, void* stream);
/* out_masked16 (16 B per secret) and/or out_records24 (24 base64 characters
 * per secret, MaskedInputData's value; device: 16-byte aligned) may be NULL.
 * n_secrets > words: the texts are decoded and every mask verified first (a
 * bad character or a MAC failure is reported as such, as the reference
 * decodes and verifies before it indexes, DefaultAmphoraClient.java:153-160),
 * and only then AMPH_E_LEN; device mode waits for the verdicts on that path. */
int amph_mask_input_b64(amph_ctx* ctx, const amph_odo_b64* mask_odos, int n_parties, size_t words,
                        const uint8_t* secrets, size_t n_secrets, uint8_t* out_masked16,
                        char* out_records24, int64_t* first_fail, int64_t* bad_char, uint32_t flags,
                        void* stream);

/* ---- Beaver open exchange wire format --------------------------------------
 * MultiplicationExchangeObject.interimValues, the FactorPair list each party
 * sends its partners (amphora-common/.../MultiplicationExchangeObject.java:
 * 20-39, FactorPair.java:16-25; built in OutputDeliveryService.java:186-200,
 * consumed by recombineDiffs :231-272), as the JSON array Jackson writes:
 * [{"a":<d_0>,"b":<e_0>},{"a":<d_1>,"b":<e_1>},...] with the signed BigIntegers
 * as plain decimal numbers.  Replaces the Jackson (de)serialisation of that
 * list on the /inter-vcp/open exchange.
 *
 * Diffs use amph_odo_pre's layout: mag16 = 2 * npairs magnitudes (LE16, d_k
 * then e_k), neg = 2 * npairs sign bytes (nonzero = negative).
 *
 * encode: out gets the compact array text, byte-identical to Jackson's
 *   default output; *out_len = its length.  Device mode: out_cap must be
 *   >= amph_exchange_max_chars(npairs) and out_len is a device word, written
 *   asynchronously.  Host mode: AMPH_E_LEN with *out_len = the needed length
 *   if out_cap is too small.
 * decode: text = the array (whitespace between tokens allowed; member order
 *   "a","b" or "b","a").  A malformed token returns AMPH_E_PARAM with
 *   *bad_index = its byte offset; a count other than npairs pairs returns
 *   AMPH_E_LEN (*bad_index = len).  Magnitudes must be < 2^128.  Device mode:
 *   bad_index is a device word (AMPH_NO_FAILURE when clean, len on a count
 *   mismatch). */
size_t amph_exchange_max_chars(size_t npairs);
int amph_exchange_encode(amph_ctx* ctx, const uint8_t* mag16, const uint8_t* neg, size_t npairs,
                         char* out, size_t out_cap, uint64_t* out_len, uint32_t flags,
                         void* stream);
int amph_exchange_decode(amph_ctx* ctx, const char* text, size_t len, size_t npairs,
                         uint8_t* mag16, uint8_t* neg, int64_t* bad_index, uint32_t flags,
                         void* stream);

/* ---- one party's Output Delivery with device-resident state ---------------
 * OutputDeliveryService.computeOutputDeliveryObject (OutputDeliveryService.java:
 * 75-286) for one request, from host buffers, with everything that is not on
 * the wire kept in device memory between the steps:
 *
 *   begin    the share data, 2*words input masks and 2*words triples in (as
 *            amph_odo_pre); y, r, v out (optional); this party's diffs encoded
 *            as its interimValues text (amph_exchange_encode), kept on the
 *            device -- amph_party_text_len / amph_party_text copy it out
 *            (multiplyShares :186-200, the MultiplicationExchangeObject sent);
 *   partner  one partner's interimValues text in (slot 1 .. n_parties-1),
 *            decoded on the device (recombineDiffs' input, :231-272);
 *   finish   every party's diffs summed, multiplySharedSecrets + the w/u
 *            encoding (:274-286, :147-152), w and u out -- or, with
 *            amph_party_finish_b64, all five ODO fields out as base64 text
 *            (the VerifiableSecretShare body's strings).
 *
 * Only the texts and the ODO fields cross PCIe: the triples, the diffs and the
 * opened values never leave the GPU (a host-path amph_odo_pre / exchange /
 * amph_open_post sequence moves them both ways).  Results are bit-identical to
 * that sequence.  A partner's text is decoded in one read (the values of each
 * 8 KiB of text in their own slots, found by finish through the decoded span
 * bases; no count pass), where amph_exchange_decode reads its text twice to
 * write pair order.  A session belongs to one context (calls are serialised by
 * its mutex), holds about 630 bytes per word of device memory (the triples,
 * the five fields raw and as base64, its own diffs and text at most) plus
 * about 1.1 x each partner text's length (that partner's diffs) and one
 * partner text at a time until amph_party_free, and may be finished once.
 * amph_party_free hands the session's device buffers back to its context,
 * which keeps up to 16 of them for the next session (one session per request
 * then allocates nothing) and frees them in amph_ctx_destroy.
 * amph_party_words = the session's word count; free sessions before their
 * context.  Status semantics
 * as the calls it replaces (amph_exchange_decode's AMPH_E_PARAM / AMPH_E_LEN
 * with *bad_index for a malformed partner text). */
typedef struct amph_party amph_party;
int amph_party_begin(amph_ctx* ctx, const uint8_t* share_data, size_t share_stride,
                     const uint8_t* mask_tuples, const uint8_t* triples, size_t words, int n_parties,
                     uint8_t* out_y, uint8_t* out_r, uint8_t* out_v, amph_party** out);
size_t amph_party_words(const amph_party* party);
uint64_t amph_party_text_len(const amph_party* party);
int amph_party_text(amph_party* party, char* out, size_t out_cap);
int amph_party_partner(amph_party* party, int slot, const char* text, size_t len, int64_t* bad_index);
int amph_party_finish(amph_party* party, int is_player0, uint8_t* out_w, uint8_t* out_u);
/* fields_b64[k], k = 0..4 (secretShares, rShares, vShares, wShares, uShares):
 * 4 * ceil(16 * words / 3) characters each, no terminator */
int amph_party_finish_b64(amph_party* party, int is_player0, char* const fields_b64[5]);
void amph_party_free(amph_party* party);

/* The same session on device buffers, for a server whose tuples and texts are
 * already in GPU memory (e.g. received by RDMA into device memory): nothing is
 * copied to or from the host and nothing synchronises the host; every call
 * is asynchronous on `stream` (one stream per session; amph_party_free waits
 * for it).  begin: share_data, mask_tuples, triples are 16-byte aligned device
 * buffers used in place -- the triples must stay unchanged until finish --
 * and out_y / out_r / out_v (optional) device outputs, which then also hold
 * the session's copies of those fields until finish.  text_dev: the device
 * addresses of this party's text and of its length (a device uint64_t), valid
 * once the stream has run begin; the text's capacity is
 * amph_exchange_max_chars(2 * words).  partner_dev: text is device memory of
 * the given length; *bad_index is a device word set as amph_exchange_decode's
 * device mode sets it (AMPH_NO_FAILURE when the text held) -- check it before
 * finishing.  finish_b64_dev: the five fields as base64 text in the session's
 * device memory, *fields_b64[k] their addresses (amph_party_finish_b64's
 * lengths; valid until amph_party_free) -- the response is sent from there.
 * amph_party_partner_dev writes its verdict to *bad_index on `stream` and
 * the session keeps its own copy (a device word it owns, copied on that
 * stream, plus an event recorded there): the caller may reuse or free
 * bad_index once `stream` has passed the call, and finish_b64_dev waits for
 * every accepted partner call's work (the decoded diffs and the verdict)
 * even when it runs on another stream.
 * If any partner's verdict reports a failure when finish_b64_dev's
 * kernels run, the five fields come out poisoned: their first four
 * characters are "!!!!" (no base64 decoder accepts them), so a response sent
 * without checking the verdicts cannot carry values computed from a rejected
 * text.  To resubmit a slot whose text was rejected, amph_party_reset_partner
 * it first (same stream, or after synchronising).
 * A device-mode session takes only these calls (and amph_party_words /
 * amph_party_reset_partner / amph_party_free; amph_party_text_len reads 0 for
 * it -- its length is the device word); a multi-device context is refused. */
int amph_party_begin_dev(amph_ctx* ctx, const uint8_t* share_data, size_t share_stride,
                         const uint8_t* mask_tuples, const uint8_t* triples, size_t words, int n_parties,
                         uint8_t* out_y, uint8_t* out_r, uint8_t* out_v, void* stream, amph_party** out);
int amph_party_text_dev(amph_party* party, const char** text, const uint64_t** text_len);
int amph_party_partner_dev(amph_party* party, int slot, const char* text, size_t len, int64_t* bad_index,
                           void* stream);
int amph_party_finish_b64_dev(amph_party* party, int is_player0, const char* fields_b64[5], void* stream);
/* Frees partner slot `slot` (1 .. n_parties-1) of an unfinished session
 * (either mode) for another amph_party_partner(_dev) call. */
int amph_party_reset_partner(amph_party* party, int slot);

/* ---- benchmark / test input generation (device pointers only) ---------- */
/* Honest n-party ODOs: out_fields[k * n_parties + j] = field k (y,r,v,w,u) of
 * party j (device, words x 16 B each).  out_plain_y (optional, device) gets the
 * canonical secrets.  fault_index >= 0 adds 1 to party 1's w share there
 * (party 0 if n_parties == 1); noncanon_permille words per 1000 are written as
 * [x] + p (when p > 2^127).  Async on `stream`. */
int amph_synth_odos(amph_ctx* ctx, uint64_t seed, int n_parties, size_t words,
                    uint8_t* const* out_fields, uint8_t* out_plain_y, int64_t fault_index,
                    int noncanon_permille, void* stream);
/* Uniform canonical field elements (LE16), device, async on `stream`. */
int amph_synth_words(amph_ctx* ctx, uint64_t seed, size_t count, uint8_t* out, void* stream);
/* Measurement only (bench.py): K_MASK's exact memory pattern -- the 5n
 * ODO word arrays + the secrets read with the same nontemporal 16-B loads,
 * one 16-B word written per word, same grid -- with the field arithmetic
 * replaced by an XOR.  Device pointers, async on `stream`; honours
 * amph_time_next_launch.  Its duration is the bandwidth this access pattern
 * achieves at this size on this GPU, the practical ceiling for K_MASK. */
int amph_stream_probe(amph_ctx* ctx, const amph_odo* odos, int n_parties, const uint8_t* secrets,
                      size_t words, uint8_t* out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* AMPHORA_H_ */

/*
 * libamphora_jni: the JNI layer between the Java drop-ins under java/ and
 * libamphora_hip (include/amphora.h).  It only pins Java arrays and maps
 * statuses to exceptions; lengths are checked and the C ABI is called by the
 * JNI-independent core (amphora_jni_core.c, tested without a JDK by
 * tests/test_jni_core.py).
 *
 *   io.carbynestack.amphora.client.NativeShareArithmetic
 *     <- client SecretShareUtil.java:48-141, DefaultAmphoraClient.java:150-217,476-505
 *   io.carbynestack.amphora.service.calculation.NativeShareArithmetic
 *     <- service SecretShareUtil.java:58-107, OutputDeliveryService.java:75-286
 *
 * Pinning: GetPrimitiveArrayCritical; inside a critical region a thread may
 * make no JNI call but further Get/ReleasePrimitiveArrayCritical, so every
 * array element and length is fetched before the first array is pinned.  A
 * refused pin (NULL, OutOfMemoryError pending) releases the others and
 * returns.  Up to 5 x 16 + 2 element references are live at once, more than
 * the 16 a native method is guaranteed, so EnsureLocalCapacity reserves them.  A
 * verify failure is RETURNED (the smallest failing word index); the Java side
 * builds the IntegrityVerificationException message from that word's values,
 * as SecretShareUtil.java:116-129 does.  Other failures are thrown here:
 * IllegalArgumentException for length / argument errors (the reference's
 * messages where it has one), IllegalStateException for runtime errors.
 *
 * Large calls: a critical region blocks the
 * JVM's garbage collector for as long as it is open, and a GPU call at C4
 * sizes lasts tens of milliseconds.  So only calls that move at most
 * AMPH_JNI_REGION_BYTES (default 2 MiB, libamphora_hip's small-call size) pin
 * their arrays.  Above it the word-array calls hand libamphora_hip
 * amph_host_array descriptors (AMPH_F_HOST_IO): the library's staging threads
 * copy each batch with Get/SetByteArrayRegion as its pipeline consumes and
 * produces it (those threads attach to the VM as daemons once), so no
 * critical region is open during the GPU call; the party-session calls copy
 * their arrays into native buffers with region copies instead.
 *
 * Build: jni/Makefile (skipped when no JDK is found -- this image has none).
 */
#include <jni.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "amphora_jni_core.h"

#define MAXP AMPH_MAX_PARTIES

typedef struct {
  jbyteArray ref;
  jsize len;
  jbyte* p;
} Pin;

static void throw_status(JNIEnv* env, int status) {
  const char* cls = amphj_exception_class(status);
  jclass c = cls ? (*env)->FindClass(env, cls) : NULL;
  if (c) (*env)->ThrowNew(env, c, amphj_message());
}

static int throw_arg(JNIEnv* env, const char* msg) {
  jclass c = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
  if (c) (*env)->ThrowNew(env, c, msg);
  return -1;
}

/* refs + lengths of one array (null allowed only when `optional`) */
static int ref(JNIEnv* env, jbyteArray a, Pin* p) {
  if (!a) return throw_arg(env, "null array");
  p->ref = a;
  p->len = (*env)->GetArrayLength(env, a);
  p->p = NULL;
  return 0;
}

/* room for `count` more local references (plus the few a throw needs) */
static int reserve(JNIEnv* env, int count) {
  return (*env)->EnsureLocalCapacity(env, count + 4) < 0 ? -1 : 0;  /* < 0: OutOfMemoryError pending */
}

/* byte[][] fields (one per party) of k = 0..4 into pins[k * n + j] */
static int refs_odo(JNIEnv* env, jobjectArray f[5], Pin* pins, int* n) {
  for (int k = 0; k < 5; ++k)
    if (!f[k]) return throw_arg(env, "null ODO field list");
  *n = (*env)->GetArrayLength(env, f[0]);
  if (*n < 1 || *n > MAXP) return throw_arg(env, "n_parties must be in [1, 16]");
  if (reserve(env, 5 * *n)) return -1;
  for (int k = 0; k < 5; ++k) {
    if ((*env)->GetArrayLength(env, f[k]) != *n)
      return throw_arg(env, "The provided shares must be of the same length");
    for (int j = 0; j < *n; ++j)
      if (ref(env, (jbyteArray)(*env)->GetObjectArrayElement(env, f[k], j), &pins[k * *n + j])) return -1;
  }
  return 0;
}

static int refs_list(JNIEnv* env, jobjectArray a, Pin* pins, int* n) {
  if (!a) return throw_arg(env, "null array list");
  *n = (*env)->GetArrayLength(env, a);
  if (*n < 1 || *n > MAXP) return throw_arg(env, "n_parties must be in [1, 16]");
  if (reserve(env, *n)) return -1;
  for (int j = 0; j < *n; ++j)
    if (ref(env, (jbyteArray)(*env)->GetObjectArrayElement(env, a, j), &pins[j])) return -1;
  return 0;
}

/* outputs (written) are committed, inputs aborted (never copied back) */
static void unpin_all(JNIEnv* env, Pin* pins, int count, int first_output) {
  for (int i = count - 1; i >= 0; --i)
    if (pins[i].p)
      (*env)->ReleasePrimitiveArrayCritical(env, pins[i].ref, pins[i].p, i >= first_output ? 0 : JNI_ABORT);
}

/* -1 if the VM refused a pin (OutOfMemoryError pending): the pins taken are
   released unwritten and nothing reaches the C ABI */
static int pin_all(JNIEnv* env, Pin* pins, int count) {
  for (int i = 0; i < count; ++i) {
    pins[i].p = (*env)->GetPrimitiveArrayCritical(env, pins[i].ref, NULL);
    if (!pins[i].p) {
      unpin_all(env, pins, i, i);
      return -1;
    }
  }
  return 0;
}

/* ---- large calls: region copies instead of pins ----------------------------- */
static size_t region_bytes(void) {
  const char* e = getenv("AMPH_JNI_REGION_BYTES");
  return e ? (size_t)strtoull(e, NULL, 10) : (size_t)2 << 20;
}

static size_t total_len(const Pin* pins, int count) {
  size_t t = 0;
  for (int i = 0; i < count; ++i) t += (size_t)pins[i].len;
  return t;
}

typedef struct {
  amph_host_array a; /* first: the descriptor libamphora_hip sees */
  JavaVM* vm;
  jbyteArray gref;
} JArr;

/* A native thread must detach before it exits (JNI spec, "Detaching from the
   VM").  libamphora_hip's staging and device-worker threads are joined when
   their context is destroyed; a thread-specific key whose destructor detaches
   runs as each of them exits. */
static pthread_key_t g_detach_key;
static pthread_once_t g_detach_once = PTHREAD_ONCE_INIT;
static int g_detach_ok;

static void detach_at_exit(void* vm) {
  JavaVM* v = (JavaVM*)vm;
  (*v)->DetachCurrentThread(v);
}

static void make_detach_key(void) { g_detach_ok = pthread_key_create(&g_detach_key, detach_at_exit) == 0; }

/* the JNIEnv of whichever thread runs the callback: the calling Java thread,
   or one of libamphora_hip's staging threads, attached as a daemon on first use
   (and detached when it exits) */
static JNIEnv* env_here(JavaVM* vm) {
  JNIEnv* e = NULL;
  if ((*vm)->GetEnv(vm, (void**)&e, JNI_VERSION_1_6) == JNI_OK) return e;
  pthread_once(&g_detach_once, make_detach_key);
  if (!g_detach_ok) return NULL; /* could not arrange the detach: do not attach */
  if ((*vm)->AttachCurrentThreadAsDaemon(vm, (void**)&e, NULL) != JNI_OK) return NULL;
  if (pthread_setspecific(g_detach_key, vm) != 0) {
    (*vm)->DetachCurrentThread(vm);
    return NULL;
  }
  return e;
}

static int jarr_read(const amph_host_array* a, size_t off, size_t bytes, void* dst) {
  const JArr* j = (const JArr*)a;
  JNIEnv* e = env_here(j->vm);
  if (!e) return -1;
  (*e)->GetByteArrayRegion(e, j->gref, (jsize)off, (jsize)bytes, (jbyte*)dst);
  if ((*e)->ExceptionCheck(e)) {  /* out of range: the lengths were checked, so not expected */
    (*e)->ExceptionClear(e);
    return -1;
  }
  return 0;
}

static int jarr_write(const amph_host_array* a, size_t off, size_t bytes, const void* src) {
  const JArr* j = (const JArr*)a;
  JNIEnv* e = env_here(j->vm);
  if (!e) return -1;
  (*e)->SetByteArrayRegion(e, j->gref, (jsize)off, (jsize)bytes, (const jbyte*)src);
  if ((*e)->ExceptionCheck(e)) {
    (*e)->ExceptionClear(e);
    return -1;
  }
  return 0;
}

typedef struct {
  int regions;
  JArr ja[5 * MAXP + 2];
} Access;

static void release_access(JNIEnv* env, Pin* pins, int count, int first_output, Access* acc);

/* Small call: pin every array.  Large call: a global reference and an
   amph_host_array descriptor per array (pins[i].p points at it), and the
   core passes AMPH_F_HOST_IO.  -1: an exception is pending, nothing held. */
static int acquire(JNIEnv* env, Pin* pins, int count, Access* acc) {
  acc->regions = total_len(pins, count) > region_bytes();
  if (!acc->regions) return pin_all(env, pins, count);
  JavaVM* vm = NULL;
  if ((*env)->GetJavaVM(env, &vm) != 0 || !vm) return throw_arg(env, "no JavaVM");
  for (int i = 0; i < count; ++i) {
    acc->ja[i].gref = (jbyteArray)(*env)->NewGlobalRef(env, pins[i].ref);
    if (!acc->ja[i].gref) { /* OutOfMemoryError pending */
      release_access(env, pins, i, i, acc);
      return -1;
    }
    acc->ja[i].a.read = jarr_read;
    acc->ja[i].a.write = jarr_write;
    acc->ja[i].a.user = NULL;
    acc->ja[i].vm = vm;
    pins[i].p = (jbyte*)&acc->ja[i].a;
  }
  amphj_set_host_io(1);
  return 0;
}

static void release_access(JNIEnv* env, Pin* pins, int count, int first_output, Access* acc) {
  if (!acc->regions) {
    unpin_all(env, pins, count, first_output);
    return;
  }
  amphj_set_host_io(0);
  for (int i = 0; i < count; ++i) {
    (*env)->DeleteGlobalRef(env, acc->ja[i].gref);
    pins[i].p = NULL;
  }
}

/* party-session calls above the threshold: native copies, filled / drained
   with region copies, so nothing is pinned while the session runs */
static int stage_native(JNIEnv* env, Pin* pins, int count, int first_output) {
  for (int i = 0; i < count; ++i) {
    if (!pins[i].ref) continue;
    pins[i].p = (jbyte*)malloc(pins[i].len ? (size_t)pins[i].len : 1);
    if (!pins[i].p) {
      for (int k = 0; k < i; ++k) free(pins[k].p), pins[k].p = NULL;
      jclass c = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
      if (c) (*env)->ThrowNew(env, c, "native staging of a Java array");
      return -1;
    }
    if (i < first_output) (*env)->GetByteArrayRegion(env, pins[i].ref, 0, pins[i].len, pins[i].p);
  }
  return 0;
}

static void unstage_native(JNIEnv* env, Pin* pins, int count, int first_output, int commit) {
  for (int i = 0; i < count; ++i) {
    if (!pins[i].ref || !pins[i].p) continue;
    if (commit && i >= first_output) (*env)->SetByteArrayRegion(env, pins[i].ref, 0, pins[i].len, pins[i].p);
    free(pins[i].p);
    pins[i].p = NULL;
  }
}

static void ptrs_of(const Pin* pins, int count, const uint8_t** ptrs, size_t* lens) {
  for (int i = 0; i < count; ++i) {
    ptrs[i] = (const uint8_t*)pins[i].p;
    lens[i] = (size_t)pins[i].len;
  }
}

static jlong ctx_create(JNIEnv* env, jbyteArray p, jbyteArray r, jbyteArray rinv, jintArray devices) {
  Pin a[3];
  if (ref(env, p, &a[0]) || ref(env, r, &a[1]) || ref(env, rinv, &a[2])) return 0;
  jint dev[MAXP];
  int ndev = 0;
  if (devices) {
    ndev = (*env)->GetArrayLength(env, devices);
    if (ndev > MAXP) return throw_arg(env, "at most 16 devices"), 0;
    (*env)->GetIntArrayRegion(env, devices, 0, ndev, dev);
  }
  jbyte b[3][16];
  for (int i = 0; i < 3; ++i) {
    if (a[i].len != 16) return throw_arg(env, "prime, r and rInv must be 16-byte little-endian integers"), 0;
    (*env)->GetByteArrayRegion(env, a[i].ref, 0, 16, b[i]);
  }
  void* ctx = NULL;
  const int st = amphj_ctx_create((const uint8_t*)b[0], 16, (const uint8_t*)b[1], 16, (const uint8_t*)b[2], 16,
                                  dev, ndev, &ctx);
  if (st != AMPH_OK) {
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)ctx;
}

#define CTX(x) ((void*)(intptr_t)(x))

/* ---- client ------------------------------------------------------------------- */
#define CLIENT(name) Java_io_carbynestack_amphora_client_NativeShareArithmetic_##name

JNIEXPORT jlong JNICALL CLIENT(ctxCreate)(JNIEnv* env, jclass cls, jbyteArray p, jbyteArray r, jbyteArray rinv,
                                          jintArray devices) {
  (void)cls;
  return ctx_create(env, p, r, rinv, devices);
}

JNIEXPORT void JNICALL CLIENT(ctxDestroy)(JNIEnv* env, jclass cls, jlong ctx) {
  (void)env;
  (void)cls;
  amphj_ctx_destroy(CTX(ctx));
}

/* DefaultAmphoraClient.verifyOutputDeliveryObjects :476-505 -> -1 or the failing word */
JNIEXPORT jlong JNICALL CLIENT(recombineVerify)(JNIEnv* env, jclass cls, jlong ctx, jobjectArray y,
                                                jobjectArray r, jobjectArray v, jobjectArray w, jobjectArray u,
                                                jbyteArray out) {
  (void)cls;
  jobjectArray f[5] = {y, r, v, w, u};
  Pin pins[5 * MAXP + 1];
  int n;
  if (refs_odo(env, f, pins, &n) || ref(env, out, &pins[5 * n])) return -1;
  const uint8_t* ptrs[5 * MAXP];
  size_t lens[5 * MAXP];
  int64_t fail = -1;
  Access acc;
  if (acquire(env, pins, 5 * n + 1, &acc)) return -1;
  ptrs_of(pins, 5 * n, ptrs, lens);
  const int st = amphj_recombine_verify(CTX(ctx), n, ptrs, lens, (uint8_t*)pins[5 * n].p,
                                        (size_t)pins[5 * n].len, &fail);
  release_access(env, pins, 5 * n + 1, 5 * n, &acc);
  if (st != AMPH_OK && st != AMPH_E_VERIFY) throw_status(env, st);
  return st == AMPH_E_VERIFY ? (jlong)fail : -1;
}

/* createSecret arithmetic :150-160: verify the mask ODOs + maskInput per word */
JNIEXPORT jlong JNICALL CLIENT(maskInput)(JNIEnv* env, jclass cls, jlong ctx, jobjectArray y, jobjectArray r,
                                          jobjectArray v, jobjectArray w, jobjectArray u, jbyteArray secrets,
                                          jbyteArray out) {
  (void)cls;
  jobjectArray f[5] = {y, r, v, w, u};
  Pin pins[5 * MAXP + 2];
  int n;
  if (refs_odo(env, f, pins, &n) || ref(env, secrets, &pins[5 * n]) || ref(env, out, &pins[5 * n + 1])) return -1;
  const uint8_t* ptrs[5 * MAXP];
  size_t lens[5 * MAXP];
  int64_t fail = -1;
  Access acc;
  if (acquire(env, pins, 5 * n + 2, &acc)) return -1;
  ptrs_of(pins, 5 * n, ptrs, lens);
  const int st = amphj_mask_input(CTX(ctx), n, ptrs, lens, (const uint8_t*)pins[5 * n].p, (size_t)pins[5 * n].len,
                                  (uint8_t*)pins[5 * n + 1].p, (size_t)pins[5 * n + 1].len, &fail);
  release_access(env, pins, 5 * n + 2, 5 * n + 1, &acc);
  if (st != AMPH_OK && st != AMPH_E_VERIFY) throw_status(env, st);
  return st == AMPH_E_VERIFY ? (jlong)fail : -1;
}

/* SecretShareUtil.recombineObject :70-90 */
JNIEXPORT void JNICALL CLIENT(recombine)(JNIEnv* env, jclass cls, jlong ctx, jobjectArray shares, jbyteArray out) {
  (void)cls;
  Pin pins[MAXP + 1];
  int n;
  if (refs_list(env, shares, pins, &n) || ref(env, out, &pins[n])) return;
  const uint8_t* ptrs[MAXP];
  size_t lens[MAXP];
  Access acc;
  if (acquire(env, pins, n + 1, &acc)) return;
  ptrs_of(pins, n, ptrs, lens);
  const int st = amphj_recombine(CTX(ctx), n, ptrs, lens, (uint8_t*)pins[n].p, (size_t)pins[n].len);
  release_access(env, pins, n + 1, n, &acc);
  if (st != AMPH_OK) throw_status(env, st);
}

/* SecretShareUtil.verifySecrets :102-141 over canonical LE16 arrays -> -1 or the failing word */
JNIEXPORT jlong JNICALL CLIENT(verify)(JNIEnv* env, jclass cls, jlong ctx, jbyteArray ys, jbyteArray rs,
                                       jbyteArray us, jbyteArray vs, jbyteArray ws) {
  (void)cls;
  Pin pins[5];
  jbyteArray a[5] = {ys, rs, us, vs, ws};
  for (int k = 0; k < 5; ++k)
    if (ref(env, a[k], &pins[k])) return -1;
  const uint8_t* ptrs[5];
  size_t lens[5];
  int64_t fail = -1;
  Access acc;
  if (acquire(env, pins, 5, &acc)) return -1;
  ptrs_of(pins, 5, ptrs, lens);
  const int st = amphj_verify(CTX(ctx), ptrs, lens, &fail);
  release_access(env, pins, 5, 5, &acc);
  if (st != AMPH_OK && st != AMPH_E_VERIFY) throw_status(env, st);
  return st == AMPH_E_VERIFY ? (jlong)fail : -1;
}

/* SecretShareUtil.maskInput :65-68 over canonical LE16 secrets and masks */
JNIEXPORT void JNICALL CLIENT(maskWords)(JNIEnv* env, jclass cls, jlong ctx, jbyteArray secrets, jbyteArray masks,
                                         jbyteArray out) {
  (void)cls;
  Pin pins[3];
  if (ref(env, secrets, &pins[0]) || ref(env, masks, &pins[1]) || ref(env, out, &pins[2])) return;
  Access acc;
  if (acquire(env, pins, 3, &acc)) return;
  const int st = amphj_mask_words(CTX(ctx), (const uint8_t*)pins[0].p, (size_t)pins[0].len,
                                  (const uint8_t*)pins[1].p, (size_t)pins[1].len, (uint8_t*)pins[2].p,
                                  (size_t)pins[2].len);
  release_access(env, pins, 3, 2, &acc);
  if (st != AMPH_OK) throw_status(env, st);
}

/* SecretShareUtil.maskInput :65-68 for ONE word, as DefaultAmphoraClient.java:155-160 calls it:
   16-byte region copies in and out (no critical region) and host arithmetic in
   libamphora_hip (amph_mask_word_host) -- no kernel launch per word */
JNIEXPORT jbyteArray JNICALL CLIENT(maskWord)(JNIEnv* env, jclass cls, jlong ctx, jbyteArray secret,
                                              jbyteArray mask) {
  (void)cls;
  Pin a[2];
  if (ref(env, secret, &a[0]) || ref(env, mask, &a[1])) return NULL;
  if (a[0].len != 16 || a[1].len != 16) return throw_arg(env, "maskWord takes two 16-byte words"), NULL;
  jbyte s[16], m[16], o[16];
  (*env)->GetByteArrayRegion(env, secret, 0, 16, s);
  (*env)->GetByteArrayRegion(env, mask, 0, 16, m);
  const int st = amphj_mask_word(CTX(ctx), (const uint8_t*)s, (const uint8_t*)m, (uint8_t*)o);
  if (st != AMPH_OK) {
    throw_status(env, st);
    return NULL;
  }
  jbyteArray out = (*env)->NewByteArray(env, 16);
  if (out) (*env)->SetByteArrayRegion(env, out, 0, 16, o);
  return out;
}

/* the IntegrityVerificationException text of SecretShareUtil.java:116-129 */
JNIEXPORT jstring JNICALL CLIENT(verifyMessage)(JNIEnv* env, jclass cls, jlong ctx, jbyteArray y, jbyteArray r,
                                                jbyteArray u, jbyteArray v, jbyteArray w) {
  (void)cls;
  jbyteArray a[5] = {y, r, u, v, w};
  jbyte b[5][16];
  for (int k = 0; k < 5; ++k) {
    if (!a[k] || (*env)->GetArrayLength(env, a[k]) != 16) return throw_arg(env, "16-byte words expected"), NULL;
    (*env)->GetByteArrayRegion(env, a[k], 0, 16, b[k]);
  }
  char buf[1024];
  const int st = amphj_verify_message(CTX(ctx), (const uint8_t*)b[0], (const uint8_t*)b[1], (const uint8_t*)b[2],
                                      (const uint8_t*)b[3], (const uint8_t*)b[4], buf, sizeof buf);
  if (st != AMPH_OK) {
    throw_status(env, st);
    return NULL;
  }
  return (*env)->NewStringUTF(env, buf);
}

/* getSecret straight from the five base64 strings per party (ASCII bytes) */
JNIEXPORT jlong JNICALL CLIENT(recombineVerifyB64)(JNIEnv* env, jclass cls, jlong ctx, jobjectArray y,
                                                   jobjectArray r, jobjectArray v, jobjectArray w, jobjectArray u,
                                                   jlong words, jbyteArray out) {
  (void)cls;
  jobjectArray f[5] = {y, r, v, w, u};
  Pin pins[5 * MAXP + 1];
  int n;
  if (words < 0) return throw_arg(env, "negative word count");
  if (refs_odo(env, f, pins, &n) || ref(env, out, &pins[5 * n])) return -1;
  const uint8_t* ptrs[5 * MAXP];
  size_t lens[5 * MAXP];
  int64_t fail = -1;
  if (pin_all(env, pins, 5 * n + 1)) return -1;
  ptrs_of(pins, 5 * n, ptrs, lens);
  const int st = amphj_recombine_verify_b64(CTX(ctx), n, (const char* const*)ptrs, lens, (size_t)words,
                                            (uint8_t*)pins[5 * n].p, (size_t)pins[5 * n].len, &fail);
  unpin_all(env, pins, 5 * n + 1, 5 * n);
  if (st != AMPH_OK && st != AMPH_E_VERIFY) throw_status(env, st);
  return st == AMPH_E_VERIFY ? (jlong)fail : -1;
}

/* createSecret from the /input-masks text: verify + mask + the 24-character MaskedInputData records */
JNIEXPORT jlong JNICALL CLIENT(maskInputB64)(JNIEnv* env, jclass cls, jlong ctx, jobjectArray y, jobjectArray r,
                                             jobjectArray v, jobjectArray w, jobjectArray u, jlong words,
                                             jbyteArray secrets, jbyteArray records) {
  (void)cls;
  jobjectArray f[5] = {y, r, v, w, u};
  Pin pins[5 * MAXP + 2];
  int n;
  if (words < 0) return throw_arg(env, "negative word count");
  if (refs_odo(env, f, pins, &n) || ref(env, secrets, &pins[5 * n]) || ref(env, records, &pins[5 * n + 1]))
    return -1;
  const uint8_t* ptrs[5 * MAXP];
  size_t lens[5 * MAXP];
  int64_t fail = -1;
  if (pin_all(env, pins, 5 * n + 2)) return -1;
  ptrs_of(pins, 5 * n, ptrs, lens);
  const int st = amphj_mask_input_b64(CTX(ctx), n, (const char* const*)ptrs, lens, (size_t)words,
                                      (const uint8_t*)pins[5 * n].p, (size_t)pins[5 * n].len,
                                      (char*)pins[5 * n + 1].p, (size_t)pins[5 * n + 1].len, &fail);
  unpin_all(env, pins, 5 * n + 2, 5 * n + 1);
  if (st != AMPH_OK && st != AMPH_E_VERIFY) throw_status(env, st);
  return st == AMPH_E_VERIFY ? (jlong)fail : -1;
}

/* ---- service ------------------------------------------------------------------ */
#define SERVICE(name) Java_io_carbynestack_amphora_service_calculation_NativeShareArithmetic_##name

JNIEXPORT jlong JNICALL SERVICE(ctxCreate)(JNIEnv* env, jclass cls, jbyteArray p, jbyteArray r,
                                           jbyteArray rinv, jintArray devices) {
  (void)cls;
  return ctx_create(env, p, r, rinv, devices);
}

JNIEXPORT void JNICALL SERVICE(ctxDestroy)(JNIEnv* env, jclass cls, jlong ctx) {
  (void)env;
  (void)cls;
  amphj_ctx_destroy(CTX(ctx));
}

/* SecretShareUtil.convertToSecretShare :58-107 -> SecretShare.data (32 B per word) */
JNIEXPORT void JNICALL SERVICE(convertShare)(JNIEnv* env, jclass cls, jlong ctx, jbyteArray masked,
                                             jbyteArray tuples, jbyteArray macKeyLe, jboolean useZeroInputAsData,
                                             jbyteArray out) {
  (void)cls;
  Pin pins[3], key;
  if (ref(env, masked, &pins[0]) || ref(env, tuples, &pins[1]) || ref(env, out, &pins[2]) ||
      ref(env, macKeyLe, &key))
    return;
  jbyte k16[16] = {0};  /* the key is read on this thread: a region copy, never a descriptor */
  if (key.len == 16) (*env)->GetByteArrayRegion(env, macKeyLe, 0, 16, k16);
  Access acc;
  if (acquire(env, pins, 3, &acc)) return;
  const int st = amphj_convert_share(CTX(ctx), (const uint8_t*)pins[0].p, (size_t)pins[0].len,
                                     (const uint8_t*)pins[1].p, (size_t)pins[1].len, (const uint8_t*)k16,
                                     (size_t)key.len, useZeroInputAsData ? 1 : 0, (uint8_t*)pins[2].p,
                                     (size_t)pins[2].len);
  release_access(env, pins, 3, 2, &acc);
  if (st != AMPH_OK) throw_status(env, st);
}

/* computeOutputDeliveryObject :100-139 + multiplyShares' local diffs :186-200 */
JNIEXPORT void JNICALL SERVICE(odoPre)(JNIEnv* env, jclass cls, jlong ctx, jbyteArray share, jint stride,
                                       jbyteArray masks, jbyteArray triples, jbyteArray y, jbyteArray r,
                                       jbyteArray v, jbyteArray mag, jbyteArray neg) {
  (void)cls;
  Pin pins[8];
  jbyteArray a[8] = {share, masks, triples, y, r, v, mag, neg};
  for (int i = 0; i < 8; ++i)
    if (ref(env, a[i], &pins[i])) return;
  if (pins[3].len != pins[4].len || pins[3].len != pins[5].len) {
    throw_arg(env, "The provided shares must be of the same length");
    return;
  }
  Access acc;
  if (acquire(env, pins, 8, &acc)) return;
  const int st = amphj_odo_pre(CTX(ctx), (const uint8_t*)pins[0].p, (size_t)pins[0].len, stride,
                               (const uint8_t*)pins[1].p, (size_t)pins[1].len, (const uint8_t*)pins[2].p,
                               (size_t)pins[2].len, (uint8_t*)pins[3].p, (uint8_t*)pins[4].p, (uint8_t*)pins[5].p,
                               (size_t)pins[3].len, (uint8_t*)pins[6].p, (size_t)pins[6].len, (uint8_t*)pins[7].p,
                               (size_t)pins[7].len);
  release_access(env, pins, 8, 3, &acc);
  if (st != AMPH_OK) throw_status(env, st);
}

/* recombineDiffs :231-272 + multiplySharedSecrets :274-286 + the w/u encoding :147-152 */
JNIEXPORT void JNICALL SERVICE(openPost)(JNIEnv* env, jclass cls, jlong ctx, jobjectArray mags, jobjectArray negs,
                                         jbyteArray triples, jboolean isPlayer0, jbyteArray w, jbyteArray u) {
  (void)cls;
  Pin pins[2 * MAXP + 3];
  int n, n2;
  if (refs_list(env, mags, pins, &n) || refs_list(env, negs, pins + n, &n2)) return;
  if (n2 != n) {
    throw_arg(env, "one sign array per magnitude array");
    return;
  }
  if (ref(env, triples, &pins[2 * n]) || ref(env, w, &pins[2 * n + 1]) || ref(env, u, &pins[2 * n + 2])) return;
  if (pins[2 * n + 1].len != pins[2 * n + 2].len) {
    throw_arg(env, "The provided shares must be of the same length");
    return;
  }
  const uint8_t* ptrs[2 * MAXP];
  size_t lens[2 * MAXP];
  Access acc;
  if (acquire(env, pins, 2 * n + 3, &acc)) return;
  ptrs_of(pins, 2 * n, ptrs, lens);
  const int st = amphj_open_post(CTX(ctx), n, ptrs, lens, ptrs + n, lens + n, (const uint8_t*)pins[2 * n].p,
                                 (size_t)pins[2 * n].len, isPlayer0 ? 1 : 0, (uint8_t*)pins[2 * n + 1].p,
                                 (uint8_t*)pins[2 * n + 2].p, (size_t)pins[2 * n + 1].len);
  release_access(env, pins, 2 * n + 3, 2 * n + 1, &acc);
  if (st != AMPH_OK) throw_status(env, st);
}

/* MultiplicationExchangeObject.interimValues: signed diffs -> the JSON array text Jackson writes */
JNIEXPORT jbyteArray JNICALL SERVICE(exchangeEncode)(JNIEnv* env, jclass cls, jlong ctx, jbyteArray mag,
                                                     jbyteArray neg) {
  (void)cls;
  Pin pins[2];
  if (ref(env, mag, &pins[0]) || ref(env, neg, &pins[1])) return NULL;
  const size_t cap = amphj_exchange_max_chars((size_t)pins[0].len / 32);
  char* text = (char*)malloc(cap ? cap : 1);
  if (!text) {
    jclass c = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
    if (c) (*env)->ThrowNew(env, c, "exchange text");
    return NULL;
  }
  uint64_t len = 0;
  if (pin_all(env, pins, 2)) {
    free(text);
    return NULL;
  }
  const int st = amphj_exchange_encode(CTX(ctx), (const uint8_t*)pins[0].p, (size_t)pins[0].len,
                                       (const uint8_t*)pins[1].p, (size_t)pins[1].len, text, cap, &len);
  unpin_all(env, pins, 2, 2);
  jbyteArray out = NULL;
  if (st != AMPH_OK) {
    throw_status(env, st);
  } else if (len > 0x7FFFFFFFull) {
    throw_arg(env, "the exchange text exceeds a Java array (2^31 - 1 bytes)");
  } else {
    out = (*env)->NewByteArray(env, (jsize)len);
    if (out) (*env)->SetByteArrayRegion(env, out, 0, (jsize)len, (const jbyte*)text);
  }
  free(text);
  return out;
}

/* the interimValues array span of a received body -> signed diffs */
JNIEXPORT void JNICALL SERVICE(exchangeDecode)(JNIEnv* env, jclass cls, jlong ctx, jbyteArray body, jint off,
                                               jint len, jlong npairs, jbyteArray mag, jbyteArray neg) {
  (void)cls;
  Pin pins[3];
  if (ref(env, body, &pins[0]) || ref(env, mag, &pins[1]) || ref(env, neg, &pins[2])) return;
  if (off < 0 || len < 0 || (jlong)off + len > pins[0].len || npairs < 0) {
    throw_arg(env, "interimValues span outside the body");
    return;
  }
  if (pin_all(env, pins, 3)) return;
  const int st = amphj_exchange_decode(CTX(ctx), (const char*)pins[0].p + off, (size_t)len, (size_t)npairs,
                                       (uint8_t*)pins[1].p, (size_t)pins[1].len, (uint8_t*)pins[2].p,
                                       (size_t)pins[2].len);
  unpin_all(env, pins, 3, 1);
  if (st != AMPH_OK) throw_status(env, st);
}

/* ---- service: one request's Output Delivery with device-resident state ------------- */
/* an optional array: NULL stays NULL (len 0) */
static int ref_opt(JNIEnv* env, jbyteArray a, Pin* p) {
  if (!a) {
    p->ref = NULL;
    p->len = 0;
    p->p = NULL;
    return 0;
  }
  return ref(env, a, p);
}

/* pins only the arrays that are present */
static int pin_present(JNIEnv* env, Pin* pins, int count) {
  for (int i = 0; i < count; ++i) {
    if (!pins[i].ref) continue;
    pins[i].p = (*env)->GetPrimitiveArrayCritical(env, pins[i].ref, NULL);
    if (!pins[i].p) {
      unpin_all(env, pins, i, i);
      return -1;
    }
  }
  return 0;
}

/* computeOutputDeliveryObject :100-139 + multiplyShares :186-200 -> a session handle
   (y, r, v: null, or the secretShares / rShares / vShares arrays to fill) */
JNIEXPORT jlong JNICALL SERVICE(partyBegin)(JNIEnv* env, jclass cls, jlong ctx, jbyteArray share, jint stride,
                                            jbyteArray masks, jbyteArray triples, jint nParties, jbyteArray y,
                                            jbyteArray r, jbyteArray v) {
  (void)cls;
  Pin pins[6];
  if (ref(env, share, &pins[0]) || ref(env, masks, &pins[1]) || ref(env, triples, &pins[2]) ||
      ref_opt(env, y, &pins[3]) || ref_opt(env, r, &pins[4]) || ref_opt(env, v, &pins[5]))
    return 0;
  if (pins[3].len != pins[4].len || pins[3].len != pins[5].len) {
    throw_arg(env, "The provided shares must be of the same length");
    return 0;
  }
  const int staged = total_len(pins, 6) > region_bytes();
  if (staged ? stage_native(env, pins, 6, 3) : pin_present(env, pins, 6)) return 0;
  void* session = NULL;
  const int st = amphj_party_begin(CTX(ctx), (const uint8_t*)pins[0].p, (size_t)pins[0].len, stride,
                                   (const uint8_t*)pins[1].p, (size_t)pins[1].len, (const uint8_t*)pins[2].p,
                                   (size_t)pins[2].len, nParties, (uint8_t*)pins[3].p, (uint8_t*)pins[4].p,
                                   (uint8_t*)pins[5].p, (size_t)pins[3].len, &session);
  if (staged) unstage_native(env, pins, 6, 3, st == AMPH_OK);
  else unpin_all(env, pins, 6, 3);
  if (st != AMPH_OK) {
    throw_status(env, st);
    return 0;
  }
  return (jlong)(intptr_t)session;
}

/* this party's MultiplicationExchangeObject.interimValues, as the JSON array text */
JNIEXPORT jbyteArray JNICALL SERVICE(partyText)(JNIEnv* env, jclass cls, jlong session) {
  (void)cls;
  if (!session) return throw_arg(env, "null party session"), NULL;
  const uint64_t len = amphj_party_text_len(CTX(session));
  if (len > 0x7FFFFFFFull) return throw_arg(env, "the exchange text exceeds a Java array (2^31 - 1 bytes)"), NULL;
  jbyteArray out = (*env)->NewByteArray(env, (jsize)len);
  if (!out) return NULL; /* OutOfMemoryError pending */
  Pin pin;
  if (ref(env, out, &pin)) return NULL;
  const int staged = (size_t)pin.len > region_bytes();
  if (staged ? stage_native(env, &pin, 1, 0) : pin_all(env, &pin, 1)) return NULL;
  const int st = amphj_party_text(CTX(session), (char*)pin.p, (size_t)pin.len);
  if (staged) unstage_native(env, &pin, 1, 0, st == AMPH_OK);
  else unpin_all(env, &pin, 1, 0);
  if (st != AMPH_OK) {
    throw_status(env, st);
    return NULL;
  }
  return out;
}

/* a partner's interimValues span of its received body (recombineDiffs' input :231-272) */
JNIEXPORT void JNICALL SERVICE(partyPartner)(JNIEnv* env, jclass cls, jlong session, jint slot, jbyteArray body,
                                             jint off, jint len) {
  (void)cls;
  Pin pin;
  if (ref(env, body, &pin)) return;
  if (off < 0 || len < 0 || (jlong)off + len > pin.len) {
    throw_arg(env, "interimValues span outside the body");
    return;
  }
  /* above the threshold only the interimValues span is copied out of the body */
  const int staged = (size_t)len > region_bytes();
  Pin span = {pin.ref, len, NULL};
  const char* text;
  if (staged) {
    span.p = (jbyte*)malloc(len ? (size_t)len : 1);
    if (!span.p) {
      jclass c = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
      if (c) (*env)->ThrowNew(env, c, "native staging of a Java array");
      return;
    }
    (*env)->GetByteArrayRegion(env, body, off, len, span.p);
    text = (const char*)span.p;
  } else {
    if (pin_all(env, &pin, 1)) return;
    text = (const char*)pin.p + off;
  }
  const int st = amphj_party_partner(CTX(session), slot, text, (size_t)len);
  if (staged) free(span.p);
  else unpin_all(env, &pin, 1, 1);
  if (st != AMPH_OK) throw_status(env, st);
}

/* recombineDiffs + multiplySharedSecrets + the w/u encoding :147-152, :231-286 */
JNIEXPORT void JNICALL SERVICE(partyFinish)(JNIEnv* env, jclass cls, jlong session, jboolean isPlayer0,
                                            jbyteArray w, jbyteArray u) {
  (void)cls;
  Pin pins[2];
  if (ref(env, w, &pins[0]) || ref(env, u, &pins[1])) return;
  if (pins[0].len != pins[1].len) {
    throw_arg(env, "The provided shares must be of the same length");
    return;
  }
  const int staged = total_len(pins, 2) > region_bytes();
  if (staged ? stage_native(env, pins, 2, 0) : pin_all(env, pins, 2)) return;
  const int st = amphj_party_finish(CTX(session), isPlayer0 ? 1 : 0, (uint8_t*)pins[0].p, (uint8_t*)pins[1].p,
                                    (size_t)pins[0].len);
  if (staged) unstage_native(env, pins, 2, 0, st == AMPH_OK);
  else unpin_all(env, pins, 2, 0);
  if (st != AMPH_OK) throw_status(env, st);
}

/* the same, with all five ODO fields returned as base64 (ASCII) in fields[0..4] */
JNIEXPORT void JNICALL SERVICE(partyFinishBase64)(JNIEnv* env, jclass cls, jlong session, jboolean isPlayer0,
                                                  jobjectArray fields) {
  (void)cls;
  Pin pins[5];
  int n;
  if (refs_list(env, fields, pins, &n)) return;
  if (n != 5) {
    throw_arg(env, "five field arrays: secretShares, rShares, vShares, wShares, uShares");
    return;
  }
  const int staged = total_len(pins, 5) > region_bytes();
  if (staged ? stage_native(env, pins, 5, 0) : pin_all(env, pins, 5)) return;
  char* ptrs[5];
  size_t lens[5];
  for (int k = 0; k < 5; ++k) {
    ptrs[k] = (char*)pins[k].p;
    lens[k] = (size_t)pins[k].len;
  }
  const int st = amphj_party_finish_b64(CTX(session), isPlayer0 ? 1 : 0, ptrs, lens);
  if (staged) unstage_native(env, pins, 5, 0, st == AMPH_OK);
  else unpin_all(env, pins, 5, 0);
  if (st != AMPH_OK) throw_status(env, st);
}

JNIEXPORT void JNICALL SERVICE(partyFree)(JNIEnv* env, jclass cls, jlong session) {
  (void)env;
  (void)cls;
  amphj_party_free(CTX(session));
}

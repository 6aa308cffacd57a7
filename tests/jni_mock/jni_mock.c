/*
 * TEST HARNESS ONLY: a mock JNIEnv over plain C arrays (see jni.h here).
 * Built with jni/amphora_jni.c and jni/amphora_jni_core.c into
 * libjni_mock.so, which tests/test_jni_core.py drives through ctypes: Java
 * arrays are made with mock_bytes / mock_objects, the Java_* entry points are
 * called with mock_env(), and the mock records the thrown exception, the
 * release mode of every pinned array, and any JNI call made inside a
 * critical region (a JNI rule the layer must keep).
 */
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { KIND_BYTES = 1, KIND_INTS, KIND_OBJECTS, KIND_CLASS, KIND_STRING };

struct mock_obj {
  int kind;
  jsize len;
  void* data;          /* bytes / ints / jobject* / char* */
  int pinned;          /* open critical pins of this array */
  int released_commit; /* releases with mode 0 (copy back) */
  int released_abort;  /* releases with JNI_ABORT */
  struct mock_obj* next;
};

static struct mock_obj* g_all;
static int g_critical;    /* open critical regions */
static int g_violations;  /* JNI calls made inside one (or from an unattached thread) */
static char g_exc_class[256];
static char g_exc_msg[1024];
static int g_local;          /* local references made in this native call */
static int g_capacity = 16;  /* the JNI guarantee, or what EnsureLocalCapacity reserved */
static int g_ref_overflows;  /* local references beyond it */
static int g_fail_pin;       /* > 0: the g_fail_pin-th pin from now returns NULL */
static int g_pins;           /* critical pins taken since mock_clear */
/* region-copy callbacks run on the library's staging threads: atomics */
static long g_region_copies; /* Get/SetByteArrayRegion calls since mock_clear */
static int g_attaches;       /* threads attached to the mock VM */
static int g_detaches;       /* ... and detached again (at their exit) */
static int g_bad_detaches;   /* DetachCurrentThread on the calling "Java" thread */
static int g_global_refs;    /* live global references */
static int g_foreign_regions; /* region copies made on threads other than mock_env()'s */
static __thread int t_attached;

static struct mock_obj* obj_new(int kind, jsize len, size_t elem) {
  struct mock_obj* o = (struct mock_obj*)calloc(1, sizeof *o);
  o->kind = kind;
  o->len = len;
  o->data = calloc(len > 0 ? (size_t)len : 1, elem);
  o->next = g_all;
  g_all = o;
  return o;
}

static void outside_critical(void) {
  if (g_critical) ++g_violations;
}

static void new_local(void) {
  if (++g_local > g_capacity) ++g_ref_overflows;
}

static void pending(const char* cls, const char* msg) {
  if (!g_exc_class[0]) {  /* the first pending exception wins, as in a JVM */
    strncpy(g_exc_class, cls, sizeof g_exc_class - 1);
    strncpy(g_exc_msg, msg ? msg : "", sizeof g_exc_msg - 1);
  }
}

static jclass m_FindClass(JNIEnv* env, const char* name) {
  (void)env;
  outside_critical();
  struct mock_obj* o = obj_new(KIND_CLASS, (jsize)strlen(name) + 1, 1);
  memcpy(o->data, name, strlen(name) + 1);
  new_local();
  return o;
}

static jint m_ThrowNew(JNIEnv* env, jclass c, const char* msg) {
  (void)env;
  outside_critical();
  pending((const char*)c->data, msg);
  return 0;
}

static jsize m_GetArrayLength(JNIEnv* env, jarray a) {
  (void)env;
  outside_critical();
  return a->len;
}

static jobject m_GetObjectArrayElement(JNIEnv* env, jobjectArray a, jsize i) {
  (void)env;
  outside_critical();
  new_local();
  return (i >= 0 && i < a->len) ? ((jobject*)a->data)[i] : NULL;
}

static void* m_GetPrimitiveArrayCritical(JNIEnv* env, jarray a, jboolean* is_copy) {
  (void)env;
  if (is_copy) *is_copy = JNI_FALSE;
  if (g_fail_pin > 0 && --g_fail_pin == 0) {  /* as a JVM out of memory: NULL + a pending error */
    pending("java/lang/OutOfMemoryError", "mock: pin refused");
    return NULL;
  }
  ++g_critical;
  ++g_pins;
  ++a->pinned;
  return a->data;
}

static void m_ReleasePrimitiveArrayCritical(JNIEnv* env, jarray a, void* p, jint mode) {
  (void)env;
  (void)p;
  --g_critical;
  --a->pinned;
  if (mode == JNI_ABORT) ++a->released_abort;
  else ++a->released_commit;
}

static void m_GetIntArrayRegion(JNIEnv* env, jintArray a, jsize start, jsize len, jint* buf) {
  (void)env;
  outside_critical();
  memcpy(buf, (jint*)a->data + start, (size_t)len * sizeof(jint));
}

static void region_call(void) {
  __atomic_fetch_add(&g_region_copies, 1, __ATOMIC_RELAXED);
  if (!t_attached) __atomic_fetch_add(&g_violations, 1, __ATOMIC_RELAXED); /* JNI from an unattached thread */
  if (t_attached == 2) __atomic_fetch_add(&g_foreign_regions, 1, __ATOMIC_RELAXED);
}

static void m_GetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize start, jsize len, jbyte* buf) {
  (void)env;
  outside_critical();
  region_call();
  if (start < 0 || len < 0 || start + len > a->len) {
    pending("java/lang/ArrayIndexOutOfBoundsException", "mock: region outside the array");
    return;
  }
  memcpy(buf, (jbyte*)a->data + start, (size_t)len);
}

static void m_SetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize start, jsize len, const jbyte* buf) {
  (void)env;
  outside_critical();
  region_call();
  if (start < 0 || len < 0 || start + len > a->len) {
    pending("java/lang/ArrayIndexOutOfBoundsException", "mock: region outside the array");
    return;
  }
  memcpy((jbyte*)a->data + start, buf, (size_t)len);
}

static jbyteArray m_NewByteArray(JNIEnv* env, jsize len) {
  (void)env;
  outside_critical();
  new_local();
  return obj_new(KIND_BYTES, len, 1);
}

static jstring m_NewStringUTF(JNIEnv* env, const char* s) {
  (void)env;
  outside_critical();
  struct mock_obj* o = obj_new(KIND_STRING, (jsize)strlen(s), 1);
  free(o->data);
  o->data = strdup(s);
  new_local();
  return o;
}

static jint m_EnsureLocalCapacity(JNIEnv* env, jint n) {
  (void)env;
  outside_critical();
  if (g_local + n > g_capacity) g_capacity = g_local + n;
  return 0;
}

static JNIEnv g_env;
static JavaVM g_vm;

static jint m_GetJavaVM(JNIEnv* env, JavaVM** vm) {
  (void)env;
  outside_critical();
  *vm = &g_vm;
  return 0;
}

static jobject m_NewGlobalRef(JNIEnv* env, jobject o) {
  (void)env;
  outside_critical();
  __atomic_fetch_add(&g_global_refs, 1, __ATOMIC_RELAXED);
  return o;
}

static void m_DeleteGlobalRef(JNIEnv* env, jobject o) {
  (void)env;
  (void)o;
  outside_critical();
  __atomic_fetch_sub(&g_global_refs, 1, __ATOMIC_RELAXED);
}

static jboolean m_ExceptionCheck(JNIEnv* env) {
  (void)env;
  return g_exc_class[0] ? JNI_TRUE : JNI_FALSE;
}

static void m_ExceptionClear(JNIEnv* env) {
  (void)env;
  g_exc_class[0] = g_exc_msg[0] = 0;
}

static jint vm_GetEnv(JavaVM* vm, void** penv, jint version) {
  (void)vm;
  (void)version;
  if (!t_attached) return JNI_EDETACHED;
  *penv = &g_env;
  return JNI_OK;
}

static jint vm_AttachCurrentThreadAsDaemon(JavaVM* vm, void** penv, void* args) {
  (void)vm;
  (void)args;
  if (!t_attached) {
    t_attached = 2; /* a native thread the layer attached */
    __atomic_fetch_add(&g_attaches, 1, __ATOMIC_RELAXED);
  }
  *penv = &g_env;
  return JNI_OK;
}

static const struct JNINativeInterface_ g_table = {
    m_FindClass,          m_ThrowNew,          m_GetArrayLength,     m_GetObjectArrayElement,
    m_GetPrimitiveArrayCritical, m_ReleasePrimitiveArrayCritical, m_GetIntArrayRegion,
    m_GetByteArrayRegion, m_SetByteArrayRegion, m_NewByteArray,      m_NewStringUTF,
    m_EnsureLocalCapacity, m_GetJavaVM,        m_NewGlobalRef,       m_DeleteGlobalRef,
    m_ExceptionCheck,     m_ExceptionClear,
};
static jint vm_DetachCurrentThread(JavaVM* vm) {
  (void)vm;
  if (t_attached == 1) __atomic_fetch_add(&g_bad_detaches, 1, __ATOMIC_RELAXED); /* the Java thread itself */
  if (t_attached == 2) __atomic_fetch_add(&g_detaches, 1, __ATOMIC_RELAXED);
  t_attached = 0;
  return JNI_OK;
}

static const struct JNIInvokeInterface_ g_vm_table = {vm_GetEnv, vm_AttachCurrentThreadAsDaemon,
                                                      vm_DetachCurrentThread};
static JNIEnv g_env = &g_table;
static JavaVM g_vm = &g_vm_table;

/* ---- harness API (ctypes) ---- */
JNIEXPORT JNIEnv* mock_env(void) {
  t_attached = 1; /* the "Java" thread that calls the entry points */
  return &g_env;
}

JNIEXPORT jobject mock_bytes(const uint8_t* data, jsize len) {
  struct mock_obj* o = obj_new(KIND_BYTES, len, 1);
  if (data && len) memcpy(o->data, data, (size_t)len);
  return o;
}

JNIEXPORT jobject mock_ints(const int32_t* data, jsize len) {
  struct mock_obj* o = obj_new(KIND_INTS, len, sizeof(jint));
  if (data && len) memcpy(o->data, data, (size_t)len * sizeof(jint));
  return o;
}

JNIEXPORT jobject mock_objects(jobject* elems, jsize len) {
  struct mock_obj* o = obj_new(KIND_OBJECTS, len, sizeof(jobject));
  memcpy(o->data, elems, (size_t)len * sizeof(jobject));
  return o;
}

JNIEXPORT jsize mock_len(jobject o) { return o ? o->len : -1; }
JNIEXPORT const void* mock_data(jobject o) { return o ? o->data : NULL; }
JNIEXPORT int mock_commits(jobject o) { return o->released_commit; }
JNIEXPORT int mock_aborts(jobject o) { return o->released_abort; }
JNIEXPORT const char* mock_exception_class(void) { return g_exc_class; }
JNIEXPORT const char* mock_exception_message(void) { return g_exc_msg; }
JNIEXPORT int mock_violations(void) { return g_violations; }
JNIEXPORT int mock_open_criticals(void) { return g_critical; }
JNIEXPORT int mock_ref_overflows(void) { return g_ref_overflows; }
JNIEXPORT void mock_fail_pin(int k) { g_fail_pin = k; }
JNIEXPORT int mock_pins(void) { return g_pins; }
JNIEXPORT long mock_region_copies(void) { return __atomic_load_n(&g_region_copies, __ATOMIC_RELAXED); }
JNIEXPORT int mock_foreign_regions(void) { return __atomic_load_n(&g_foreign_regions, __ATOMIC_RELAXED); }
JNIEXPORT int mock_attaches(void) { return __atomic_load_n(&g_attaches, __ATOMIC_RELAXED); }
JNIEXPORT int mock_detaches(void) { return __atomic_load_n(&g_detaches, __ATOMIC_RELAXED); }
JNIEXPORT int mock_bad_detaches(void) { return __atomic_load_n(&g_bad_detaches, __ATOMIC_RELAXED); }
JNIEXPORT int mock_global_refs(void) { return __atomic_load_n(&g_global_refs, __ATOMIC_RELAXED); }

JNIEXPORT void mock_clear(void) {
  g_exc_class[0] = g_exc_msg[0] = 0;
  g_violations = 0;
  g_local = 0;  /* a new native call */
  g_capacity = 16;
  g_ref_overflows = 0;
  g_fail_pin = 0;
  g_pins = 0;
  __atomic_store_n(&g_region_copies, 0, __ATOMIC_RELAXED);
  __atomic_store_n(&g_foreign_regions, 0, __ATOMIC_RELAXED);
}

JNIEXPORT void mock_free_all(void) {
  while (g_all) {
    struct mock_obj* n = g_all->next;
    free(g_all->data);
    free(g_all);
    g_all = n;
  }
  g_critical = 0;
  mock_clear();
}

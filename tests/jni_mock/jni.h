/*
 * TEST HARNESS ONLY -- a mock of the JNI surface jni/amphora_jni.c uses, so
 * the JNI layer compiles and RUNS without a JDK (none exists in this image).
 * Not the JDK's jni.h: same type names and call syntax ((*env)->Fn(env, ...)),
 * but the function table holds only the entries amphora_jni.c calls and is
 * not layout-compatible with a JVM.  The entries are implemented by
 * jni_mock.c over plain C arrays, which also checks the JNI rule that no
 * other JNI function is called inside a Get/ReleasePrimitiveArrayCritical
 * region, that at most 16 local references (or what EnsureLocalCapacity
 * reserved) are live in one native call, and lets a test make a pin fail.
 * The JavaVM half (GetEnv / AttachCurrentThreadAsDaemon / DetachCurrentThread)
 * lets the region-copy callbacks run on libamphora_hip's staging threads, which
 * attach as daemons and must detach before they exit.
 * The real build (jni/Makefile) uses $JAVA_HOME/include/jni.h.
 */
#ifndef JNI_MOCK_H_
#define JNI_MOCK_H_

#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_ABORT 2
#define JNI_OK 0
#define JNI_EDETACHED (-2)
#define JNI_VERSION_1_6 0x00010006

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef jint jsize;

typedef struct mock_obj* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jobjectArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;
struct JNIInvokeInterface_;
typedef const struct JNIInvokeInterface_* JavaVM;

struct JNIInvokeInterface_ {
  jint (*GetEnv)(JavaVM*, void**, jint);
  jint (*AttachCurrentThreadAsDaemon)(JavaVM*, void**, void*);
  jint (*DetachCurrentThread)(JavaVM*);
};

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv*, const char*);
  jint (*ThrowNew)(JNIEnv*, jclass, const char*);
  jsize (*GetArrayLength)(JNIEnv*, jarray);
  jobject (*GetObjectArrayElement)(JNIEnv*, jobjectArray, jsize);
  void* (*GetPrimitiveArrayCritical)(JNIEnv*, jarray, jboolean*);
  void (*ReleasePrimitiveArrayCritical)(JNIEnv*, jarray, void*, jint);
  void (*GetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, jint*);
  void (*GetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*);
  void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*);
  jbyteArray (*NewByteArray)(JNIEnv*, jsize);
  jstring (*NewStringUTF)(JNIEnv*, const char*);
  jint (*EnsureLocalCapacity)(JNIEnv*, jint);
  jint (*GetJavaVM)(JNIEnv*, JavaVM**);
  jobject (*NewGlobalRef)(JNIEnv*, jobject);
  void (*DeleteGlobalRef)(JNIEnv*, jobject);
  jboolean (*ExceptionCheck)(JNIEnv*);
  void (*ExceptionClear)(JNIEnv*);
};

#endif /* JNI_MOCK_H_ */

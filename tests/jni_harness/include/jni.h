/*
 * jni.h -- TEST HARNESS ONLY.  Neither this container nor the GPU box has a JDK, so the real
 * <jni.h> is absent.  This header declares the subset of the JNI interface that
 * recommendation-models_amd/jni/rmx_jni.c uses, with the JNI specification's type and function
 * names, so the shim compiles and can be driven by fake_jni.c (an in-process stand-in for the JVM's
 * array and exception functions, NOT a JVM).  The function-table layout is NOT the real JNI one:
 * a librmx_jni.so for a JVM must be built against the JDK's jni.h.
 */
#ifndef RMX_FAKE_JNI_H
#define RMX_FAKE_JNI_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;
typedef uint8_t jboolean;

typedef struct fake_obj* jobject;
typedef jobject jclass;
typedef jobject jarray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jfloatArray;
typedef jarray jbyteArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv* env, const char* name);
  jint (*ThrowNew)(JNIEnv* env, jclass cls, const char* msg);
  jsize (*GetArrayLength)(JNIEnv* env, jarray a);
  jint* (*GetIntArrayElements)(JNIEnv* env, jintArray a, jboolean* is_copy);
  void (*ReleaseIntArrayElements)(JNIEnv* env, jintArray a, jint* p, jint mode);
  void* (*GetPrimitiveArrayCritical)(JNIEnv* env, jarray a, jboolean* is_copy);
  void (*ReleasePrimitiveArrayCritical)(JNIEnv* env, jarray a, void* p, jint mode);
  jintArray (*NewIntArray)(JNIEnv* env, jsize n);
  jfloatArray (*NewFloatArray)(JNIEnv* env, jsize n);
  jbyteArray (*NewByteArray)(JNIEnv* env, jsize n);
  void (*GetByteArrayRegion)(JNIEnv* env, jbyteArray a, jsize start, jsize n, jbyte* buf);
  void (*SetByteArrayRegion)(JNIEnv* env, jbyteArray a, jsize start, jsize n, const jbyte* buf);
};
#endif

/*
 * jni.h — a MINIMAL stand-in for the JDK header, test infrastructure only (tests/test_jni_shim.py).
 * This container has no JDK; the stand-in declares exactly the JNI types and the JNIEnv function
 * table entries jni/stcjni.c uses, with the JNI specification's signatures (C binding: JNIEnv is a
 * pointer to the function table), so that the shim can be type-checked with gcc and exercised
 * against a mock JNIEnv (tests/jni_stub/mock_env.c).  The table's layout is NOT the JDK's: a shim
 * built against it must never be loaded by a JVM.
 */
#ifndef STC_TEST_JNI_H_
#define STC_TEST_JNI_H_
#include <stdint.h>

typedef int32_t jint;
typedef long jlong; /* LP64, as the JDK's linux jni_md.h */
typedef signed char jbyte;
typedef unsigned char jboolean;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jdoubleArray;

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv*, const char*);
  jint (*ThrowNew)(JNIEnv*, jclass, const char*);
  jboolean (*ExceptionCheck)(JNIEnv*);
  jsize (*GetArrayLength)(JNIEnv*, jarray);
  jstring (*NewStringUTF)(JNIEnv*, const char*);
  jbyteArray (*NewByteArray)(JNIEnv*, jsize);
  jlongArray (*NewLongArray)(JNIEnv*, jsize);
  jdoubleArray (*NewDoubleArray)(JNIEnv*, jsize);
  jbyte* (*GetByteArrayElements)(JNIEnv*, jbyteArray, jboolean*);
  jint* (*GetIntArrayElements)(JNIEnv*, jintArray, jboolean*);
  jlong* (*GetLongArrayElements)(JNIEnv*, jlongArray, jboolean*);
  jdouble* (*GetDoubleArrayElements)(JNIEnv*, jdoubleArray, jboolean*);
  void (*ReleaseByteArrayElements)(JNIEnv*, jbyteArray, jbyte*, jint);
  void (*ReleaseIntArrayElements)(JNIEnv*, jintArray, jint*, jint);
  void (*ReleaseLongArrayElements)(JNIEnv*, jlongArray, jlong*, jint);
  void (*ReleaseDoubleArrayElements)(JNIEnv*, jdoubleArray, jdouble*, jint);
  void (*GetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*);
  void (*GetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, jlong*);
  void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*);
  void (*SetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, const jlong*);
  void (*SetDoubleArrayRegion)(JNIEnv*, jdoubleArray, jsize, jsize, const jdouble*);
};
#endif

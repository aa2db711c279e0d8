/* jni.h -- TEST-ONLY declaration of the JNI C types and of the JNIEnv functions that
 * jni/vectorwave_amd_jni.c calls, so the glue compiles and runs without a JDK (none is installed in this
 * image).  Names, argument types and const-ness follow the JNI specification's C binding (JDK 21
 * jni.h / jni_md.h on LP64 Linux); the function table holds only the entries the glue uses, so this header
 * proves source compatibility of the glue's calls, not binary layout.  tests/jni_harness/harness.c
 * implements the table over plain C arrays.  Not used by any product build: jni/Makefile compiles the glue
 * against $JAVA_HOME/include. */
#ifndef VW_TEST_JNI_H
#define VW_TEST_JNI_H

#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1

typedef unsigned char jboolean;
typedef signed char jbyte;
typedef unsigned short jchar;
typedef short jshort;
typedef int jint;
typedef long jlong;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject *jobject;
typedef jobject jclass;
typedef jobject jthrowable;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jdoubleArray;
typedef jarray jlongArray;
typedef jarray jobjectArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;

struct JNINativeInterface_ {
  jclass (JNICALL *FindClass)(JNIEnv *env, const char *name);
  jint (JNICALL *ThrowNew)(JNIEnv *env, jclass clazz, const char *msg);
  jboolean (JNICALL *ExceptionCheck)(JNIEnv *env);
  void (JNICALL *DeleteLocalRef)(JNIEnv *env, jobject obj);
  jstring (JNICALL *NewStringUTF)(JNIEnv *env, const char *utf);
  jsize (JNICALL *GetArrayLength)(JNIEnv *env, jarray array);
  jobject (JNICALL *GetObjectArrayElement)(JNIEnv *env, jobjectArray array, jsize index);
  void (JNICALL *GetLongArrayRegion)(JNIEnv *env, jlongArray array, jsize start, jsize len, jlong *buf);
  void (JNICALL *GetDoubleArrayRegion)(JNIEnv *env, jdoubleArray array, jsize start, jsize len, jdouble *buf);
  void (JNICALL *SetDoubleArrayRegion)(JNIEnv *env, jdoubleArray array, jsize start, jsize len, const jdouble *buf);
  void *(JNICALL *GetDirectBufferAddress)(JNIEnv *env, jobject buf);
  jlong (JNICALL *GetDirectBufferCapacity)(JNIEnv *env, jobject buf);
};

#endif

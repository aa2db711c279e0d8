/* harness.c -- TEST INFRASTRUCTURE: a fake JNIEnv over plain C arrays, so tests/test_jni_glue.py can call the
 * JNI glue (jni/vectorwave_amd_jni.c, compiled into the same library) through ctypes with no JVM.
 *
 * Java objects are h_obj records: double[] / long[] (data points at the caller's memory, e.g. a numpy row),
 * Object[] (an array of h_obj pointers), direct ByteBuffers, classes and strings.  The table enforces what
 * the JNI specification requires of a caller and what a JVM would do:
 *   - Get/Set<Type>ArrayRegion and GetObjectArrayElement out of range raise ArrayIndexOutOfBoundsException
 *     (pending, nothing copied);
 *   - calling any function but ExceptionCheck / DeleteLocalRef with an exception pending is counted as a
 *     misuse (h_misuse), and so is a wrong object kind;
 *   - local references from GetObjectArrayElement are counted (live and peak: the JNI guarantees 16).
 * ThrowNew / FindClass record the pending exception as "class: message" (h_pending). */
#include <jni.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { K_DOUBLES = 1, K_LONGS, K_OBJECTS, K_DIRECT, K_CLASS, K_STRING };

struct _jobject {
  int kind;
  jsize len;
  void *data;    /* doubles / longs / h_obj* array / direct memory / string text */
  jlong cap;     /* direct buffer capacity in bytes */
  char name[96]; /* class name */
};

static char g_pending[512];
static int g_has_pending;
static int g_misuse;
static long g_live_refs, g_peak_refs;

static void raise_(const char *cls, const char *msg) {
  if (g_has_pending) return;
  snprintf(g_pending, sizeof g_pending, "%s: %s", cls, msg);
  g_has_pending = 1;
}

/* every function but ExceptionCheck / DeleteLocalRef: no exception may be pending, object of the right kind */
static int guard(jobject o, int kind) {
  if (g_has_pending) { ++g_misuse; return 0; }
  if (kind && (!o || o->kind != kind)) { ++g_misuse; return 0; }
  return 1;
}

static jclass JNICALL FindClass(JNIEnv *env, const char *name) {
  (void)env;
  if (!guard(NULL, 0)) return NULL;
  jclass k = calloc(1, sizeof *k);
  k->kind = K_CLASS;
  snprintf(k->name, sizeof k->name, "%s", name);
  ++g_live_refs;
  if (g_live_refs > g_peak_refs) g_peak_refs = g_live_refs;
  return k;
}

static jint JNICALL ThrowNew(JNIEnv *env, jclass clazz, const char *msg) {
  (void)env;
  if (!guard(clazz, K_CLASS)) return -1;
  raise_(clazz->name, msg);
  return 0;
}

static jboolean JNICALL ExceptionCheck(JNIEnv *env) {
  (void)env;
  return g_has_pending ? JNI_TRUE : JNI_FALSE;
}

static void JNICALL DeleteLocalRef(JNIEnv *env, jobject obj) {
  (void)env;
  if (!obj) return;
  --g_live_refs;
  if (obj->kind == K_CLASS) free(obj);
}

static jstring JNICALL NewStringUTF(JNIEnv *env, const char *utf) {
  (void)env;
  if (!guard(NULL, 0)) return NULL;
  jstring s = calloc(1, sizeof *s);
  s->kind = K_STRING;
  s->data = strdup(utf ? utf : "");
  s->len = (jsize)strlen((const char *)s->data);
  return s;
}

static jsize JNICALL GetArrayLength(JNIEnv *env, jarray a) {
  (void)env;
  if (g_has_pending || !a || (a->kind != K_DOUBLES && a->kind != K_LONGS && a->kind != K_OBJECTS)) {
    ++g_misuse;
    return 0;
  }
  return a->len;
}

static jobject JNICALL GetObjectArrayElement(JNIEnv *env, jobjectArray a, jsize i) {
  (void)env;
  if (!guard(a, K_OBJECTS)) return NULL;
  if (i < 0 || i >= a->len) {
    raise_("java/lang/ArrayIndexOutOfBoundsException", "object array index out of range");
    return NULL;
  }
  jobject o = ((jobject *)a->data)[i];
  if (o) {
    ++g_live_refs;
    if (g_live_refs > g_peak_refs) g_peak_refs = g_live_refs;
  }
  return o;
}

static int region_ok(jarray a, jsize start, jsize len) {
  if (start < 0 || len < 0 || (long)start + (long)len > (long)a->len) {
    raise_("java/lang/ArrayIndexOutOfBoundsException", "array region out of range");
    return 0;
  }
  return 1;
}

static void JNICALL GetLongArrayRegion(JNIEnv *env, jlongArray a, jsize start, jsize len, jlong *buf) {
  (void)env;
  if (!guard(a, K_LONGS) || !region_ok(a, start, len)) return;
  memcpy(buf, (const jlong *)a->data + start, (size_t)len * sizeof(jlong));
}

static void JNICALL GetDoubleArrayRegion(JNIEnv *env, jdoubleArray a, jsize start, jsize len, jdouble *buf) {
  (void)env;
  if (!guard(a, K_DOUBLES) || !region_ok(a, start, len)) return;
  memcpy(buf, (const jdouble *)a->data + start, (size_t)len * sizeof(jdouble));
}

static void JNICALL SetDoubleArrayRegion(JNIEnv *env, jdoubleArray a, jsize start, jsize len, const jdouble *buf) {
  (void)env;
  if (!guard(a, K_DOUBLES) || !region_ok(a, start, len)) return;
  memcpy((jdouble *)a->data + start, buf, (size_t)len * sizeof(jdouble));
}

static void *JNICALL GetDirectBufferAddress(JNIEnv *env, jobject b) {
  (void)env;
  if (!guard(NULL, 0)) return NULL;
  return b && b->kind == K_DIRECT ? b->data : NULL;  /* NULL for a non-direct buffer, as a JVM */
}

static jlong JNICALL GetDirectBufferCapacity(JNIEnv *env, jobject b) {
  (void)env;
  if (!guard(NULL, 0)) return -1;
  return b && b->kind == K_DIRECT ? b->cap : -1;
}

static const struct JNINativeInterface_ g_table = {
    FindClass, ThrowNew, ExceptionCheck, DeleteLocalRef, NewStringUTF, GetArrayLength, GetObjectArrayElement,
    GetLongArrayRegion, GetDoubleArrayRegion, SetDoubleArrayRegion, GetDirectBufferAddress, GetDirectBufferCapacity};
static JNIEnv g_env = &g_table;

/* ---- the test's side (ctypes) --------------------------------------------------------------- */
JNIEXPORT JNIEnv *h_env(void) { return &g_env; }

static jobject mk(int kind, jsize len, void *data) {
  jobject o = calloc(1, sizeof *o);
  o->kind = kind;
  o->len = len;
  o->data = data;
  return o;
}
JNIEXPORT jobject h_doubles(double *data, jsize len) { return mk(K_DOUBLES, len, data); }
JNIEXPORT jobject h_longs(jlong *data, jsize len) { return mk(K_LONGS, len, data); }
JNIEXPORT jobject h_objects(jsize len) { return mk(K_OBJECTS, len, calloc((size_t)(len > 0 ? len : 1), sizeof(jobject))); }
JNIEXPORT void h_set(jobject arr, jsize i, jobject elem) { ((jobject *)arr->data)[i] = elem; }
JNIEXPORT jobject h_direct(void *data, jlong cap) {
  jobject o = mk(K_DIRECT, 0, data);
  o->cap = cap;
  return o;
}
JNIEXPORT void h_free(jobject o) {
  if (!o) return;
  if (o->kind == K_OBJECTS || o->kind == K_STRING) free(o->data);
  free(o);
}
JNIEXPORT const char *h_string(jobject s) { return s && s->kind == K_STRING ? (const char *)s->data : NULL; }
JNIEXPORT const char *h_pending(void) { return g_has_pending ? g_pending : NULL; }
JNIEXPORT void h_clear(void) { g_has_pending = 0; g_pending[0] = 0; }
JNIEXPORT int h_misuse(void) { return g_misuse; }
JNIEXPORT long h_live_refs(void) { return g_live_refs; }
JNIEXPORT long h_peak_refs(void) { return g_peak_refs; }
JNIEXPORT void h_reset_counts(void) { g_misuse = 0; g_live_refs = 0; g_peak_refs = 0; }

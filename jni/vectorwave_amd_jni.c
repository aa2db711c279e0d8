/* vectorwave_amd_jni.c -- JNI glue between VectorWave's Java API and the MI355X engine's C-ABI
 * (include/vectorwave_amd.h).  Built where a JDK is present (jni/Makefile checks $JAVA_HOME/include/jni.h);
 * the Java side is jni/java/com/morphiqlabs/wavelet/amd/AmdNative.java.  Without a JDK the same source is
 * compiled against tests/jni_harness/jni.h (a test-only declaration of the JNIEnv functions used here) and
 * driven by tests/test_jni_glue.py through a fake JNIEnv: that exercises this file's logic (copies, chunking,
 * error paths, local references), not JNI ABI compatibility.
 *
 * One native call per batch, never one per row.  Three ways in:
 *
 *  - double[] arrays (the MODWTOptimizer SPI, core/api/spi/MODWTOptimizer.java:12-84, and flat batches):
 *    COPIED into native buffers (GetDoubleArrayRegion) and the results copied back (SetDoubleArrayRegion).
 *    No Java array is pinned while the GPU works, so the collector is never blocked for the length of a
 *    transform (a critical section held across a multi-millisecond call stalls every GC in the JVM).
 *  - double[][] / double[][][] as the Java API holds them (BatchMODWT.*AoS, ext/extensions/modwt/
 *    BatchMODWT.java:90-178; BatchStreamingMODWT, :55-275): rows gathered into one native block per chunk
 *    and scattered back row by row.
 *  - direct ByteBuffers (...Direct methods): the caller's off-heap memory goes straight to the engine's host
 *    staging (GetDirectBufferAddress), no extra copy and no pinning; the FFM form of the same is INTEGRATION.md
 *    section 4.
 *
 * Every engine call passes VW_FLAG_HOST_MEMORY | VW_FLAG_SYNC: the engine stages through its per-context
 * device pool and returns when the results are in the caller's memory.  Engine status codes are returned to
 * Java unchanged; AmdNative.check() maps them to the reference's exceptions.
 * Malformed arguments the glue finds itself (bad taps, short arrays, null or ragged rows, planes of the wrong
 * size) throw IllegalArgumentException / NullPointerException here, with their own message, so Java never
 * reports an unrelated vw_last_error() left by an earlier call.
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "vectorwave_amd.h"

#define VW_JNI(name) Java_com_morphiqlabs_wavelet_amd_AmdNative_##name
#define HOST_FLAGS (VW_FLAG_HOST_MEMORY | VW_FLAG_SYNC)
#define CTX(h) ((vw_ctx *)(intptr_t)(h))
#define STREAM(h) ((vw_stream *)(intptr_t)(h))

/* ---- Java exceptions raised by the glue ------------------------------------------------------ */
/* The exception is pending when the native returns: Java throws it there, AmdNative.check is not reached.
 * A pending exception (e.g. an ArrayIndexOutOfBoundsException from a Get...Region) is never replaced. */
static jint throw_java(JNIEnv *e, const char *cls, const char *msg, jint status) {
  if (!(*e)->ExceptionCheck(e)) {
    jclass k = (*e)->FindClass(e, cls);
    if (k) {
      (*e)->ThrowNew(e, k, msg);
      (*e)->DeleteLocalRef(e, k);
    }
  }
  return status;
}
static jint arg_error(JNIEnv *e, const char *msg) {
  return throw_java(e, "java/lang/IllegalArgumentException", msg, VW_ERR_ARG);
}
static jint null_error(JNIEnv *e, const char *msg) {
  return throw_java(e, "java/lang/NullPointerException", msg, VW_ERR_NULL);
}
static jint oom_error(JNIEnv *e) {
  return throw_java(e, "java/lang/OutOfMemoryError", "native staging buffer allocation failed", VW_ERR_DEVICE);
}

/* ---- per-thread native copy buffers ---------------------------------------------------------- */
/* Reused across calls (a JVM worker transforms batch after batch).  Slot 0..3: inputs / outputs of one
 * call.  Buffers above kKeepBytes are released after the call. */
enum { kSlots = 4 };
static const size_t kKeepBytes = (size_t)256 << 20;
static __thread double *t_buf[kSlots];
static __thread size_t t_cap[kSlots];

static double *slot(int k, size_t count) {
  size_t bytes = (count ? count : 1) * sizeof(double);
  if (bytes > t_cap[k]) {
    free(t_buf[k]);
    t_buf[k] = (double *)malloc(bytes);
    t_cap[k] = t_buf[k] ? bytes : 0;
  }
  return t_buf[k];
}

static void trim_slots(void) {
  for (int k = 0; k < kSlots; ++k)
    if (t_cap[k] > kKeepBytes) {
      free(t_buf[k]);
      t_buf[k] = NULL;
      t_cap[k] = 0;
    }
}

/* Copy a Java double[] (count elements) into native slot k; NULL array -> NULL. */
static double *copy_in(JNIEnv *e, jdoubleArray a, int k, size_t count, int *oom) {
  if (!a) return NULL;
  double *p = slot(k, count);
  if (!p) { *oom = 1; return NULL; }
  if (count) (*e)->GetDoubleArrayRegion(e, a, 0, (jsize)count, p);
  return p;
}

static double *out_buf(int k, size_t count, int *oom) {
  double *p = slot(k, count);
  if (!p) *oom = 1;
  return p;
}

static void copy_out(JNIEnv *e, jdoubleArray a, const double *p, size_t count) {
  if (a && p && count) (*e)->SetDoubleArrayRegion(e, a, 0, (jsize)count, p);
}

/* Taps are short (<= 64): a stack copy.  Both filters present, 1..64 taps, equal lengths. */
typedef struct { double v[64]; int n; } Taps;
static int get_taps(JNIEnv *e, jdoubleArray lo, jdoubleArray hi, Taps *tl, Taps *th) {
  if (!lo || !hi) { null_error(e, "filter taps cannot be null"); return 0; }
  tl->n = (*e)->GetArrayLength(e, lo);
  th->n = (*e)->GetArrayLength(e, hi);
  if (tl->n < 1 || tl->n > 64 || tl->n != th->n) {
    arg_error(e, "filter taps must be 1..64 values, low and high pass of equal length");
    return 0;
  }
  (*e)->GetDoubleArrayRegion(e, lo, 0, tl->n, tl->v);
  (*e)->GetDoubleArrayRegion(e, hi, 0, th->n, th->v);
  return 1;
}

static size_t alen(JNIEnv *e, jdoubleArray a) { return a ? (size_t)(*e)->GetArrayLength(e, a) : 0; }

static int flat_ok(JNIEnv *e, jint B, jint N) {
  if (B < 1 || N < 1) { arg_error(e, "batch and signal length must be > 0"); return 0; }
  return 1;
}

/* ---- contexts ------------------------------------------------------------------------------ */
JNIEXPORT jlong JNICALL VW_JNI(ctxCreate)(JNIEnv *e, jclass c, jint device) {
  (void)e; (void)c;
  vw_ctx *ctx = NULL;
  return vw_ctx_create(device, &ctx) == VW_OK ? (jlong)(intptr_t)ctx : 0;
}

JNIEXPORT jint JNICALL VW_JNI(ctxDestroy)(JNIEnv *e, jclass c, jlong ctx) {
  (void)e; (void)c;
  return vw_ctx_destroy(CTX(ctx));
}

JNIEXPORT jint JNICALL VW_JNI(maxLevels)(JNIEnv *e, jclass c, jlong n, jint L) {
  (void)e; (void)c;
  return vw_max_levels(n, L);
}

JNIEXPORT jstring JNICALL VW_JNI(lastError)(JNIEnv *e, jclass c) {
  (void)c;
  return (*e)->NewStringUTF(e, vw_last_error());
}

JNIEXPORT jlong JNICALL VW_JNI(lastErrorIndex)(JNIEnv *e, jclass c) {
  (void)e; (void)c;
  return vw_last_error_index();
}

/* ---- single level: MODWTTransform.forward / forwardBatch, inverse / inverseBatch ------------- */
/* x: B*N (row-major), approx / detail: B*N.  MODWTOptimizer.forward is B = 1. */
JNIEXPORT jint JNICALL VW_JNI(modwt1Forward)(JNIEnv *e, jclass c, jlong ctx, jdoubleArray x, jint B, jint N,
                                             jdoubleArray lo, jdoubleArray hi, jint boundary, jint flags,
                                             jdoubleArray approx, jdoubleArray detail) {
  (void)c;
  Taps tl, th;
  if (!get_taps(e, lo, hi, &tl, &th) || !flat_ok(e, B, N)) return VW_ERR_ARG;
  if (!x || !approx || !detail) return null_error(e, "signal and output arrays cannot be null");
  const size_t n = (size_t)B * (size_t)N;
  if (alen(e, x) < n || alen(e, approx) < n || alen(e, detail) < n) return arg_error(e, "array shorter than B * N");
  int oom = 0;
  double *px = copy_in(e, x, 0, n, &oom), *pa = out_buf(1, n, &oom), *pd = out_buf(2, n, &oom);
  if (oom) return oom_error(e);
  vw_status st = vw_modwt1_forward_f64(CTX(ctx), px, B, N, N, tl.v, th.v, tl.n, boundary,
                                       (unsigned)flags | HOST_FLAGS, pa, pd);
  if (st == VW_OK) { copy_out(e, approx, pa, n); copy_out(e, detail, pd, n); }
  trim_slots();
  return st;
}

JNIEXPORT jint JNICALL VW_JNI(modwt1Inverse)(JNIEnv *e, jclass c, jlong ctx, jdoubleArray approx,
                                             jdoubleArray detail, jint B, jint N, jdoubleArray lo, jdoubleArray hi,
                                             jint boundary, jint flags, jdoubleArray y) {
  (void)c;
  Taps tl, th;
  if (!get_taps(e, lo, hi, &tl, &th) || !flat_ok(e, B, N)) return VW_ERR_ARG;
  if (!approx || !detail || !y) return null_error(e, "coefficient and output arrays cannot be null");
  const size_t n = (size_t)B * (size_t)N;
  if (alen(e, approx) < n || alen(e, detail) < n || alen(e, y) < n) return arg_error(e, "array shorter than B * N");
  int oom = 0;
  double *pa = copy_in(e, approx, 0, n, &oom), *pd = copy_in(e, detail, 1, n, &oom), *py = out_buf(2, n, &oom);
  if (oom) return oom_error(e);
  vw_status st = vw_modwt1_inverse_f64(CTX(ctx), pa, pd, B, N, tl.v, th.v, tl.n, boundary,
                                       (unsigned)flags | HOST_FLAGS, py);
  if (st == VW_OK) copy_out(e, y, py, n);
  trim_slots();
  return st;
}

/* ---- multi level: MultiLevelMODWTTransform.decompose / reconstruct over flat arrays ------------ */
/* x: B*N, details: J*B*N ([level 1..J][B][N]), approx: B*N. */
JNIEXPORT jint JNICALL VW_JNI(modwtForward)(JNIEnv *e, jclass c, jlong ctx, jdoubleArray x, jint B, jint N,
                                            jdoubleArray lo, jdoubleArray hi, jint wid, jint boundary, jint J,
                                            jint flags, jdoubleArray details, jdoubleArray approx) {
  (void)c;
  Taps tl, th;
  if (!get_taps(e, lo, hi, &tl, &th) || !flat_ok(e, B, N)) return VW_ERR_ARG;
  if (J < 1) return arg_error(e, "levels must be >= 1");
  if (!x || !details || !approx) return null_error(e, "signal and output arrays cannot be null");
  const size_t n = (size_t)B * (size_t)N;
  if (alen(e, x) < n || alen(e, details) < (size_t)J * n || alen(e, approx) < n)
    return arg_error(e, "array shorter than B * N (details: levels * B * N)");
  int oom = 0;
  double *px = copy_in(e, x, 0, n, &oom), *pd = out_buf(1, (size_t)J * n, &oom), *pa = out_buf(2, n, &oom);
  if (oom) return oom_error(e);
  vw_status st = vw_modwt_forward_f64(CTX(ctx), px, B, N, N, tl.v, th.v, tl.n, wid, boundary, J,
                                      (unsigned)flags | HOST_FLAGS, pd, pa);
  if (st == VW_OK) { copy_out(e, details, pd, (size_t)J * n); copy_out(e, approx, pa, n); }
  trim_slots();
  return st;
}

JNIEXPORT jint JNICALL VW_JNI(modwtInverse)(JNIEnv *e, jclass c, jlong ctx, jdoubleArray details,
                                            jdoubleArray approx, jint B, jint N, jdoubleArray lo, jdoubleArray hi,
                                            jint wid, jint boundary, jint J, jint detailMask, jboolean approxZero,
                                            jint flags, jdoubleArray y) {
  (void)c;
  Taps tl, th;
  if (!get_taps(e, lo, hi, &tl, &th) || !flat_ok(e, B, N)) return VW_ERR_ARG;
  if (J < 1) return arg_error(e, "levels must be >= 1");
  if (!y || (detailMask && !details) || (!approxZero && !approx))
    return null_error(e, "coefficient and output arrays cannot be null");
  const size_t n = (size_t)B * (size_t)N;
  if ((detailMask && alen(e, details) < (size_t)J * n) || (!approxZero && alen(e, approx) < n) || alen(e, y) < n)
    return arg_error(e, "array shorter than B * N (details: levels * B * N)");
  int oom = 0;
  double *pd = detailMask ? copy_in(e, details, 0, (size_t)J * n, &oom) : NULL;
  double *pa = approxZero ? NULL : copy_in(e, approx, 1, n, &oom);
  double *py = out_buf(2, n, &oom);
  if (oom) return oom_error(e);
  vw_status st = vw_modwt_inverse_f64(CTX(ctx), pd, pa, B, N, tl.v, th.v, tl.n, wid, boundary, J,
                                      (unsigned)detailMask, approxZero ? 1 : 0, (unsigned)flags | HOST_FLAGS, py);
  if (st == VW_OK) copy_out(e, y, py, n);
  trim_slots();
  return st;
}

/* One batch over several contexts (one std::thread per context inside the engine). */
JNIEXPORT jint JNICALL VW_JNI(modwtForwardMulti)(JNIEnv *e, jclass c, jlongArray ctxs, jdoubleArray x, jint B,
                                                 jint N, jdoubleArray lo, jdoubleArray hi, jint wid, jint boundary,
                                                 jint J, jint flags, jdoubleArray details, jdoubleArray approx) {
  (void)c;
  Taps tl, th;
  if (!ctxs) return null_error(e, "contexts cannot be null");
  if (!get_taps(e, lo, hi, &tl, &th) || !flat_ok(e, B, N)) return VW_ERR_ARG;
  if (J < 1) return arg_error(e, "levels must be >= 1");
  const jsize nctx = (*e)->GetArrayLength(e, ctxs);
  if (nctx < 1 || nctx > 256) return arg_error(e, "1..256 contexts");
  if (!x || !details || !approx) return null_error(e, "signal and output arrays cannot be null");
  const size_t n = (size_t)B * (size_t)N;
  if (alen(e, x) < n || alen(e, details) < (size_t)J * n || alen(e, approx) < n)
    return arg_error(e, "array shorter than B * N (details: levels * B * N)");
  jlong hs[256];
  (*e)->GetLongArrayRegion(e, ctxs, 0, nctx, hs);
  vw_ctx *cs[256];
  for (jsize k = 0; k < nctx; ++k) cs[k] = CTX(hs[k]);
  int oom = 0;
  double *px = copy_in(e, x, 0, n, &oom), *pd = out_buf(1, (size_t)J * n, &oom), *pa = out_buf(2, n, &oom);
  if (oom) return oom_error(e);
  vw_status st = vw_modwt_forward_multi_f64(cs, nctx, px, B, N, N, tl.v, th.v, tl.n, wid, boundary, J,
                                            (unsigned)flags | VW_FLAG_HOST_MEMORY, pd, pa);
  if (st == VW_OK) { copy_out(e, details, pd, (size_t)J * n); copy_out(e, approx, pa, n); }
  trim_slots();
  return st;
}

/* ---- denoising: VectorWaveSwtAdapter.denoise, WaveletDenoiser ------------------------------ */
JNIEXPORT jint JNICALL VW_JNI(swtDenoise)(JNIEnv *e, jclass c, jlong ctx, jdoubleArray x, jint B, jint N,
                                          jdoubleArray lo, jdoubleArray hi, jint wid, jint boundary, jint J,
                                          jdouble threshold, jboolean soft, jint flags, jdoubleArray y,
                                          jdoubleArray thresholdsOut) {
  (void)c;
  Taps tl, th;
  if (!get_taps(e, lo, hi, &tl, &th) || !flat_ok(e, B, N)) return VW_ERR_ARG;
  if (!x || !y) return null_error(e, "signal and output arrays cannot be null");
  const size_t n = (size_t)B * (size_t)N;
  if (alen(e, x) < n || alen(e, y) < n || (thresholdsOut && alen(e, thresholdsOut) < (size_t)B))
    return arg_error(e, "array shorter than B * N (thresholds: B)");
  int oom = 0;
  double *px = copy_in(e, x, 0, n, &oom), *py = out_buf(1, n, &oom);
  double *pt = thresholdsOut ? out_buf(2, (size_t)B, &oom) : NULL;
  if (oom) return oom_error(e);
  vw_status st = vw_swt_denoise_f64(CTX(ctx), px, B, N, N, tl.v, th.v, tl.n, wid, boundary, J, threshold,
                                    soft ? 1 : 0, (unsigned)flags | HOST_FLAGS, py, pt);
  if (st == VW_OK) { copy_out(e, y, py, n); copy_out(e, thresholdsOut, pt, (size_t)B); }
  trim_slots();
  return st;
}

JNIEXPORT jint JNICALL VW_JNI(waveletDenoise)(JNIEnv *e, jclass c, jlong ctx, jdoubleArray x, jint B, jint N,
                                              jdoubleArray lo, jdoubleArray hi, jint wid, jint boundary,
                                              jint levels, jint method, jdouble fixedThreshold, jboolean soft,
                                              jint flags, jdoubleArray y, jdoubleArray thresholdsOut) {
  (void)c;
  Taps tl, th;
  if (!get_taps(e, lo, hi, &tl, &th) || !flat_ok(e, B, N)) return VW_ERR_ARG;
  if (!x || !y) return null_error(e, "signal and output arrays cannot be null");
  const size_t n = (size_t)B * (size_t)N, nt = (size_t)(levels > 0 ? levels : 1) * (size_t)B;
  if (alen(e, x) < n || alen(e, y) < n || (thresholdsOut && alen(e, thresholdsOut) < nt))
    return arg_error(e, "array shorter than B * N (thresholds: max(levels, 1) * B)");
  int oom = 0;
  double *px = copy_in(e, x, 0, n, &oom), *py = out_buf(1, n, &oom);
  double *pt = thresholdsOut ? out_buf(2, nt, &oom) : NULL;
  if (oom) return oom_error(e);
  vw_status st = vw_wavelet_denoise_f64(CTX(ctx), px, B, N, N, tl.v, th.v, tl.n, wid, boundary, levels, method,
                                        fixedThreshold, soft ? 1 : 0, (unsigned)flags | HOST_FLAGS, py, pt);
  if (st == VW_OK) { copy_out(e, y, py, n); copy_out(e, thresholdsOut, pt, nt); }
  trim_slots();
  return st;
}

/* VectorWaveSwtAdapter.estimateNoiseSigma (core/swt/VectorWaveSwtAdapter.java:627-645): sigma[b] =
 * median(|coeffs[b]|) / 0.6745 for B rows of N (flat), exact selection on the device. */
JNIEXPORT jint JNICALL VW_JNI(noiseSigma)(JNIEnv *e, jclass c, jlong ctx, jdoubleArray coeffs, jint B, jint N,
                                          jdoubleArray sigmaOut) {
  (void)c;
  if (!coeffs || !sigmaOut) return null_error(e, "coefficients and output cannot be null");
  if (!flat_ok(e, B, N)) return VW_ERR_ARG;
  const size_t n = (size_t)B * (size_t)N;
  if (alen(e, coeffs) < n || alen(e, sigmaOut) < (size_t)B) return arg_error(e, "array shorter than B * N");
  int oom = 0;
  double *pc = copy_in(e, coeffs, 0, n, &oom), *ps = out_buf(1, (size_t)B, &oom);
  if (oom) return oom_error(e);
  vw_status st = vw_noise_sigma_f64(CTX(ctx), pc, B, N, HOST_FLAGS, ps);
  if (st == VW_OK) copy_out(e, sigmaOut, ps, (size_t)B);
  trim_slots();
  return st;
}

/* ---- direct ByteBuffers: zero-copy host path ----------------------------------------------- */
static double *direct(JNIEnv *e, jobject buf, size_t count) {
  if (!buf) return NULL;
  void *p = (*e)->GetDirectBufferAddress(e, buf);
  jlong cap = (*e)->GetDirectBufferCapacity(e, buf);
  if (!p || cap < 0 || (size_t)cap < count * sizeof(double)) return NULL;
  return (double *)p;
}

JNIEXPORT jint JNICALL VW_JNI(modwtForwardDirect)(JNIEnv *e, jclass c, jlong ctx, jobject x, jint B, jint N,
                                                  jdoubleArray lo, jdoubleArray hi, jint wid, jint boundary, jint J,
                                                  jint flags, jobject details, jobject approx) {
  (void)c;
  Taps tl, th;
  if (!get_taps(e, lo, hi, &tl, &th) || !flat_ok(e, B, N)) return VW_ERR_ARG;
  if (J < 1) return arg_error(e, "levels must be >= 1");
  const size_t n = (size_t)B * (size_t)N;
  double *px = direct(e, x, n), *pd = direct(e, details, (size_t)J * n), *pa = direct(e, approx, n);
  if (!px || !pd || !pa) return arg_error(e, "buffers must be direct and hold B * N doubles (details: levels * B * N)");
  return vw_modwt_forward_f64(CTX(ctx), px, B, N, N, tl.v, th.v, tl.n, wid, boundary, J,
                              (unsigned)flags | HOST_FLAGS, pd, pa);
}

JNIEXPORT jint JNICALL VW_JNI(modwtInverseDirect)(JNIEnv *e, jclass c, jlong ctx, jobject details, jobject approx,
                                                  jint B, jint N, jdoubleArray lo, jdoubleArray hi, jint wid,
                                                  jint boundary, jint J, jint flags, jobject y) {
  (void)c;
  Taps tl, th;
  if (!get_taps(e, lo, hi, &tl, &th) || !flat_ok(e, B, N)) return VW_ERR_ARG;
  if (J < 1) return arg_error(e, "levels must be >= 1");
  const size_t n = (size_t)B * (size_t)N;
  double *pd = direct(e, details, (size_t)J * n), *pa = direct(e, approx, n), *py = direct(e, y, n);
  if (!pd || !pa || !py) return arg_error(e, "buffers must be direct and hold B * N doubles (details: levels * B * N)");
  return vw_modwt_inverse_f64(CTX(ctx), pd, pa, B, N, tl.v, th.v, tl.n, wid, boundary, J, 0xFFFFFFFFu, 0,
                              (unsigned)flags | HOST_FLAGS, py);
}

/* ---- AoS batches: double[][] rows straight into the engine's staging ------------------------
 * BatchMODWT.multiLevelAoS / inverseMultiLevelAoS (ext/extensions/modwt/BatchMODWT.java:90-111,
 * :151-178) and VectorWaveSwtAdapter.forward / denoise over a batch.  The Java side passes its double[][]
 * (and double[][][] for the details) unchanged: rows are gathered into one native block per chunk
 * (GetDoubleArrayRegion per row -- the only copy; no Java-side flattening, no array pinned across the GPU
 * call) and the results scattered back row by row.  Chunks of rows keep each native block under
 * VW_JNI_CHUNK_BYTES and every size in size_t, so a batch whose B*N or J*B*N exceeds Integer.MAX_VALUE (a
 * Java array's limit, e.g. 256 x 2^20 x 10 details) still goes through.  Each chunk's engine call names its
 * first row as the signal base (vw_set_signal_base): a non-finite error names the batch's signal.  Shapes
 * are checked before the first chunk runs; earlier chunks of a batch whose later chunk fails validation
 * have run (their outputs are left in the caller's arrays, which the facades then discard).  Local
 * references are released per row: the JNI guarantees only 16. */
#ifndef VW_JNI_CHUNK_BYTES
#define VW_JNI_CHUNK_BYTES ((size_t)512 << 20) /* tests/jni_harness builds the glue with a few KiB */
#endif

static jsize chunk_rows(size_t per_row_doubles, jsize B) {
  size_t r = (size_t)VW_JNI_CHUNK_BYTES / (per_row_doubles * sizeof(double));
  if (r < 1) r = 1;
  return r < (size_t)B ? (jsize)r : B;
}

/* rows[b0 .. b0+nb) (each of length n) <-> dst[nb][n]; 0 (and the exception) on a null or ragged row */
static int gather_rows(JNIEnv *e, jobjectArray rows, jsize b0, jsize nb, jsize n, double *dst) {
  for (jsize b = 0; b < nb; ++b) {
    jdoubleArray r = (jdoubleArray)(*e)->GetObjectArrayElement(e, rows, b0 + b);
    if (!r) { arg_error(e, "all signals must be non-null and same length"); return 0; }
    int ok = (*e)->GetArrayLength(e, r) == n;
    if (ok) (*e)->GetDoubleArrayRegion(e, r, 0, n, dst + (size_t)b * (size_t)n);
    (*e)->DeleteLocalRef(e, r);
    if (!ok) { arg_error(e, "all signals must be non-null and same length"); return 0; }
  }
  return 1;
}

static int scatter_rows(JNIEnv *e, jobjectArray rows, jsize b0, jsize nb, jsize n, const double *src) {
  for (jsize b = 0; b < nb; ++b) {
    jdoubleArray r = (jdoubleArray)(*e)->GetObjectArrayElement(e, rows, b0 + b);
    if (!r) { arg_error(e, "output rows must be non-null"); return 0; }
    int ok = (*e)->GetArrayLength(e, r) == n;
    if (ok) (*e)->SetDoubleArrayRegion(e, r, 0, n, src + (size_t)b * (size_t)n);
    (*e)->DeleteLocalRef(e, r);
    if (!ok) { arg_error(e, "output rows must have the signal length"); return 0; }
  }
  return 1;
}

/* level plane l of a double[][][] ([levels][batch][length]) */
static jobjectArray plane(JNIEnv *e, jobjectArray dpl, jsize l) {
  return (jobjectArray)(*e)->GetObjectArrayElement(e, dpl, l);
}

/* a double[][] of exactly `rows` rows (the exception otherwise) */
static int rows_ok(JNIEnv *e, jobjectArray a, jsize rows, const char *what) {
  if (!a) { null_error(e, what); return 0; }
  if ((*e)->GetArrayLength(e, a) != rows) { arg_error(e, what); return 0; }
  return 1;
}

/* every plane of a double[][][] ([levels][batch][length]) non-null and of `batch` rows */
static int planes_ok(JNIEnv *e, jobjectArray dpl, jsize levels, jsize batch) {
  for (jsize l = 0; l < levels; ++l) {
    jobjectArray pl = plane(e, dpl, l);
    const int ok = pl && (*e)->GetArrayLength(e, pl) == batch;
    if (pl) (*e)->DeleteLocalRef(e, pl);
    if (!ok) { arg_error(e, "detailPerLevel[L] must be non-null and length=batch for all L"); return 0; }
  }
  return 1;
}

/* length of row 0 of a non-empty double[][]; -1 (and the exception) otherwise (BatchMODWT.validateAoS
 * :201-212 messages) */
static jsize row_len(JNIEnv *e, jobjectArray rows) {
  if (!rows || (*e)->GetArrayLength(e, rows) < 1) { arg_error(e, "signals must be non-null and non-empty"); return -1; }
  jdoubleArray r = (jdoubleArray)(*e)->GetObjectArrayElement(e, rows, 0);
  if (!r) { arg_error(e, "all signals must be non-null and same length"); return -1; }
  jsize n = (*e)->GetArrayLength(e, r);
  (*e)->DeleteLocalRef(e, r);
  if (n < 1) { arg_error(e, "signal length must be > 0"); return -1; }
  return n;
}

JNIEXPORT jint JNICALL VW_JNI(modwtForwardAoS)(JNIEnv *e, jclass c, jlong ctx, jobjectArray x, jdoubleArray lo,
                                               jdoubleArray hi, jint wid, jint boundary, jint J, jint flags,
                                               jobjectArray details, jobjectArray approx) {
  (void)c;
  Taps tl, th;
  if (!get_taps(e, lo, hi, &tl, &th)) return VW_ERR_ARG;
  if (J < 1) return arg_error(e, "levels must be >= 1");
  const jsize N = row_len(e, x);
  if (N < 1) return VW_ERR_ARG;
  const jsize B = (*e)->GetArrayLength(e, x);
  if (!rows_ok(e, details, J, "details must hold one plane per level") ||
      !rows_ok(e, approx, B, "approx must hold one row per signal") || !planes_ok(e, details, J, B))
    return VW_ERR_ARG;
  const jsize CB = chunk_rows((size_t)(J + 2) * (size_t)N, B);
  int oom = 0;
  double *px = out_buf(0, (size_t)CB * N, &oom), *pd = out_buf(1, (size_t)J * CB * N, &oom);
  double *pa = out_buf(2, (size_t)CB * N, &oom);
  if (oom) return oom_error(e);
  vw_status st = VW_OK;
  for (jsize b0 = 0; b0 < B && st == VW_OK; b0 += CB) {
    const jsize nb = B - b0 < CB ? B - b0 : CB;
    if (!gather_rows(e, x, b0, nb, N, px)) { st = VW_ERR_ARG; break; }
    vw_set_signal_base(b0);
    st = vw_modwt_forward_f64(CTX(ctx), px, nb, N, N, tl.v, th.v, tl.n, wid, boundary, J,
                              (unsigned)flags | HOST_FLAGS, pd, pa);
    vw_set_signal_base(0);
    for (jsize l = 0; l < J && st == VW_OK; ++l) {
      jobjectArray pl = plane(e, details, l);
      if (!scatter_rows(e, pl, b0, nb, N, pd + (size_t)l * nb * N)) st = VW_ERR_ARG;
      (*e)->DeleteLocalRef(e, pl);
    }
    if (st == VW_OK && !scatter_rows(e, approx, b0, nb, N, pa)) st = VW_ERR_ARG;
  }
  trim_slots();
  return st;
}

JNIEXPORT jint JNICALL VW_JNI(modwtInverseAoS)(JNIEnv *e, jclass c, jlong ctx, jobjectArray details,
                                               jobjectArray approx, jdoubleArray lo, jdoubleArray hi, jint wid,
                                               jint boundary, jint flags, jobjectArray y) {
  (void)c;
  Taps tl, th;
  if (!get_taps(e, lo, hi, &tl, &th)) return VW_ERR_ARG;
  if (!details) return null_error(e, "detailPerLevel cannot be null");
  const jsize J = (*e)->GetArrayLength(e, details);
  if (J < 1) return arg_error(e, "levels must be > 0");
  const jsize N = row_len(e, approx);
  if (N < 1) return VW_ERR_ARG;
  const jsize B = (*e)->GetArrayLength(e, approx);
  if (!rows_ok(e, y, B, "output must hold one row per signal") || !planes_ok(e, details, J, B)) return VW_ERR_ARG;
  const jsize CB = chunk_rows((size_t)(J + 2) * (size_t)N, B);
  int oom = 0;
  double *pd = out_buf(0, (size_t)J * CB * N, &oom), *pa = out_buf(1, (size_t)CB * N, &oom);
  double *py = out_buf(2, (size_t)CB * N, &oom);
  if (oom) return oom_error(e);
  vw_status st = VW_OK;
  for (jsize b0 = 0; b0 < B && st == VW_OK; b0 += CB) {
    const jsize nb = B - b0 < CB ? B - b0 : CB;
    for (jsize l = 0; l < J && st == VW_OK; ++l) {
      jobjectArray pl = plane(e, details, l);
      if (!gather_rows(e, pl, b0, nb, N, pd + (size_t)l * nb * N)) st = VW_ERR_ARG;
      (*e)->DeleteLocalRef(e, pl);
    }
    if (st != VW_OK) break;
    if (!gather_rows(e, approx, b0, nb, N, pa)) { st = VW_ERR_ARG; break; }
    vw_set_signal_base(b0);
    st = vw_modwt_inverse_f64(CTX(ctx), pd, pa, nb, N, tl.v, th.v, tl.n, wid, boundary, J, 0xFFFFFFFFu, 0,
                              (unsigned)flags | HOST_FLAGS, py);
    vw_set_signal_base(0);
    if (st == VW_OK && !scatter_rows(e, y, b0, nb, N, py)) st = VW_ERR_ARG;
  }
  trim_slots();
  return st;
}

JNIEXPORT jint JNICALL VW_JNI(swtDenoiseAoS)(JNIEnv *e, jclass c, jlong ctx, jobjectArray x, jdoubleArray lo,
                                             jdoubleArray hi, jint wid, jint boundary, jint J, jdouble threshold,
                                             jboolean soft, jint flags, jobjectArray y) {
  (void)c;
  Taps tl, th;
  if (!get_taps(e, lo, hi, &tl, &th)) return VW_ERR_ARG;
  const jsize N = row_len(e, x);
  if (N < 1) return VW_ERR_ARG;
  const jsize B = (*e)->GetArrayLength(e, x);
  if (!rows_ok(e, y, B, "output must hold one row per signal")) return VW_ERR_ARG;
  const jsize CB = chunk_rows(2 * (size_t)N, B);
  int oom = 0;
  double *px = out_buf(0, (size_t)CB * N, &oom), *py = out_buf(1, (size_t)CB * N, &oom);
  if (oom) return oom_error(e);
  vw_status st = VW_OK;
  for (jsize b0 = 0; b0 < B && st == VW_OK; b0 += CB) {
    const jsize nb = B - b0 < CB ? B - b0 : CB;
    if (!gather_rows(e, x, b0, nb, N, px)) { st = VW_ERR_ARG; break; }
    vw_set_signal_base(b0);
    st = vw_swt_denoise_f64(CTX(ctx), px, nb, N, N, tl.v, th.v, tl.n, wid, boundary, J, threshold, soft ? 1 : 0,
                            (unsigned)flags | HOST_FLAGS, py, NULL);
    vw_set_signal_base(0);
    if (st == VW_OK && !scatter_rows(e, y, b0, nb, N, py)) st = VW_ERR_ARG;
  }
  trim_slots();
  return st;
}

/* ---- BatchStreamingMODWT ZERO_PADDING / SYMMETRIC (ext/extensions/modwt/BatchStreamingMODWT.java:55-380)
 * over vw_stream_*: the per-level left history lives on the device between blocks.  (PERIODIC blocks are
 * independent: the Java facade sends them through the BatchMODWT natives, as the reference does.)  A block
 * is one native call, not chunked: the history is per row of the whole batch. */
JNIEXPORT jlong JNICALL VW_JNI(streamCreate)(JNIEnv *e, jclass c, jlong ctx, jdoubleArray lo, jdoubleArray hi,
                                             jint boundary, jint levels) {
  (void)c;
  Taps tl, th;
  if (!get_taps(e, lo, hi, &tl, &th)) return 0;
  vw_stream *s = NULL;
  return vw_stream_create(CTX(ctx), tl.v, th.v, tl.n, boundary, levels, &s) == VW_OK ? (jlong)(intptr_t)s : 0;
}

JNIEXPORT jint JNICALL VW_JNI(streamDestroy)(JNIEnv *e, jclass c, jlong stream) {
  (void)e; (void)c;
  return vw_stream_destroy(STREAM(stream));
}

JNIEXPORT jlong JNICALL VW_JNI(streamHistoryLength)(JNIEnv *e, jclass c, jlong stream, jint level) {
  (void)e; (void)c;
  return vw_stream_history_length(STREAM(stream), level);
}

/* the engine writes [levels][B][n] details: the Java planes must be exactly the configured levels */
static int stream_levels_ok(JNIEnv *e, vw_stream *s, jsize J) {
  if (J >= 1 && vw_stream_history_length(s, J) >= 0 && vw_stream_history_length(s, J + 1) < 0) return 1;
  arg_error(e, "details must hold one plane per configured level");
  return 0;
}

/* processSingleLevel / processMultiLevel (:55-175): block [B][n] -> details [levels][B][n], approx [B][n]. */
JNIEXPORT jint JNICALL VW_JNI(streamProcessAoS)(JNIEnv *e, jclass c, jlong stream, jobjectArray block,
                                                jobjectArray details, jobjectArray approx) {
  (void)c;
  vw_stream *s = STREAM(stream);
  if (!s) return null_error(e, "stream is closed");
  const jsize N = row_len(e, block);
  if (N < 1) return VW_ERR_ARG;
  const jsize B = (*e)->GetArrayLength(e, block);
  if (!details) return null_error(e, "details cannot be null");
  const jsize J = (*e)->GetArrayLength(e, details);
  if (!stream_levels_ok(e, s, J) || !rows_ok(e, approx, B, "approx must hold one row per signal") ||
      !planes_ok(e, details, J, B))
    return VW_ERR_ARG;
  const size_t n = (size_t)B * (size_t)N;
  int oom = 0;
  double *px = out_buf(0, n, &oom), *pd = out_buf(1, (size_t)J * n, &oom), *pa = out_buf(2, n, &oom);
  if (oom) return oom_error(e);
  if (!gather_rows(e, block, 0, B, N, px)) { trim_slots(); return VW_ERR_ARG; }
  vw_status st = vw_stream_process_f64(s, px, B, N, HOST_FLAGS | VW_FLAG_REF_NONFINITE, pd, pa);
  for (jsize l = 0; l < J && st == VW_OK; ++l) {
    jobjectArray pl = plane(e, details, l);
    if (!scatter_rows(e, pl, 0, B, N, pd + (size_t)l * n)) st = VW_ERR_ARG;
    (*e)->DeleteLocalRef(e, pl);
  }
  if (st == VW_OK && !scatter_rows(e, approx, 0, B, N, pa)) st = VW_ERR_ARG;
  trim_slots();
  return st;
}

/* flushSingleLevel / flushMultiLevel (:181-275): the synthetic tail of tailLength samples per signal of the
 * last block's batch (details [levels][B][tail], approx [B][tail]); the Java side sizes the outputs. */
JNIEXPORT jint JNICALL VW_JNI(streamFlushAoS)(JNIEnv *e, jclass c, jlong stream, jint tailLength,
                                              jobjectArray details, jobjectArray approx) {
  (void)c;
  vw_stream *s = STREAM(stream);
  if (!s) return null_error(e, "stream is closed");
  if (!details || !approx) return null_error(e, "outputs cannot be null");
  const jsize B = (*e)->GetArrayLength(e, approx), J = (*e)->GetArrayLength(e, details);
  if (!stream_levels_ok(e, s, J) || !planes_ok(e, details, J, B)) return VW_ERR_ARG;
  if (tailLength > 0 && vw_stream_batch(s) > 0 && (int64_t)B != vw_stream_batch(s))
    return arg_error(e, "flush outputs must hold one row per signal of the last block");
  const size_t n = (size_t)B * (size_t)(tailLength > 0 ? tailLength : 0);
  int oom = 0;
  double *pd = out_buf(1, (size_t)J * n, &oom), *pa = out_buf(2, n, &oom);
  if (oom) return oom_error(e);
  vw_status st = vw_stream_flush_f64(s, tailLength, HOST_FLAGS | VW_FLAG_REF_NONFINITE, pd, pa);
  for (jsize l = 0; l < J && st == VW_OK && tailLength > 0; ++l) {
    jobjectArray pl = plane(e, details, l);
    if (!scatter_rows(e, pl, 0, B, tailLength, pd + (size_t)l * n)) st = VW_ERR_ARG;
    (*e)->DeleteLocalRef(e, pl);
  }
  if (st == VW_OK && tailLength > 0 && !scatter_rows(e, approx, 0, B, tailLength, pa)) st = VW_ERR_ARG;
  trim_slots();
  return st;
}

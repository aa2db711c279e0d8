/*
 * vectorwave_amd.h -- C ABI of the MI355X (gfx950) MODWT / SWT engine.
 *
 * Drop-in boundary for VectorWave's MODWT/SWT hot path: the per-level a-trous
 * low/high-pass convolutions (forward and inverse, PERIODIC / ZERO_PADDING /
 * SYMMETRIC).  Plain C types only -- no torch, no HIP types in signatures --
 * so a JNI (or Java 22+ FFM) shim, ctypes, or C/C++ host code can bind it.
 *
 * Reference interfaces each entry point replaces (paths relative to
 * /root/reference, prefixes core/ = vectorwave-core/src/main/java/com/morphiqlabs/wavelet/,
 * ext/ = vectorwave-extensions/src/main/java/com/morphiqlabs/wavelet/):
 *
 *   vw_modwt_forward_*      MultiLevelMODWTTransform.decompose / decomposeMutable
 *                             core/modwt/MultiLevelMODWTTransform.java:209-330
 *                           BatchMODWT.multiLevelAoS  ext/extensions/modwt/BatchMODWT.java:90-111
 *                           BatchSIMDMODWT.batchMultiLevelMODWTSoA  ext/extensions/modwt/BatchSIMDMODWT.java:343-424
 *                           VectorWaveSwtAdapter.forward  core/swt/VectorWaveSwtAdapter.java:198-394
 *   vw_modwt_inverse_*      MultiLevelMODWTTransform.reconstruct / reconstructFromLevel / reconstructLevels
 *                             core/modwt/MultiLevelMODWTTransform.java:339-446, :554-645
 *                           BatchMODWT.inverseMultiLevelAoS  ext/extensions/modwt/BatchMODWT.java:151-178
 *                           VectorWaveSwtAdapter.inverse / extractLevel  core/swt/VectorWaveSwtAdapter.java:435-487, :576-598
 *   vw_modwt1_forward_*     MODWTTransform.forward / forwardBatch  core/modwt/MODWTTransform.java:131-189, :486-614
 *                           BatchMODWT.singleLevelAoS  ext/extensions/modwt/BatchMODWT.java:62-79
 *   vw_modwt1_inverse_*     MODWTTransform.inverse / inverseBatch  core/modwt/MODWTTransform.java:203-299, :531-689
 *                           BatchMODWT.inverseSingleLevelAoS  ext/extensions/modwt/BatchMODWT.java:122-139
 *   vw_swt_denoise_*        VectorWaveSwtAdapter.denoise  core/swt/VectorWaveSwtAdapter.java:532-562
 *   vw_noise_sigma_*        VectorWaveSwtAdapter.estimateNoiseSigma  core/swt/VectorWaveSwtAdapter.java:627-645
 *   vw_threshold_*          MutableMultiLevelMODWTResult.applyThreshold  core/modwt/MutableMultiLevelMODWTResult.java:83-114
 *   vw_wavelet_denoise_*    WaveletDenoiser.denoise / denoiseMultiLevel / denoiseFixed
 *                             core/denoising/WaveletDenoiser.java:111-549
 *   vw_transpose_*          BatchSIMDMODWT.convertToSoA / convertFromSoA  ext/extensions/modwt/BatchSIMDMODWT.java:282-308
 *   vw_stream_*             BatchStreamingMODWT  ext/extensions/modwt/BatchStreamingMODWT.java:55-275
 *   vw_max_levels           MultiLevelMODWTTransform.getMaximumLevels  core/modwt/MultiLevelMODWTTransform.java:455-501, :693-695
 *   status codes            core/exception/ErrorCode.java:24-118 (see the table below)
 *
 * Memory: by default every array argument is a DEVICE pointer (hipMalloc /
 * torch CUDA storage) on the context's device, and work is enqueued on the
 * context's stream (the call returns after enqueueing unless VW_FLAG_SYNC or
 * validation needs a result).  With VW_FLAG_HOST_MEMORY all arrays are host
 * pointers: the engine stages them through its own device workspace and the
 * call is synchronous (the JNI/FFM path).  Filter taps (lo/hi) are always host
 * pointers of L doubles: the caller passes wavelet.lowPassDecomposition() /
 * highPassDecomposition() (== reconstruction filters for orthogonal
 * wavelets), exactly as the reference reads them.
 *
 * Layout: x[B][ldx] row-major (row b at x + b*ldx, ldx >= N), details
 * [J][B][N] (level 1 = finest first; BatchMODWT's detailPerLevel order),
 * approx [B][N], y [B][N].
 *
 * Threading: a context may be used from several host threads (calls are
 * serialized by its mutex and run on its stream); several contexts -- on one
 * device or on several -- run concurrently from different threads, e.g. through
 * vw_modwt_forward_multi_f64.  The engine retains no caller buffer after a
 * call returns (host-memory calls stage through a pool the context keeps).
 */
#ifndef VECTORWAVE_AMD_H
#define VECTORWAVE_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VW_API __attribute__((visibility("default")))

typedef struct vw_ctx vw_ctx;
typedef struct vw_stream vw_stream;
typedef int vw_status;

/* Status codes.  Reference ErrorCode (core/exception/ErrorCode.java) -> status. */
enum {
    VW_OK = 0,
    VW_ERR_NULL = 1,          /* NullPointerException                         */
    VW_ERR_EMPTY = 2,         /* VAL_006 VAL_EMPTY (empty signal / batch)     */
    VW_ERR_NONFINITE = 3,     /* VAL_003 VAL_NON_FINITE_VALUES; index via vw_last_error_index() */
    VW_ERR_LEVEL = 4,         /* CFG_004 CFG_INVALID_DECOMPOSITION_LEVEL      */
    VW_ERR_TOO_LARGE = 5,     /* VAL_005 VAL_TOO_LARGE (L_j > N)              */
    VW_ERR_BOUNDARY = 6,      /* CFG_003 CFG_UNSUPPORTED_BOUNDARY_MODE        */
    VW_ERR_ARG = 7,           /* IllegalArgumentException (shapes, ld, taps)  */
    VW_ERR_DEVICE = 8,        /* HIP runtime failure                          */
    VW_ERR_UNSUPPORTED = 9,   /* UnsupportedOperationException                */
    VW_ERR_STATE = 10         /* IllegalStateException (streaming)            */
};

/* BoundaryMode (core/api/BoundaryMode.java:20-50); CONSTANT is not a MODWT mode. */
enum { VW_PERIODIC = 0, VW_SYMMETRIC = 1, VW_ZERO_PADDING = 2 };

/* Wavelet identity for SymmetricAlignmentStrategy.decide, which compares
 * object identity (core/modwt/SymmetricAlignmentStrategy.java:65-96).
 * VW_WID_OTHER means "decide by filter length" (Haar if L <= 2, the L >= 12
 * rule, else the DB4 rule). */
enum {
    VW_WID_OTHER = 0, VW_WID_HAAR = 1, VW_WID_DB2 = 2, VW_WID_DB4 = 4, VW_WID_DB6 = 6,
    VW_WID_DB8 = 8, VW_WID_DB10 = 10, VW_WID_SYM4 = 104, VW_WID_SYM8 = 108,
    VW_WID_COIF1 = 201, VW_WID_COIF2 = 202, VW_WID_COIF3 = 203, VW_WID_COIF5 = 205
};

/* Semantics flags (OR-able). */
enum {
    /* MultiLevelMODWTTransform / SWT semantics: level cap 9 (calculateMaxLevels) and the
     * L_j > N guard.  Without it: BatchMODWT semantics (no cap, levels >= 1). */
    VW_FLAG_CORE_LEVELS = 1u << 0,
    /* Non-finite input check (ValidationUtils.validateFiniteValues) and result re-validation
     * (MODWTResultImpl ctor) -> VW_ERR_NONFINITE.  Fused into the kernels. */
    VW_FLAG_VALIDATE = 1u << 1,
    /* MultiLevelMODWTTransform.decompose PERIODIC dispatch: levels with N >= 1024 and
     * N/8 < L_j <= N/2 use WaveletOperations' FFT path, which zero-pads to nextPow2(N)
     * (core/modwt/MultiLevelMODWTTransform.java:734-742, core/util/FftHeuristics.java:30-34).
     * The engine computes that linear-over-nextPow2 convolution directly (no FFT). */
    VW_FLAG_FFT_SWITCH = 1u << 2,
    /* Fused multiply-add accumulation (faster; differs from the Java order by ~1 ulp per tap).
     * Default (flag clear) is EXACT: separate multiply and add in the reference's order,
     * bit-identical to vectorwave-core. */
    VW_FLAG_FMA = 1u << 3,
    /* All array arguments are host pointers (staged through the context workspace). */
    VW_FLAG_HOST_MEMORY = 1u << 4,
    /* Synchronize the context stream before returning. */
    VW_FLAG_SYNC = 1u << 5,
    /* Single-level inverse, SYMMETRIC: use MODWTTransform.inverseBatchOptimized's (t+l)
     * orientation (core/modwt/MODWTTransform.java:671-684) instead of inverse's (t-l). */
    VW_FLAG_BATCH_SYM_INVERSE = 1u << 6,
    /* Single-level forward: BatchSIMDMODWT.haarBatchMODWTSoA's hard-coded 0.5/-0.5 taps
     * (ext/extensions/modwt/BatchSIMDMODWT.java:86-140) when L == 2. */
    VW_FLAG_BATCH_HAAR = 1u << 7,
    /* The unvalidated callers' non-finite semantics (multi-level calls without VW_FLAG_VALIDATE):
     * the reference multiplies every tap of the upsampled filters, zeros included, so a NaN / +-Inf
     * turns each output whose window reaches it through a zero tap into NaN (0 * Inf)
     * -- BatchMODWT.multiLevelAoS (ext/extensions/modwt/BatchSIMDMODWT.java:384-424),
     * inverseMultiLevelAoS -> MultiLevelMODWTTransform.reconstruct (core/modwt/MultiLevelMODWTTransform.java
     * :339-349, :554-645), VectorWaveSwtAdapter.forwardParallel / inverse (core/swt/VectorWaveSwtAdapter.java
     * :210-335, :435-487).  With this flag every row where a level input holds a non-finite value (found
     * on the cascade's final output, a_J / y, which every such value reaches) is recomputed with the
     * reference's full-tap loops (exact arithmetic, also under VW_FLAG_FMA): NaN and +-Inf land exactly
     * where the reference puts them.  Costs one read of that output plane (none where the kernel probes
     * its own rows) and one fix-up launch.  Streaming
     * (vw_stream_*) ZERO / SYMMETRIC blocks and flushes are covered too: the history convolution
     * (BatchSIMDMODWT.generalBatchMODWTSoAWithScaledFiltersAndHistory :447-507) multiplies every tap, and
     * the recomputed rows rewrite the histories they leave for the next block. */
    VW_FLAG_REF_NONFINITE = 1u << 8
};

/* ---- context ---------------------------------------------------------- */
VW_API vw_status vw_ctx_create(int device, vw_ctx **out);
VW_API vw_status vw_ctx_destroy(vw_ctx *ctx);
/* Use an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL = own stream. */
VW_API vw_status vw_ctx_set_stream(vw_ctx *ctx, void *hip_stream);
/* Enqueue on the device's null (legacy default) stream, e.g. torch's default stream (handle 0). */
VW_API vw_status vw_ctx_use_null_stream(vw_ctx *ctx);
VW_API void *vw_ctx_get_stream(vw_ctx *ctx);
/* Kernel-path switches of this context (A/B experiments, tests), named like the environment
 * variables read once at vw_ctx_create (VW_FORCE_TILED, VW_MULTI_TILE, VW_INV_BLK, VW_NV, ...);
 * value < 0 restores the default.  VW_ERR_ARG for an unknown name. */
VW_API vw_status vw_ctx_set_option(vw_ctx *ctx, const char *key, int value);
VW_API vw_status vw_ctx_synchronize(vw_ctx *ctx);
VW_API int vw_ctx_device(vw_ctx *ctx);

/* Thread-local message / index of the last failing call on this thread. */
VW_API const char *vw_last_error(void);
VW_API int64_t vw_last_error_index(void);
VW_API const char *vw_version(void);
/* Signal numbers in this thread's VW_ERR_NONFINITE messages count from `base`: a caller that splits one
 * batch into row chunks (the JNI AoS natives, jni/vectorwave_amd_jni.c) sets each chunk's first row so the
 * message names the batch's signal (AmdMultiLevelMODWT.decomposeBatch's contract); 0 restores. */
VW_API void vw_set_signal_base(int64_t base);

/* ---- bookkeeping (host only) ------------------------------------------ */
/* getMaximumLevels(N) for a base filter of length L: largest J <= 9 with (L-1)*2^(J-1)+1 <= N. */
VW_API int vw_max_levels(int64_t N, int L);
/* (L-1)*2^(level-1)+1 */
VW_API int64_t vw_upsampled_length(int L, int level);

/* ---- multi-level MODWT ------------------------------------------------- */
VW_API vw_status vw_modwt_forward_f64(vw_ctx *ctx, const double *x, int64_t B, int64_t N, int64_t ldx,
                                      const double *lo, const double *hi, int L, int wavelet_id,
                                      int boundary, int J, unsigned flags,
                                      double *details, double *approx);
VW_API vw_status vw_modwt_forward_f32(vw_ctx *ctx, const float *x, int64_t B, int64_t N, int64_t ldx,
                                      const double *lo, const double *hi, int L, int wavelet_id,
                                      int boundary, int J, unsigned flags,
                                      float *details, float *approx);

/* detail_mask bit (j-1) set = use d_j, clear = zero details at level j
 * (reconstructFromLevel / reconstructLevels / extractLevel); approx_zero = 1 starts from a
 * zero approximation.  details may be NULL when detail_mask == 0; approx may be NULL when
 * approx_zero == 1.  Plain reconstruct: detail_mask = ~0u, approx_zero = 0. */
VW_API vw_status vw_modwt_inverse_f64(vw_ctx *ctx, const double *details, const double *approx,
                                      int64_t B, int64_t N, const double *lo, const double *hi, int L,
                                      int wavelet_id, int boundary, int J, unsigned detail_mask,
                                      int approx_zero, unsigned flags, double *y);
VW_API vw_status vw_modwt_inverse_f32(vw_ctx *ctx, const float *details, const float *approx,
                                      int64_t B, int64_t N, const double *lo, const double *hi, int L,
                                      int wavelet_id, int boundary, int J, unsigned detail_mask,
                                      int approx_zero, unsigned flags, float *y);

/* ---- one batch over several contexts (one host thread per context) ----------------------------
 * Replaces the reference's in-process parallelism over one batch call: BatchMODWT.multiLevelAoS /
 * inverseMultiLevelAoS (ext/extensions/modwt/BatchMODWT.java:90-111, :151-178) and the
 * VectorWaveSwtAdapter executor (core/swt/VectorWaveSwtAdapter.java:210-267).  The B rows are split
 * into n contiguous blocks (the first B % n blocks one row longer; min(n, B) blocks), block k runs on
 * ctxs[k] from its own host thread (ctxs[0] on the calling thread); the call returns when every
 * block is done.  Contexts may live on different devices or share one.  flags must include
 * VW_FLAG_HOST_MEMORY: the arrays are the caller's host arrays, laid out as the single-context
 * calls (details [J][B][N]); each thread stages its block through its context.  Errors: the first
 * failing block's status; vw_last_error() names the block. */
VW_API vw_status vw_modwt_forward_multi_f64(vw_ctx *const *ctxs, int nctx, const double *x, int64_t B, int64_t N,
                                            int64_t ldx, const double *lo, const double *hi, int L, int wavelet_id,
                                            int boundary, int J, unsigned flags, double *details, double *approx);
VW_API vw_status vw_modwt_inverse_multi_f64(vw_ctx *const *ctxs, int nctx, const double *details,
                                            const double *approx, int64_t B, int64_t N, const double *lo,
                                            const double *hi, int L, int wavelet_id, int boundary, int J,
                                            unsigned detail_mask, int approx_zero, unsigned flags, double *y);

/* Device-resident form of the two calls above (each device has its own context,
 * stream, input and output buffers; one host thread per device): context k works on ITS OWN device
 * buffers -- x[k] is rows[k] x ldx on ctxs[k]'s device, details[k] is [J][rows[k]][N], approx[k] and
 * y[k] are [rows[k]][N] -- so an FFM / JNI caller that keeps one batch shard resident per GPU calls all
 * of them at once with no host staging.  Host thread k enqueues on ctxs[k]'s stream (ctxs[0] on the
 * calling thread); the call returns when every context's work is enqueued, or finished with
 * VW_FLAG_SYNC.  rows[k] = 0 skips context k.  VW_FLAG_HOST_MEMORY is refused (VW_ERR_ARG).  Errors:
 * the first failing context's status; vw_last_error() names the context.
 * Replaces: BatchMODWT.multiLevelAoS / inverseMultiLevelAoS (ext/extensions/modwt/BatchMODWT.java:90-111,
 * :151-178) over a batch already sharded across devices. */
VW_API vw_status vw_modwt_forward_multi_dev_f64(vw_ctx *const *ctxs, int nctx, const double *const *x,
                                                const int64_t *rows, int64_t N, int64_t ldx, const double *lo,
                                                const double *hi, int L, int wavelet_id, int boundary, int J,
                                                unsigned flags, double *const *details, double *const *approx);
VW_API vw_status vw_modwt_inverse_multi_dev_f64(vw_ctx *const *ctxs, int nctx, const double *const *details,
                                                const double *const *approx, const int64_t *rows, int64_t N,
                                                const double *lo, const double *hi, int L, int wavelet_id,
                                                int boundary, int J, unsigned detail_mask, int approx_zero,
                                                unsigned flags, double *const *y);

/* ---- single-level MODWT (MODWTTransform: pairwise inverse sums, any N >= 1) --- */
VW_API vw_status vw_modwt1_forward_f64(vw_ctx *ctx, const double *x, int64_t B, int64_t N, int64_t ldx,
                                       const double *lo, const double *hi, int L, int boundary,
                                       unsigned flags, double *approx, double *detail);
VW_API vw_status vw_modwt1_inverse_f64(vw_ctx *ctx, const double *approx, const double *detail,
                                       int64_t B, int64_t N, const double *lo, const double *hi, int L,
                                       int boundary, unsigned flags, double *y);

/* ---- SWT denoise -------------------------------------------------------- */
/* threshold < 0: universal threshold sigma*sqrt(2 ln N), sigma = median(|d_1|)/0.6745 per signal;
 * threshold >= 0: that value on every detail level.  soft: 1 soft, 0 hard.
 * thresholds_out (optional, [B], same memory kind as y) receives the threshold used per signal. */
VW_API vw_status vw_swt_denoise_f64(vw_ctx *ctx, const double *x, int64_t B, int64_t N, int64_t ldx,
                                    const double *lo, const double *hi, int L, int wavelet_id,
                                    int boundary, int J, double threshold, int soft, unsigned flags,
                                    double *y, double *thresholds_out);
/* ---- AoS <-> SoA layout (BatchSIMDMODWT.convertToSoA / convertFromSoA) -- */
/* out[c][r] = in[r][c] for a rows x cols row-major matrix (out of place).  AoS double[B][N] -> the
 * facade's SoA double[N*B] (index t*B + b): rows = B, cols = N; back: rows = N, cols = B.
 * ext/extensions/modwt/BatchSIMDMODWT.java:282-308. */
VW_API vw_status vw_transpose_f64(vw_ctx *ctx, const double *in, int64_t rows, int64_t cols, unsigned flags,
                                  double *out);
VW_API vw_status vw_transpose_f32(vw_ctx *ctx, const float *in, int64_t rows, int64_t cols, unsigned flags,
                                  float *out);

/* ---- WaveletDenoiser ---------------------------------------------------- */
/* Replaces com.morphiqlabs.wavelet.denoising.WaveletDenoiser (core/denoising/WaveletDenoiser.java):
 *   levels == 0, method != FIXED : denoise(signal, method, type)            :124-143
 *   levels == 0, method == FIXED : denoiseFixed(signal, fixed_threshold, type) :354-364
 *   levels >= 1                  : denoiseMultiLevel(signal, levels, method, type) :155-170, with
 *                                  DenoisedMultiLevelResult's per-level thresholds :204-231
 *                                  (sigma = MAD(d_1)/0.6745, level j uses sigma / sqrt(2^j)).
 * method: VW_THR_* (calculateThreshold :394-436).  SURE needs N <= 16384 (VW_ERR_UNSUPPORTED).
 * soft: 1 SOFT, 0 HARD.  thresholds_out (optional, [max(levels,1)][B], same memory kind as y). */
#define VW_THR_UNIVERSAL 0
#define VW_THR_SURE 1
#define VW_THR_MINIMAX 2
#define VW_THR_BAYES 3
#define VW_THR_FIXED 4
VW_API vw_status vw_wavelet_denoise_f64(vw_ctx *ctx, const double *x, int64_t B, int64_t N, int64_t ldx,
                                        const double *lo, const double *hi, int L, int wavelet_id,
                                        int boundary, int levels, int method, double fixed_threshold, int soft,
                                        unsigned flags, double *y, double *thresholds_out);

/* sigma[b] = median(|coeffs[b][:]|) / 0.6745 (exact selection, even N = mean of middle pair). */
VW_API vw_status vw_noise_sigma_f64(vw_ctx *ctx, const double *coeffs, int64_t B, int64_t N,
                                    unsigned flags, double *sigma);
/* In-place soft/hard threshold of c[B][N] with per-signal thresholds thr[B] (device or host per flags). */
VW_API vw_status vw_threshold_f64(vw_ctx *ctx, double *c, int64_t B, int64_t N, const double *thr,
                                  int soft, unsigned flags);

/* ---- MODWTStreamingDenoiser statistics (device pointers only) ------------ */
/* core/modwt/streaming/MODWTStreamingDenoiser.java:133-272 with core/util/MathUtils.java:94-257.
 * median_out[b] = median(|x[b][:] - center[b]|) (center NULL: median(|x[b][:]|)), exact order
 * statistics, even N = mean of the middle pair (MathUtils.median); the two passes of
 * medianAbsoluteDeviation on non-negative data (any N; rows longer than 16384 with a center write the
 * deviations into a per-context scratch buffer first: it grows outside a capture only -- run such a
 * call once before recording it -- and never moves the workspace that recorded graphs use). */
VW_API vw_status vw_median_f64(vw_ctx *ctx, const double *x, int64_t B, int64_t N, const double *center,
                               unsigned flags, double *median_out);
/* out[0] = MathUtils.standardDeviation(x[0..N)) -- sequential sums, sqrt(ssd / (N-1)); N >= 2. */
VW_API vw_status vw_stddev_f64(vw_ctx *ctx, const double *x, int64_t N, unsigned flags, double *out);
/* updateNoiseEstimation's ring write: window[(start+k) % wsize] = |src[idx[k]]|, k < count <= wsize;
 * idx is a host array (the stratified sampling positions). */
VW_API vw_status vw_window_gather_abs_f64(vw_ctx *ctx, const double *src, const int32_t *idx, int64_t count,
                                          double *window, int64_t wsize, int64_t start);

/* ---- streaming (BatchStreamingMODWT) ------------------------------------ */
/* levels >= 1.  PERIODIC: every block independent (== vw_modwt_forward, no cap).
 * ZERO_PADDING / SYMMETRIC: per-level left history of L_j - 1 samples kept on the device. */
VW_API vw_status vw_stream_create(vw_ctx *ctx, const double *lo, const double *hi, int L,
                                  int boundary, int levels, vw_stream **out);
VW_API vw_status vw_stream_destroy(vw_stream *s);
/* block [B][n] -> details [levels][B][n], approx [B][n] (f64). */
VW_API vw_status vw_stream_process_f64(vw_stream *s, const double *block, int64_t B, int64_t n,
                                       unsigned flags, double *details, double *approx);
/* Synthetic tail of tail_len samples (ZERO/SYMMETRIC only); tail_len <= min history length. */
VW_API vw_status vw_stream_flush_f64(vw_stream *s, int64_t tail_len, unsigned flags,
                                     double *details, double *approx);
VW_API int64_t vw_stream_history_length(vw_stream *s, int level);
/* Batch of the last processed block (the rows a flush emits); -1 before the first block. */
VW_API int64_t vw_stream_batch(vw_stream *s);

/* ---- captured steps ------------------------------------------------------- */
/* A caller that repeats the same calls on the same buffers (a JNI server's per-batch loop, a
 * benchmark) records them once and replays them with one host call: host planning, argument
 * packing and the per-kernel launch cost are paid at capture.  Between vw_capture_begin and
 * vw_capture_end the context's calls are recorded (HIP stream capture of the context stream),
 * not run; calls that must synchronize (VW_FLAG_VALIDATE, VW_FLAG_HOST_MEMORY, VW_FLAG_SYNC, a
 * fixed denoise threshold, stream flush, workspace growth) fail with VW_ERR_STATE.  The context
 * must be bound to a stream other than the null stream.  No reference counterpart: the Java
 * callers re-enter per call; this is the device-side amortisation of that loop. */
typedef struct vw_graph vw_graph;
VW_API vw_status vw_capture_begin(vw_ctx *ctx);
VW_API vw_status vw_capture_end(vw_ctx *ctx, vw_graph **out);
/* Replays the recorded calls `count` times, in order, on the context's stream (asynchronous).
 * Timing enabled during the capture (vw_ctx_enable_timing) records every launch's HIP events as
 * event nodes of the graph; with timing enabled at launch, vw_ctx_kernel_time then reports the
 * launches of the last replay of the call. */
VW_API vw_status vw_graph_launch(vw_graph *graph, int64_t count);
VW_API vw_status vw_graph_destroy(vw_graph *graph);

/* ---- pipelined round trips ---------------------------------------------------
 * A caller that runs forward + inverse over successive batches (a server's per-batch loop over
 * BatchMODWT.multiLevelAoS then inverseMultiLevelAoS, ext/extensions/modwt/BatchMODWT.java:90-111,
 * :151-178; the blocks of BatchStreamingMODWT) keeps R >= 2 device buffer sets and lets the engine
 * issue the steps: step i works on set i mod R, its forward on fwd_ctx's stream, then (event) its
 * inverse on inv_ctx's stream; step i's forward waits for step i - R's inverse.  Step i + 1's forward
 * thus overlaps step i's inverse -- what keeps a small batch (<= 2 signals per CU) from leaving the
 * GPU half idle at each pass's ends -- and the steps are issued from C++, not one host call per pass.
 * x[r] is [B][N] (ldx = N), details[r] [J][B][N], approx[r] and y[r] [B][N], elements of elem_bytes
 * (8: f64, 4: f32), all on the contexts' device (both contexts on one device; they may be the same
 * context, which serialises the steps).  flags: FMA / CORE_LEVELS; SYNC, VALIDATE and HOST_MEMORY are
 * refused (VW_ERR_ARG).  vw_pipeline_run enqueues `steps` steps and returns; vw_pipeline_join makes
 * fwd_ctx's stream wait for every enqueued inverse (then the next run starts with no pending edge).
 * Destroying a context kills its pipelines (run / join then return VW_ERR_STATE; a destroy waits for a run
 * that is issuing its steps); run / join while either context is capturing return VW_ERR_STATE.  As for
 * every call, a context must not be destroyed while another thread still passes it in. */
typedef struct vw_pipeline vw_pipeline;
VW_API vw_status vw_pipeline_create(vw_ctx *fwd_ctx, vw_ctx *inv_ctx, int elem_bytes, int sets, void *const *x,
                                    void *const *details, void *const *approx, void *const *y, int64_t B,
                                    int64_t N, const double *lo, const double *hi, int L, int wavelet_id,
                                    int boundary, int J, unsigned flags, vw_pipeline **out);
VW_API vw_status vw_pipeline_run(vw_pipeline *p, int64_t steps);
VW_API vw_status vw_pipeline_join(vw_pipeline *p);
/* buffer set of the most recently enqueued step (-1 before the first) */
VW_API int64_t vw_pipeline_last_set(vw_pipeline *p);
VW_API vw_status vw_pipeline_destroy(vw_pipeline *p);

/* ---- device utilities ---------------------------------------------------- */
/* x[i] = 2*u - 1 with u = (splitmix64(seed ^ (offset + i)) >> 11) * 2^-53. */
VW_API vw_status vw_fill_uniform_f64(vw_ctx *ctx, double *x, int64_t count, uint64_t seed, int64_t offset);
VW_API vw_status vw_fill_uniform_f32(vw_ctx *ctx, float *x, int64_t count, uint64_t seed, int64_t offset);
VW_API vw_status vw_device_alloc(vw_ctx *ctx, int64_t bytes, void **out);
VW_API vw_status vw_device_free(vw_ctx *ctx, void *p);
VW_API vw_status vw_memcpy(vw_ctx *ctx, void *dst, const void *src, int64_t bytes, int kind /*0 H2D,1 D2H,2 D2D*/);

/* Timing: average duration (ms) of the last `count` launches of the dominant kernel family
 * recorded with HIP events on the context stream when profiling is enabled. */
VW_API vw_status vw_ctx_enable_timing(vw_ctx *ctx, int enable);
VW_API vw_status vw_ctx_kernel_time(vw_ctx *ctx, const char *family, double *total_ms, int64_t *launches);
VW_API vw_status vw_ctx_reset_timing(vw_ctx *ctx);
/* Start / end (ms after ref_event, a hipEvent_t recorded earlier on any stream of the device) of the
 * timed launches of `family` not yet collected by vw_ctx_kernel_time: the wall window of a kernel
 * family when several contexts run concurrently.  *count = launches found (at most max written). */
VW_API vw_status vw_ctx_kernel_spans(vw_ctx *ctx, const char *family, void *ref_event, int64_t max,
                                     double *start_ms, double *end_ms, int64_t *count);

#ifdef __cplusplus
}
#endif
#endif /* VECTORWAVE_AMD_H */

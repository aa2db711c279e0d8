package com.morphiqlabs.wavelet.amd;

import com.morphiqlabs.wavelet.api.BoundaryMode;
import com.morphiqlabs.wavelet.api.Coiflet;
import com.morphiqlabs.wavelet.api.Daubechies;
import com.morphiqlabs.wavelet.api.Haar;
import com.morphiqlabs.wavelet.api.Symlet;
import com.morphiqlabs.wavelet.api.Wavelet;
import com.morphiqlabs.wavelet.exception.ErrorCode;
import com.morphiqlabs.wavelet.exception.InvalidArgumentException;
import com.morphiqlabs.wavelet.exception.InvalidConfigurationException;
import com.morphiqlabs.wavelet.exception.InvalidSignalException;
import com.morphiqlabs.wavelet.exception.InvalidStateException;
import com.morphiqlabs.wavelet.exception.WaveletTransformException;

import java.nio.ByteBuffer;

/**
 * Native methods of the MI355X MODWT/SWT engine (jni/vectorwave_amd_jni.c over include/vectorwave_amd.h).
 *
 * <p>One native call per batch.  double[] arguments are copied into native memory and back (no Java
 * array is pinned while the GPU works); the {@code *Direct} methods take direct ByteBuffers and copy
 * nothing.  Every method returns the engine's status; {@link #check(int)} turns it into the exception the
 * reference throws for the same condition (INTEGRATION.md section 3).  Malformed arguments the native glue
 * finds itself (null or ragged rows, short arrays, bad taps) throw IllegalArgumentException /
 * NullPointerException from the native call directly.
 *
 * <p>Status: the C glue behind these declarations is compiled and exercised against a fake JNIEnv
 * (tests/test_jni_glue.py); the Java sources of this package have never been compiled here (no JDK in the
 * build image).  They target Java 21 (pattern matching for instanceof, records) and the reference's jars:
 * experimental until compiled against them (INTEGRATION.md section 2).
 */
public final class AmdNative {
    static final boolean LOADED;

    static {
        boolean ok;
        try {
            System.loadLibrary("vectorwave_amd_jni");  // links libvectorwave_amd.so
            ok = true;
        } catch (UnsatisfiedLinkError e) {
            ok = false;
        }
        LOADED = ok;
    }

    private AmdNative() {}

    // include/vectorwave_amd.h flags
    public static final int FLAG_CORE_LEVELS = 1;
    public static final int FLAG_VALIDATE = 1 << 1;
    public static final int FLAG_FFT_SWITCH = 1 << 2;
    public static final int FLAG_FMA = 1 << 3;
    public static final int FLAG_BATCH_SYM_INVERSE = 1 << 6;
    public static final int FLAG_BATCH_HAAR = 1 << 7;
    /** Unvalidated callers: NaN / +-Inf spread through the zero taps exactly as the reference's loops. */
    public static final int FLAG_REF_NONFINITE = 1 << 8;

    // include/vectorwave_amd.h status codes
    static final int VW_OK = 0, VW_ERR_NULL = 1, VW_ERR_EMPTY = 2, VW_ERR_NONFINITE = 3, VW_ERR_LEVEL = 4,
            VW_ERR_TOO_LARGE = 5, VW_ERR_BOUNDARY = 6, VW_ERR_ARG = 7, VW_ERR_DEVICE = 8,
            VW_ERR_UNSUPPORTED = 9, VW_ERR_STATE = 10;

    static native long ctxCreate(int device);
    static native int ctxDestroy(long ctx);
    static native int maxLevels(long n, int L);
    static native String lastError();
    static native long lastErrorIndex();

    // MODWTTransform.forward / forwardBatch (x: B*N) and inverse / inverseBatch
    static native int modwt1Forward(long ctx, double[] x, int B, int N, double[] lo, double[] hi, int boundary,
                                    int flags, double[] approx, double[] detail);
    static native int modwt1Inverse(long ctx, double[] approx, double[] detail, int B, int N, double[] lo,
                                    double[] hi, int boundary, int flags, double[] y);

    // MultiLevelMODWTTransform.decompose / BatchMODWT.multiLevelAoS (details: J*B*N, level 1 first)
    static native int modwtForward(long ctx, double[] x, int B, int N, double[] lo, double[] hi, int waveletId,
                                   int boundary, int J, int flags, double[] details, double[] approx);
    // MultiLevelMODWTTransform.reconstruct / reconstructFromLevel / reconstructLevels
    static native int modwtInverse(long ctx, double[] details, double[] approx, int B, int N, double[] lo,
                                   double[] hi, int waveletId, int boundary, int J, int detailMask,
                                   boolean approxZero, int flags, double[] y);
    // one batch over several contexts (one engine thread per context)
    static native int modwtForwardMulti(long[] ctxs, double[] x, int B, int N, double[] lo, double[] hi,
                                        int waveletId, int boundary, int J, int flags, double[] details,
                                        double[] approx);
    // VectorWaveSwtAdapter.denoise (threshold < 0: universal)
    static native int swtDenoise(long ctx, double[] x, int B, int N, double[] lo, double[] hi, int waveletId,
                                 int boundary, int J, double threshold, boolean soft, int flags, double[] y,
                                 double[] thresholdsOut);
    // WaveletDenoiser (method = ThresholdMethod ordinal: UNIVERSAL, SURE, MINIMAX, BAYES, FIXED)
    static native int waveletDenoise(long ctx, double[] x, int B, int N, double[] lo, double[] hi, int waveletId,
                                     int boundary, int levels, int method, double fixedThreshold, boolean soft,
                                     int flags, double[] y, double[] thresholdsOut);

    // AoS batches as the Java API holds them (double[][] signals, double[][][] details [levels][batch][length]):
    // rows gathered / scattered by the native side in chunks (no flattening here, no int-sized B*N product)
    static native int modwtForwardAoS(long ctx, double[][] x, double[] lo, double[] hi, int waveletId, int boundary,
                                      int J, int flags, double[][][] details, double[][] approx);
    static native int modwtInverseAoS(long ctx, double[][][] details, double[][] approx, double[] lo, double[] hi,
                                      int waveletId, int boundary, int flags, double[][] y);
    static native int swtDenoiseAoS(long ctx, double[][] x, double[] lo, double[] hi, int waveletId, int boundary,
                                    int J, double threshold, boolean soft, int flags, double[][] y);

    // VectorWaveSwtAdapter.estimateNoiseSigma per row of B x N coefficients (exact median on the device)
    static native int noiseSigma(long ctx, double[] coeffs, int B, int N, double[] sigmaOut);

    // BatchStreamingMODWT ZERO_PADDING / SYMMETRIC: per-level history on the device between blocks
    static native long streamCreate(long ctx, double[] lo, double[] hi, int boundary, int levels);
    static native int streamDestroy(long stream);
    static native long streamHistoryLength(long stream, int level);
    static native int streamProcessAoS(long stream, double[][] block, double[][][] details, double[][] approx);
    static native int streamFlushAoS(long stream, int tailLength, double[][][] details, double[][] approx);

    // direct (off-heap) buffers, native byte order: no copy, no pinning
    static native int modwtForwardDirect(long ctx, ByteBuffer x, int B, int N, double[] lo, double[] hi,
                                         int waveletId, int boundary, int J, int flags, ByteBuffer details,
                                         ByteBuffer approx);
    static native int modwtInverseDirect(long ctx, ByteBuffer details, ByteBuffer approx, int B, int N,
                                         double[] lo, double[] hi, int waveletId, int boundary, int J, int flags,
                                         ByteBuffer y);

    /** Boundary mode to the engine's code (PERIODIC 0, SYMMETRIC 1, ZERO_PADDING 2; CONSTANT is refused). */
    static int boundary(BoundaryMode m) {
        switch (m) {
            case PERIODIC: return 0;
            case SYMMETRIC: return 1;
            case ZERO_PADDING: return 2;
            default:
                throw new InvalidConfigurationException(ErrorCode.CFG_UNSUPPORTED_BOUNDARY_MODE,
                        "Unsupported boundary mode: " + m);
        }
    }

    /**
     * The wavelet's identity code (VW_WID_*): SymmetricAlignmentStrategy.decide
     * (core/modwt/SymmetricAlignmentStrategy.java:43-117) chooses by object identity.
     */
    static int waveletId(Wavelet w) {
        if (w == Haar.INSTANCE) return 1;
        if (w == Daubechies.DB2) return 2;
        if (w == Daubechies.DB4) return 4;
        if (w == Daubechies.DB6) return 6;
        if (w == Daubechies.DB8) return 8;
        if (w == Daubechies.DB10) return 10;
        if (w == Symlet.SYM4) return 104;
        if (w == Symlet.SYM8) return 108;
        if (w == Coiflet.COIF1) return 201;
        if (w == Coiflet.COIF2) return 202;
        if (w == Coiflet.COIF3) return 203;
        if (w == Coiflet.COIF5) return 205;
        return 0;  // VW_WID_OTHER: decided by filter length, as the reference's fall-through branches
    }

    /** Throws what the reference throws for the condition behind a non-zero status. */
    static void check(int st) {
        if (st == VW_OK) return;
        String msg = lastError();
        switch (st) {
            case VW_ERR_NULL: throw new NullPointerException(msg);
            case VW_ERR_EMPTY: throw new InvalidSignalException(ErrorCode.VAL_EMPTY, msg);
            case VW_ERR_NONFINITE:
                throw new InvalidSignalException(ErrorCode.VAL_NON_FINITE_VALUES,
                        msg + " [index " + lastErrorIndex() + "]");
            case VW_ERR_LEVEL: throw new InvalidArgumentException(ErrorCode.CFG_INVALID_DECOMPOSITION_LEVEL, msg);
            case VW_ERR_TOO_LARGE: throw new InvalidArgumentException(ErrorCode.VAL_TOO_LARGE, msg);
            case VW_ERR_BOUNDARY:
                throw new InvalidConfigurationException(ErrorCode.CFG_UNSUPPORTED_BOUNDARY_MODE, msg);
            case VW_ERR_ARG: throw new IllegalArgumentException(msg);
            case VW_ERR_UNSUPPORTED: throw new UnsupportedOperationException(msg);
            case VW_ERR_STATE: throw new InvalidStateException(msg);
            default: throw new WaveletTransformException(msg);
        }
    }
}

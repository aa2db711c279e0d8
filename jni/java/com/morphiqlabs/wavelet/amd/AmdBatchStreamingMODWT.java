package com.morphiqlabs.wavelet.amd;

import com.morphiqlabs.wavelet.api.BoundaryMode;
import com.morphiqlabs.wavelet.api.DiscreteWavelet;
import com.morphiqlabs.wavelet.extensions.modwt.BatchMODWT;

/**
 * MI355X drop-in for ext/extensions/modwt/BatchStreamingMODWT.java (:19-470): the same builder, methods,
 * messages and result records.  PERIODIC blocks are independent and go through {@link AmdBatchMODWT}, as the
 * reference sends them to BatchMODWT (:63-65, :115-117).  ZERO_PADDING / SYMMETRIC blocks run on an engine
 * stream (vw_stream_*): each level's left history of L_j - 1 samples per signal stays in device memory between
 * blocks, initialised from the first block (zeros, or the block's half-sample mirror,
 * fillSymmetricHistoryFromSoA :326-335) and updated from each level's input (updateHistoryFromSoA :337-352);
 * a change of batch size re-initialises it (ensureHistoryCapacity :310-324); {@code flush*} (:181-275) runs
 * the synthetic tail through every level's history.  Results bit-identical to the reference in EXACT mode
 * ({@link AmdRuntime}).  Stateful and single-threaded, as the reference; {@link #close()} frees the stream.
 *
 * <p>Not built or run in this repository (no JDK in its build image): INTEGRATION.md section 2.  The natives
 * it calls are exercised through a fake JNIEnv (tests/test_jni_glue.py).
 */
public final class AmdBatchStreamingMODWT implements AutoCloseable {
    private final DiscreteWavelet wavelet;
    private final BoundaryMode boundaryMode;
    private final int levels;
    private long stream;  // engine stream (ZERO_PADDING / SYMMETRIC), 0 = none yet or closed
    private int lastBatch = -1;

    private AmdBatchStreamingMODWT(Builder b) {
        this.wavelet = b.wavelet;
        this.boundaryMode = b.boundaryMode;
        this.levels = b.levels;
        if (levels < 1) throw new IllegalArgumentException("levels must be >= 1");
        AmdNative.boundary(boundaryMode);  // CONSTANT -> CFG_UNSUPPORTED_BOUNDARY_MODE
    }

    public static Builder builder() {
        return new Builder();
    }

    private long stream() {
        if (stream == 0L) {
            stream = AmdNative.streamCreate(AmdRuntime.ctx(), wavelet.lowPassDecomposition(),
                    wavelet.highPassDecomposition(), AmdNative.boundary(boundaryMode), levels);
            if (stream == 0L) AmdNative.check(AmdNative.VW_ERR_ARG);
        }
        return stream;
    }

    /** processSingleLevel(block) (:55-102). */
    public BatchMODWT.SingleLevelResult processSingleLevel(double[][] block) {
        ensureLevels(1);
        validateAoS(block);
        if (boundaryMode == BoundaryMode.PERIODIC) return AmdBatchMODWT.singleLevelAoS(wavelet, block);
        final int batch = block.length, n = block[0].length;
        double[][][] det = new double[1][batch][n];
        double[][] app = new double[batch][n];
        AmdNative.check(AmdNative.streamProcessAoS(stream(), block, det, app));
        lastBatch = batch;
        return new BatchMODWT.SingleLevelResult(app, det[0]);
    }

    /** processMultiLevel(block) (:110-175). */
    public BatchMODWT.MultiLevelResult processMultiLevel(double[][] block) {
        validateAoS(block);
        if (boundaryMode == BoundaryMode.PERIODIC) return AmdBatchMODWT.multiLevelAoS(wavelet, block, levels);
        final int batch = block.length, n = block[0].length;
        double[][][] det = new double[levels][batch][n];
        double[][] app = new double[batch][n];
        AmdNative.check(AmdNative.streamProcessAoS(stream(), block, det, app));
        lastBatch = batch;
        return new BatchMODWT.MultiLevelResult(det, app);
    }

    /** flushSingleLevel(tailLength) (:181-225). */
    public BatchMODWT.SingleLevelResult flushSingleLevel(int tailLength) {
        ensureLevels(1);
        if (boundaryMode == BoundaryMode.PERIODIC) {
            throw new UnsupportedOperationException("Flush is only applicable to ZERO_PADDING/SYMMETRIC");
        }
        if (tailLength <= 0) return new BatchMODWT.SingleLevelResult(new double[0][0], new double[0][0]);
        if (stream == 0L || lastBatch <= 0) throw new IllegalStateException("No prior blocks processed; cannot flush");
        final int histLen = getHistoryLengthForLevel(1);
        if (tailLength > histLen) {
            throw new IllegalArgumentException(String.format(
                    "tailLength (%d) exceeds maximum allowed for this level (%d). "
                            + "Use getMinFlushTailLength() to choose a valid tail length.", tailLength, histLen));
        }
        double[][][] det = new double[1][lastBatch][tailLength];
        double[][] app = new double[lastBatch][tailLength];
        AmdNative.check(AmdNative.streamFlushAoS(stream, tailLength, det, app));
        return new BatchMODWT.SingleLevelResult(app, det[0]);
    }

    /** flushMultiLevel(tailLength) (:231-275). */
    public BatchMODWT.MultiLevelResult flushMultiLevel(int tailLength) {
        if (boundaryMode == BoundaryMode.PERIODIC) {
            throw new UnsupportedOperationException("Flush is only applicable to ZERO_PADDING/SYMMETRIC");
        }
        if (tailLength <= 0) return new BatchMODWT.MultiLevelResult(new double[levels][0][0], new double[0][0]);
        if (stream == 0L || lastBatch <= 0) throw new IllegalStateException("No prior blocks processed; cannot flush");
        final int minHist = getMinFlushTailLength();
        if (tailLength > minHist) {
            throw new IllegalArgumentException(String.format(
                    "tailLength (%d) exceeds maximum allowed across levels (%d). "
                            + "Use getMinFlushTailLength() to choose a valid tail length.", tailLength, minHist));
        }
        double[][][] det = new double[levels][lastBatch][tailLength];
        double[][] app = new double[lastBatch][tailLength];
        AmdNative.check(AmdNative.streamFlushAoS(stream, tailLength, det, app));
        return new BatchMODWT.MultiLevelResult(det, app);
    }

    /** getMinFlushTailLength() (:382-385): min over levels of L_j - 1. */
    public int getMinFlushTailLength() {
        int m = Integer.MAX_VALUE;
        for (int j = 1; j <= levels; j++) m = Math.min(m, getHistoryLengthForLevel(j));
        return m;
    }

    /** getHistoryLengthForLevel(level) (:394-400): L_j - 1. */
    public int getHistoryLengthForLevel(int level) {
        if (level < 1 || level > levels) throw new IllegalArgumentException("level must be in [1," + levels + "]");
        final long L = wavelet.lowPassDecomposition().length;
        return (int) ((L - 1) * (1L << (level - 1)));
    }

    /** suggestFlushTailLength() (:409-413). */
    public int suggestFlushTailLength() {
        return levels == 1 ? getHistoryLengthForLevel(1) : getMinFlushTailLength();
    }

    @Override
    public void close() {
        if (stream != 0L) {
            AmdNative.streamDestroy(stream);
            stream = 0L;
        }
    }

    private void ensureLevels(int expected) {
        if (levels != expected) {
            throw new IllegalStateException("This instance is configured for levels=" + levels + ", expected=" + expected);
        }
    }

    /** validateAoS (:283-290), the reference's messages. */
    private static void validateAoS(double[][] a) {
        if (a == null || a.length == 0) throw new IllegalArgumentException("block must be non-null");
        if (a[0] == null) throw new IllegalArgumentException("all rows must have equal length");
        final int n = a[0].length;
        if (n == 0) throw new IllegalArgumentException("block length must be > 0");
        for (int i = 1; i < a.length; i++) {
            if (a[i] == null || a[i].length != n) throw new IllegalArgumentException("all rows must have equal length");
        }
    }

    /** BatchStreamingMODWT.Builder (:421-462). */
    public static final class Builder {
        private DiscreteWavelet wavelet;
        private BoundaryMode boundaryMode = BoundaryMode.PERIODIC;
        private int levels = 1;

        public Builder() {}

        public Builder wavelet(DiscreteWavelet w) {
            this.wavelet = w;
            return this;
        }

        public Builder boundary(BoundaryMode mode) {
            this.boundaryMode = mode;
            return this;
        }

        public Builder levels(int levels) {
            this.levels = levels;
            return this;
        }

        public AmdBatchStreamingMODWT build() {
            if (wavelet == null) throw new IllegalArgumentException("wavelet must be set");
            return new AmdBatchStreamingMODWT(this);
        }
    }
}

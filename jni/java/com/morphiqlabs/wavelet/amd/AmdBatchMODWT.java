package com.morphiqlabs.wavelet.amd;

import com.morphiqlabs.wavelet.api.DiscreteWavelet;
import com.morphiqlabs.wavelet.extensions.modwt.BatchMODWT;

/**
 * MI355X drop-in for vectorwave-extensions' batch facade,
 * ext/extensions/modwt/BatchMODWT.java:33-212: the same four static methods, the same argument meaning,
 * validation messages and result records ({@link BatchMODWT.SingleLevelResult},
 * {@link BatchMODWT.MultiLevelResult}), computed by the engine's HIP kernels -- the north_star hot path
 * (db4 J=6 over 4096 x 4096 is {@code multiLevelAoS} + {@code inverseMultiLevelAoS}).
 *
 * <p>Semantics as the reference: PERIODIC boundary, no level cap and no finite check on the forward
 * (BatchSIMDMODWT.batchMultiLevelMODWTSoA, :343-424), the inverse = core
 * MultiLevelMODWTTransform.reconstruct per signal (:151-178); the single-level inverse = core
 * MODWTTransform.inverse per signal (:121-139).  Bit-identical to those in EXACT mode (the default,
 * {@link AmdRuntime}), non-finite samples included: both multi-level calls pass FLAG_REF_NONFINITE, so a
 * NaN / +-Inf spreads through the zero taps of the upsampled filters exactly as the reference's loops.
 *
 * <p>Memory: {@code double[][]} rows go to the engine without a flattened copy on the Java heap (the native
 * side gathers rows into its staging in chunks of at most 512 MiB), so batches whose B * N or
 * levels * B * N exceed Integer.MAX_VALUE (e.g. 256 blocks of 2^20 samples, 10 levels) work.
 *
 * <p>Not built or run in this repository (no JDK in its build image; jni/Makefile skips without
 * {@code $JAVA_HOME/include/jni.h}): see INTEGRATION.md section 2 for its status.
 */
public final class AmdBatchMODWT {
    private AmdBatchMODWT() {}

    /**
     * BatchMODWT.singleLevelAoS (:62-79 over BatchSIMDMODWT.batchMODWTSoA, :64-140): approximation and detail
     * of one PERIODIC level, Haar with the batch path's 0.5 / -0.5 taps (FLAG_BATCH_HAAR).
     */
    public static BatchMODWT.SingleLevelResult singleLevelAoS(DiscreteWavelet wavelet, double[][] signals) {
        validateAoS(signals);
        final int batch = signals.length;
        final int n = signals[0].length;
        final int flags = AmdRuntime.FMA | (wavelet instanceof com.morphiqlabs.wavelet.api.Haar
                ? AmdNative.FLAG_BATCH_HAAR : 0);
        double[][] approx = new double[batch][n];
        double[][] detail = new double[batch][n];
        final int rows = chunkRows(n, batch);
        for (int b0 = 0; b0 < batch; b0 += rows) {
            final int nb = Math.min(rows, batch - b0);
            double[] flat = flatten(signals, b0, nb, n);
            double[] a = new double[nb * n];
            double[] d = new double[nb * n];
            AmdNative.check(AmdNative.modwt1Forward(AmdRuntime.ctx(), flat, nb, n, wavelet.lowPassDecomposition(),
                    wavelet.highPassDecomposition(), 0, flags, a, d));
            unflatten(a, approx, b0, nb, n);
            unflatten(d, detail, b0, nb, n);
        }
        return new BatchMODWT.SingleLevelResult(approx, detail);
    }

    /** BatchMODWT.multiLevelAoS (:90-111): details [levels][batch][length] and the final approximation. */
    public static BatchMODWT.MultiLevelResult multiLevelAoS(DiscreteWavelet wavelet, double[][] signals, int levels) {
        if (levels < 1) throw new IllegalArgumentException("levels must be >= 1");
        validateAoS(signals);
        final int batch = signals.length;
        final int n = signals[0].length;
        checkBatchReach(wavelet, n, levels);
        double[][][] details = new double[levels][batch][n];
        double[][] approx = new double[batch][n];
        AmdNative.check(AmdNative.modwtForwardAoS(AmdRuntime.ctx(), signals, wavelet.lowPassDecomposition(),
                wavelet.highPassDecomposition(), AmdNative.waveletId(wavelet), 0, levels,
                AmdRuntime.FMA | AmdNative.FLAG_REF_NONFINITE, details, approx));
        return new BatchMODWT.MultiLevelResult(details, approx);
    }

    /** BatchMODWT.inverseSingleLevelAoS (:121-139): core MODWTTransform.inverse per signal (pairwise sums). */
    public static double[][] inverseSingleLevelAoS(DiscreteWavelet wavelet, double[][] approx, double[][] detail) {
        validateAoS(approx);
        validateAoS(detail);
        final int batch = approx.length;
        if (detail.length != batch || detail[0].length != approx[0].length) {
            throw new IllegalArgumentException("approx/detail shapes must match");
        }
        final int n = approx[0].length;
        double[][] out = new double[batch][n];
        final int rows = chunkRows(n, batch);
        for (int b0 = 0; b0 < batch; b0 += rows) {
            final int nb = Math.min(rows, batch - b0);
            double[] y = new double[nb * n];
            AmdNative.check(AmdNative.modwt1Inverse(AmdRuntime.ctx(), flatten(approx, b0, nb, n),
                    flatten(detail, b0, nb, n), nb, n, wavelet.lowPassReconstruction(),
                    wavelet.highPassReconstruction(), 0, AmdRuntime.FMA, y));
            unflatten(y, out, b0, nb, n);
        }
        return out;
    }

    /** BatchMODWT.inverseMultiLevelAoS (:151-178): core MultiLevelMODWTTransform.reconstruct per signal. */
    public static double[][] inverseMultiLevelAoS(DiscreteWavelet wavelet, double[][][] detailPerLevel,
                                                  double[][] finalApprox) {
        if (detailPerLevel == null || detailPerLevel.length == 0) {
            throw new IllegalArgumentException("levels must be > 0");
        }
        final int levels = detailPerLevel.length;
        validateAoS(finalApprox);
        final int batch = finalApprox.length;
        final int n = finalApprox[0].length;
        for (int l = 0; l < levels; l++) {
            if (detailPerLevel[l] == null || detailPerLevel[l].length != batch) {
                throw new IllegalArgumentException("detailPerLevel[L] must be non-null and length=batch for all L");
            }
            for (int b = 0; b < batch; b++) {
                if (detailPerLevel[l][b] == null || detailPerLevel[l][b].length != n) {
                    throw new IllegalArgumentException("all detail rows must have consistent length");
                }
            }
        }
        double[][] out = new double[batch][n];
        // core MultiLevelMODWTTransform.reconstruct: its level semantics (FLAG_CORE_LEVELS)
        AmdNative.check(AmdNative.modwtInverseAoS(AmdRuntime.ctx(), detailPerLevel, finalApprox,
                wavelet.lowPassReconstruction(), wavelet.highPassReconstruction(), AmdNative.waveletId(wavelet), 0,
                AmdRuntime.FMA | AmdNative.FLAG_CORE_LEVELS | AmdNative.FLAG_REF_NONFINITE, out));
        return out;
    }

    /**
     * BatchSIMDMODWT.generalBatchMODWTSoAWithScaledFilters (:384-424) indexes (t - l + N) % N: an upsampled
     * filter longer than N + 1 makes that index negative and the reference throws
     * ArrayIndexOutOfBoundsException at the first such level; so does this facade, before any work.
     */
    static void checkBatchReach(DiscreteWavelet wavelet, int n, int levels) {
        final long L = wavelet.lowPassDecomposition().length;
        for (int j = 1; j <= levels; j++) {
            final long lj = (L - 1) * (1L << Math.min(j - 1, 62)) + 1;
            if (lj > (long) n + 1) {
                throw new ArrayIndexOutOfBoundsException("Index " + (n - lj + 1) + " out of bounds for length " + n);
            }
        }
    }

    /** Rows per flat chunk so that rows * n stays a valid Java array length (no int overflow). */
    static int chunkRows(int n, int batch) {
        return (int) Math.max(1L, Math.min((long) batch, (Integer.MAX_VALUE - 8L) / n));
    }

    static double[] flatten(double[][] rows, int b0, int nb, int n) {
        double[] flat = new double[Math.multiplyExact(nb, n)];
        for (int b = 0; b < nb; b++) {
            System.arraycopy(rows[b0 + b], 0, flat, b * n, n);
        }
        return flat;
    }

    static void unflatten(double[] flat, double[][] rows, int b0, int nb, int n) {
        for (int b = 0; b < nb; b++) {
            System.arraycopy(flat, b * n, rows[b0 + b], 0, n);
        }
    }

    /** BatchMODWT.validateAoS (:201-212), same messages. */
    static void validateAoS(double[][] signals) {
        if (signals == null || signals.length == 0) {
            throw new IllegalArgumentException("signals must be non-null and non-empty");
        }
        if (signals[0] == null) {
            throw new IllegalArgumentException("all signals must be non-null and same length");
        }
        final int n = signals[0].length;
        if (n == 0) throw new IllegalArgumentException("signal length must be > 0");
        for (int i = 1; i < signals.length; i++) {
            if (signals[i] == null || signals[i].length != n) {
                throw new IllegalArgumentException("all signals must be non-null and same length");
            }
        }
    }
}

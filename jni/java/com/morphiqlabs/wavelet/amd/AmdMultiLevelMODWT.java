package com.morphiqlabs.wavelet.amd;

import com.morphiqlabs.wavelet.api.BoundaryMode;
import com.morphiqlabs.wavelet.api.Wavelet;
import com.morphiqlabs.wavelet.exception.ErrorCode;
import com.morphiqlabs.wavelet.exception.InvalidArgumentException;
import com.morphiqlabs.wavelet.exception.InvalidSignalException;
import com.morphiqlabs.wavelet.modwt.MultiLevelMODWTResult;

/**
 * MI355X drop-in for core/modwt/MultiLevelMODWTTransform.java: {@code decompose}, {@code reconstruct},
 * {@code reconstructFromLevel}, {@code reconstructLevels} with the reference's semantics -- level cap
 * ({@code getMaximumLevels}, :455-501), non-finite input rejected with VAL_NON_FINITE_VALUES, PERIODIC /
 * ZERO_PADDING / SYMMETRIC boundaries (K4 / K5 / K6, :554-645, SymmetricAlignmentStrategy), the FFT
 * switch region reproduced (:710-757) -- plus batch forms over {@code double[][]} that the reference runs
 * one signal at a time.  EXACT accumulation by default: the reference's results bit for bit
 * ({@link AmdRuntime}).
 *
 * <p>Not built or run in this repository (no JDK in its build image): INTEGRATION.md section 2.
 */
public final class AmdMultiLevelMODWT {
    private final Wavelet wavelet;
    private final BoundaryMode boundaryMode;
    private final int boundary;

    /** MultiLevelMODWTTransform(Wavelet, BoundaryMode) (:181-193). */
    public AmdMultiLevelMODWT(Wavelet wavelet, BoundaryMode boundaryMode) {
        if (wavelet == null) throw new NullPointerException("wavelet cannot be null");
        if (boundaryMode == null) throw new NullPointerException("boundaryMode cannot be null");
        this.wavelet = wavelet;
        this.boundaryMode = boundaryMode;
        this.boundary = AmdNative.boundary(boundaryMode);  // CONSTANT -> CFG_UNSUPPORTED_BOUNDARY_MODE
    }

    public Wavelet getWavelet() {
        return wavelet;
    }

    public BoundaryMode getBoundaryMode() {
        return boundaryMode;
    }

    /** getMaximumLevels (:455-501): largest J <= 9 whose upsampled filter fits the signal. */
    public int getMaximumLevels(int signalLength) {
        return AmdNative.maxLevels(signalLength, wavelet.lowPassDecomposition().length);
    }

    /** decompose(signal) (:195-207): as many levels as the signal allows. */
    public MultiLevelMODWTResult decompose(double[] signal) {
        if (signal == null) throw new NullPointerException("signal cannot be null");
        return decompose(signal, getMaximumLevels(signal.length));
    }

    /** decompose(signal, levels) (:209-255). */
    public MultiLevelMODWTResult decompose(double[] signal, int levels) {
        return decomposeBatch(new double[][] {signal}, levels)[0];
    }

    /**
     * One call for a batch of equal-length signals: element b equals {@code decompose(signals[b], levels)}.
     * Validation as decompose, per signal; the error names the first offending signal of the batch (the
     * native side may already have transformed earlier row chunks -- their results are discarded with the
     * exception).  reconstruct* validate nothing, as the reference's (FLAG_REF_NONFINITE: NaN / +-Inf in a
     * result spread as the reference's loops spread them).
     */
    public MultiLevelMODWTResult[] decomposeBatch(double[][] signals, int levels) {
        final int n = equalRows(signals);
        final int batch = signals.length;
        if (levels < 1 || levels > getMaximumLevels(n)) {
            // the reference's order (:209-240): non-finite values, empty signal, then the level range
            for (int b = 0; b < batch; b++) {
                for (int t = 0; t < n; t++) {
                    if (!Double.isFinite(signals[b][t])) {
                        throw new InvalidSignalException(ErrorCode.VAL_NON_FINITE_VALUES,
                                "signal contains non-finite values [signal " + b + ", index " + t + "]");
                    }
                }
            }
            if (n == 0) {
                throw new InvalidSignalException(ErrorCode.VAL_EMPTY, "Signal cannot be empty for multi-level MODWT");
            }
            throw new InvalidArgumentException(ErrorCode.CFG_INVALID_DECOMPOSITION_LEVEL,
                    "Invalid number of decomposition levels: " + levels + " (valid: 1.." + getMaximumLevels(n) + ")");
        }
        double[][][] det = new double[levels][batch][n];
        double[][] app = new double[batch][n];
        final int flags = AmdNative.FLAG_CORE_LEVELS | AmdNative.FLAG_VALIDATE | AmdNative.FLAG_FFT_SWITCH
                | AmdRuntime.FMA;
        AmdNative.check(AmdNative.modwtForwardAoS(AmdRuntime.ctx(), signals, wavelet.lowPassDecomposition(),
                wavelet.highPassDecomposition(), AmdNative.waveletId(wavelet), boundary, levels, flags, det, app));
        MultiLevelMODWTResult[] out = new MultiLevelMODWTResult[batch];
        for (int b = 0; b < batch; b++) {
            double[][] d = new double[levels][];
            for (int l = 0; l < levels; l++) d[l] = det[l][b];
            out[b] = new AmdMultiLevelResult(d, app[b]);
        }
        return out;
    }

    /** reconstruct (:339-349): the cascade J..1. */
    public double[] reconstruct(MultiLevelMODWTResult result) {
        if (result == null) throw new NullPointerException("result cannot be null");
        return inverse(result, ~0, false);
    }

    /** reconstructFromLevel (:361-386): details finer than startLevel are zero. */
    public double[] reconstructFromLevel(MultiLevelMODWTResult result, int startLevel) {
        if (result == null) throw new NullPointerException("result cannot be null");
        final int J = result.getLevels();
        if (startLevel < 1 || startLevel > J) {
            throw new InvalidArgumentException("Invalid start level: " + startLevel + ". Must be between 1 and " + J);
        }
        int mask = 0;
        for (int lev = startLevel; lev <= J; lev++) mask |= 1 << (lev - 1);
        return inverse(result, mask, false);
    }

    /** reconstructLevels (:398-446): only details in [minLevel, maxLevel]; the approximation only if J <= maxLevel. */
    public double[] reconstructLevels(MultiLevelMODWTResult result, int minLevel, int maxLevel) {
        if (result == null) throw new NullPointerException("result cannot be null");
        final int J = result.getLevels();
        if (minLevel < 1 || maxLevel > J || minLevel > maxLevel) {
            throw new InvalidArgumentException(ErrorCode.CFG_INVALID_DECOMPOSITION_LEVEL,
                    "Invalid level range for partial reconstruction");
        }
        int mask = 0;
        for (int lev = minLevel; lev <= maxLevel; lev++) mask |= 1 << (lev - 1);
        return inverse(result, mask, J > maxLevel);
    }

    private double[] inverse(MultiLevelMODWTResult r, int mask, boolean approxZero) {
        final int J = r.getLevels();
        final int n = r.getSignalLength();
        double[] det = new double[Math.multiplyExact(J, n)];
        for (int l = 1; l <= J; l++) {
            System.arraycopy(r.getDetailCoeffsAtLevel(l), 0, det, (l - 1) * n, n);
        }
        double[] y = new double[n];
        AmdNative.check(AmdNative.modwtInverse(AmdRuntime.ctx(), det, r.getApproximationCoeffs(), 1, n,
                wavelet.lowPassReconstruction(), wavelet.highPassReconstruction(), AmdNative.waveletId(wavelet),
                boundary, J, mask, approxZero,
                AmdNative.FLAG_CORE_LEVELS | AmdNative.FLAG_REF_NONFINITE | AmdRuntime.FMA, y));
        return y;
    }

    static int equalRows(double[][] signals) {
        if (signals == null) throw new NullPointerException("signals cannot be null");
        if (signals.length == 0 || signals[0] == null) {
            throw new IllegalArgumentException("signals must be non-null and non-empty");
        }
        final int n = signals[0].length;
        for (int i = 1; i < signals.length; i++) {
            if (signals[i] == null || signals[i].length != n) {
                throw new IllegalArgumentException("all signals must be non-null and same length");
            }
        }
        return n;
    }
}

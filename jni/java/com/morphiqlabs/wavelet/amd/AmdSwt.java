package com.morphiqlabs.wavelet.amd;

import com.morphiqlabs.wavelet.api.BoundaryMode;
import com.morphiqlabs.wavelet.api.Wavelet;
import com.morphiqlabs.wavelet.exception.ErrorCode;
import com.morphiqlabs.wavelet.exception.InvalidArgumentException;
import com.morphiqlabs.wavelet.exception.InvalidSignalException;
import com.morphiqlabs.wavelet.modwt.MutableMultiLevelMODWTResult;
import com.morphiqlabs.wavelet.modwt.MutableMultiLevelMODWTResultImpl;

import java.util.Map;
import java.util.Objects;
import java.util.concurrent.ConcurrentHashMap;

/**
 * MI355X drop-in for core/swt/VectorWaveSwtAdapter.java: the same constructors and public methods, the same
 * two forward branches, computed by the engine's HIP kernels.
 *
 * <ul>
 *   <li>{@code forward(signal, levels)} (:198-204): with parallel processing enabled, N >= parallelThreshold
 *       and levels > 2 the reference runs {@code forwardParallel} (:210-335): no finite check, no level cap,
 *       every upsampled tap multiplied (a NaN / +-Inf sample spreads as NaN through the zero taps) -- here
 *       flags 0 + {@link AmdNative#FLAG_REF_NONFINITE}.  Otherwise {@code decomposeSWT} (:337-394):
 *       non-finite values, then an empty signal, then levels outside 1..getMaximumLevels are rejected in
 *       that order -- here {@link AmdNative#FLAG_CORE_LEVELS} | {@link AmdNative#FLAG_VALIDATE}, with the
 *       non-finite scan done first when the level check would fail.</li>
 *   <li>{@code inverse} (:435-442): PERIODIC is {@code reconstructPeriodic} (:444-474, wraps (t + l) % n, no
 *       length guard), the other modes the core {@code MultiLevelMODWTTransform.reconstruct} (L_j <= N guard,
 *       VAL_TOO_LARGE); neither validates, so both carry FLAG_REF_NONFINITE.</li>
 *   <li>{@code applyUniversalThreshold} (:505-522): sigma = median(|d_1|) / 0.6745 by the engine's exact
 *       selection (Arrays.sort order: NaN above +Inf), T = sigma * sqrt(2 ln N), then the result's own
 *       {@code applyThreshold} on every detail level.</li>
 *   <li>{@code denoise} (:532-574): forward -> threshold -> inverse as ONE engine call (threshold fused into
 *       the inverse's detail loads), with the forward branch's flags.</li>
 * </ul>
 * EXACT accumulation by default: the reference's coefficients, thresholds and outputs bit for bit
 * ({@link AmdRuntime}).
 *
 * <p>Not built or run in this repository (no JDK in its build image): INTEGRATION.md section 2.
 */
public final class AmdSwt implements AutoCloseable {
    /** VectorWaveSwtAdapter.DEFAULT_PARALLEL_THRESHOLD. */
    public static final int DEFAULT_PARALLEL_THRESHOLD = 4096;

    private final Wavelet wavelet;
    private final BoundaryMode boundaryMode;
    private final boolean enableParallel;
    private final int parallelThreshold;
    private final int boundary;
    private final AmdMultiLevelMODWT modwt;

    /** VectorWaveSwtAdapter(Wavelet, BoundaryMode, boolean, int) (:140-148). */
    public AmdSwt(Wavelet wavelet, BoundaryMode boundaryMode, boolean enableParallel, int parallelThreshold) {
        this.wavelet = Objects.requireNonNull(wavelet, "Wavelet cannot be null");
        this.boundaryMode = Objects.requireNonNull(boundaryMode, "Boundary mode cannot be null");
        this.enableParallel = enableParallel;
        this.parallelThreshold = parallelThreshold;
        this.boundary = AmdNative.boundary(boundaryMode);
        this.modwt = new AmdMultiLevelMODWT(wavelet, boundaryMode);
    }

    /** VectorWaveSwtAdapter(Wavelet, BoundaryMode) (:122-124): parallel branch enabled at N >= 4096. */
    public AmdSwt(Wavelet wavelet, BoundaryMode boundaryMode) {
        this(wavelet, boundaryMode, true, DEFAULT_PARALLEL_THRESHOLD);
    }

    /** VectorWaveSwtAdapter(Wavelet) (:173-175): PERIODIC. */
    public AmdSwt(Wavelet wavelet) {
        this(wavelet, BoundaryMode.PERIODIC);
    }

    public Wavelet getWavelet() {
        return wavelet;
    }

    public BoundaryMode getBoundaryMode() {
        return boundaryMode;
    }

    /** The reference's branch test (:200): forwardParallel, which validates nothing. */
    private boolean parallelBranch(int n, int levels) {
        return enableParallel && n >= parallelThreshold && levels > 2;
    }

    /** Engine flags of a forward (and of the denoise pipeline that starts with it) on this branch. */
    private int forwardFlags(int n, int levels) {
        return (parallelBranch(n, levels) ? AmdNative.FLAG_REF_NONFINITE
                : AmdNative.FLAG_CORE_LEVELS | AmdNative.FLAG_VALIDATE) | AmdRuntime.FMA;
    }

    /** decomposeSWT's checks in its order (:339-364) when the level check is the one that fails. */
    private void rejectLevels(double[][] signals, int n, int levels) {
        if (parallelBranch(n, levels)) return;
        final int max = modwt.getMaximumLevels(n);
        if (levels >= 1 && levels <= max) return;
        for (int b = 0; b < signals.length; b++) {
            for (int t = 0; t < n; t++) {
                if (!Double.isFinite(signals[b][t])) {
                    throw new InvalidSignalException(ErrorCode.VAL_NON_FINITE_VALUES,
                            "signal contains non-finite values [signal " + b + ", index " + t + "]");
                }
            }
        }
        if (n == 0) throw new InvalidSignalException(ErrorCode.VAL_EMPTY, "Signal cannot be empty for SWT");
        throw new InvalidArgumentException(ErrorCode.CFG_INVALID_DECOMPOSITION_LEVEL,
                "Invalid SWT decomposition levels: " + levels + " (valid: 1.." + max + ")");
    }

    /** forward(signal) (:184-187): getMaximumLevels(N) levels. */
    public MutableMultiLevelMODWTResult forward(double[] signal) {
        Objects.requireNonNull(signal, "signal cannot be null");
        return forward(signal, modwt.getMaximumLevels(signal.length));
    }

    /** forward(signal, levels) (:198-204), either branch. */
    public MutableMultiLevelMODWTResult forward(double[] signal, int levels) {
        Objects.requireNonNull(signal, "signal cannot be null");
        final int n = signal.length;
        if (n == 0) throw new InvalidSignalException(ErrorCode.VAL_EMPTY, "Signal cannot be empty for SWT");
        rejectLevels(new double[][] {signal}, n, levels);
        if (levels < 1) throw new IllegalArgumentException("Number of levels must be positive");
        double[] det = new double[Math.multiplyExact(levels, n)];
        double[] app = new double[n];
        AmdNative.check(AmdNative.modwtForward(AmdRuntime.ctx(), signal, 1, n, wavelet.lowPassDecomposition(),
                wavelet.highPassDecomposition(), AmdNative.waveletId(wavelet), boundary, levels,
                forwardFlags(n, levels), det, app));
        MutableMultiLevelMODWTResultImpl r = new MutableMultiLevelMODWTResultImpl(n, levels);
        for (int l = 1; l <= levels; l++) {
            double[] d = new double[n];
            System.arraycopy(det, (l - 1) * n, d, 0, n);
            r.setDetailCoeffs(l, d);
        }
        r.setApproximationCoeffs(app);
        return r;
    }

    /** inverse(result) (:435-442). */
    public double[] inverse(MutableMultiLevelMODWTResult result) {
        Objects.requireNonNull(result, "Result cannot be null");
        return reconstruct(result, ~0, false);
    }

    private double[] reconstruct(MutableMultiLevelMODWTResult r, int mask, boolean approxZero) {
        final int J = r.getLevels();
        final int n = r.getSignalLength();
        double[] det = new double[Math.multiplyExact(J, n)];
        for (int l = 1; l <= J; l++) System.arraycopy(r.getMutableDetailCoeffs(l), 0, det, (l - 1) * n, n);
        double[] y = new double[n];
        final int guard = boundaryMode == BoundaryMode.PERIODIC ? 0 : AmdNative.FLAG_CORE_LEVELS;
        AmdNative.check(AmdNative.modwtInverse(AmdRuntime.ctx(), det, r.getMutableApproximationCoeffs(), 1, n,
                wavelet.lowPassReconstruction(), wavelet.highPassReconstruction(), AmdNative.waveletId(wavelet),
                boundary, J, mask, approxZero, guard | AmdNative.FLAG_REF_NONFINITE | AmdRuntime.FMA, y));
        return y;
    }

    /** applyThreshold(result, level, threshold, soft) (:489-493): the result's own thresholding. */
    public void applyThreshold(MutableMultiLevelMODWTResult result, int level, double threshold, boolean soft) {
        Objects.requireNonNull(result, "Result cannot be null");
        result.applyThreshold(level, threshold, soft);
    }

    /** applyUniversalThreshold(result, soft) (:505-522); sigma from d_1 on the device. */
    public void applyUniversalThreshold(MutableMultiLevelMODWTResult result, boolean soft) {
        Objects.requireNonNull(result, "Result cannot be null");
        final double[] finest = result.getMutableDetailCoeffs(1);
        final double[] sigma = new double[1];
        AmdNative.check(AmdNative.noiseSigma(AmdRuntime.ctx(), finest, 1, finest.length, sigma));
        final int n = result.getSignalLength();
        final double threshold = sigma[0] * Math.sqrt(2 * Math.log(n));
        for (int level = 1; level <= result.getLevels(); level++) {
            applyThreshold(result, level, threshold, soft);
        }
    }

    /** denoise(signal, levels) (:532-534): universal soft threshold. */
    public double[] denoise(double[] signal, int levels) {
        return denoise(signal, levels, -1, true);
    }

    /** denoise(signal, levels, threshold, soft) (:546-574): threshold < 0 selects the universal threshold. */
    public double[] denoise(double[] signal, int levels, double threshold, boolean soft) {
        Objects.requireNonNull(signal, "signal cannot be null");
        return denoiseBatch(new double[][] {signal}, levels, threshold, soft)[0];
    }

    /** Every row as {@link #denoise(double[], int, double, boolean)}, one engine call for the batch. */
    public double[][] denoiseBatch(double[][] signals, int levels, double threshold, boolean soft) {
        final int n = AmdMultiLevelMODWT.equalRows(signals);
        if (n == 0) throw new InvalidSignalException(ErrorCode.VAL_EMPTY, "Signal cannot be empty for SWT");
        rejectLevels(signals, n, levels);
        double[][] y = new double[signals.length][n];
        AmdNative.check(AmdNative.swtDenoiseAoS(AmdRuntime.ctx(), signals, wavelet.lowPassDecomposition(),
                wavelet.highPassDecomposition(), AmdNative.waveletId(wavelet), boundary, levels, threshold, soft,
                forwardFlags(n, levels), y));
        return y;
    }

    /**
     * extractLevel(signal, levels, targetLevel) (:576-598): every detail level but the target and (for a target
     * other than 0) the approximation reconstructed as zeros.
     */
    public double[] extractLevel(double[] signal, int levels, int targetLevel) {
        MutableMultiLevelMODWTResult r = forward(signal, levels);
        final int mask = targetLevel >= 1 && targetLevel <= levels ? 1 << (targetLevel - 1) : 0;
        return reconstruct(r, mask, targetLevel != 0);
    }

    /** cleanup() (:652-661): the engine context is the JVM's ({@link AmdRuntime}); nothing to release. */
    public void cleanup() {}

    @Override
    public void close() {
        cleanup();
    }

    /** getCacheStatistics() (:677-685): the reference's keys; the taps are upsampled on the device. */
    public Map<String, Object> getCacheStatistics() {
        Map<String, Object> stats = new ConcurrentHashMap<>();
        stats.put("filterCacheSize", 0);
        stats.put("parallelExecutorActive", false);
        stats.put("parallelThreshold", parallelThreshold);
        return stats;
    }
}

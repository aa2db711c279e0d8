package com.morphiqlabs.wavelet.amd;

import com.morphiqlabs.wavelet.api.BoundaryMode;
import com.morphiqlabs.wavelet.api.Daubechies;
import com.morphiqlabs.wavelet.api.Wavelet;
import com.morphiqlabs.wavelet.denoising.WaveletDenoiser.ThresholdMethod;
import com.morphiqlabs.wavelet.denoising.WaveletDenoiser.ThresholdType;
import com.morphiqlabs.wavelet.exception.ErrorCode;
import com.morphiqlabs.wavelet.exception.InvalidArgumentException;

import java.util.Objects;

/**
 * MI355X drop-in for core/denoising/WaveletDenoiser.java (:44-660), over the {@code waveletDenoise} native
 * (include/vectorwave_amd.h vw_wavelet_denoise_f64): one engine call per signal or batch runs the forward
 * transform, the noise estimate sigma = median(|d_1|) / 0.6745 (exact selection), the threshold of every
 * (level, signal) -- UNIVERSAL, SURE (the reference's O(n^2) risk search reproduced bit for bit in
 * O(n log^2 n), N <= 16384), MINIMAX, BAYES -- and the inverse with the soft / hard threshold fused into its
 * detail loads.  Same constructors, methods and enums (the reference's own {@link ThresholdMethod},
 * {@link ThresholdType}); same exceptions: a non-finite or empty signal as MODWTTransform / MultiLevelMODWTTransform
 * reject it, FIXED through {@code denoise} / {@code denoiseMultiLevel} as CFG_UNSUPPORTED_OPERATION.
 *
 * <ul>
 *   <li>{@code denoise(signal, method[, type])} (:111-143): single-level MODWTTransform, threshold from d_1.</li>
 *   <li>{@code denoiseMultiLevel(signal, levels, method, type)} (:155-231): MultiLevelMODWTTransform
 *       (level cap, FFT-switch dispatch), level j thresholded with sigma / sqrt(2^j) on its own
 *       coefficients (DenoisedMultiLevelResult).</li>
 *   <li>{@code denoiseFixed(signal, threshold, type)} (:354-364).</li>
 * </ul>
 * EXACT accumulation by default: the reference's thresholds and outputs bit for bit ({@link AmdRuntime}).
 *
 * <p>Not built or run in this repository (no JDK in its build image): INTEGRATION.md section 2.
 */
public class AmdWaveletDenoiser {
    private static final int MAX_SAFE_LEVEL_FOR_SCALING = 31;  // :57

    private final Wavelet wavelet;
    private final BoundaryMode boundaryMode;
    private final int boundary;

    /** WaveletDenoiser(Wavelet, BoundaryMode) (:80-90). */
    public AmdWaveletDenoiser(Wavelet wavelet, BoundaryMode boundaryMode) {
        if (wavelet == null) {
            throw new InvalidArgumentException(ErrorCode.VAL_NULL_ARGUMENT, "Wavelet cannot be null");
        }
        if (boundaryMode == null) {
            throw new InvalidArgumentException(ErrorCode.VAL_NULL_ARGUMENT, "Boundary mode cannot be null");
        }
        this.wavelet = wavelet;
        this.boundaryMode = boundaryMode;
        this.boundary = AmdNative.boundary(boundaryMode);
    }

    /** forFinancialData() (:99-101): DB4, PERIODIC. */
    public static AmdWaveletDenoiser forFinancialData() {
        return new AmdWaveletDenoiser(Daubechies.DB4, BoundaryMode.PERIODIC);
    }

    /** denoise(signal, method) (:111-113): soft thresholding. */
    public double[] denoise(double[] signal, ThresholdMethod method) {
        return denoise(signal, method, ThresholdType.SOFT);
    }

    /** denoise(signal, method, type) (:124-143). */
    public double[] denoise(double[] signal, ThresholdMethod method, ThresholdType type) {
        return denoiseBatch(new double[][] {signal}, 0, method, type)[0];
    }

    /** denoiseMultiLevel(signal, levels, method, type) (:155-170). */
    public double[] denoiseMultiLevel(double[] signal, int levels, ThresholdMethod method, ThresholdType type) {
        if (levels > MAX_SAFE_LEVEL_FOR_SCALING) {
            throw new InvalidArgumentException(ErrorCode.VAL_TOO_LARGE,
                    "Decomposition level exceeds safe limit for scale-dependent thresholds");
        }
        return denoiseBatch(new double[][] {signal}, Math.max(levels, 0), method, type)[0];
    }

    /** denoiseFixed(signal, threshold, type) (:354-364). */
    public double[] denoiseFixed(double[] signal, double threshold, ThresholdType type) {
        Objects.requireNonNull(type, "type cannot be null");
        Objects.requireNonNull(signal, "signal cannot be null");
        double[] y = new double[signal.length];
        AmdNative.check(AmdNative.waveletDenoise(AmdRuntime.ctx(), signal, 1, signal.length,
                wavelet.lowPassDecomposition(), wavelet.highPassDecomposition(), AmdNative.waveletId(wavelet),
                boundary, 0, ThresholdMethod.FIXED.ordinal(), threshold, type == ThresholdType.SOFT,
                AmdNative.FLAG_VALIDATE | AmdRuntime.FMA, y, null));
        return y;
    }

    /**
     * Every row as {@code denoise} (levels == 0) or {@code denoiseMultiLevel} (levels >= 1), one engine call for
     * the batch; thresholds are per (level, signal) exactly as the per-signal calls compute them.
     */
    public double[][] denoiseBatch(double[][] signals, int levels, ThresholdMethod method, ThresholdType type) {
        Objects.requireNonNull(method, "method cannot be null");
        Objects.requireNonNull(type, "type cannot be null");
        final int n = AmdMultiLevelMODWT.equalRows(signals);
        final int batch = signals.length;
        // MODWTTransform / MultiLevelMODWTTransform validate the signal first, calculateThreshold then refuses
        // FIXED (:415-424): the validation runs in the engine (a forward over the batch) before that error
        final int flags = AmdNative.FLAG_VALIDATE | AmdRuntime.FMA
                | (levels > 0 ? AmdNative.FLAG_CORE_LEVELS | AmdNative.FLAG_FFT_SWITCH : 0);
        if (method == ThresholdMethod.FIXED) {
            final int J = Math.max(levels, 1);
            AmdNative.check(AmdNative.modwtForwardAoS(AmdRuntime.ctx(), signals, wavelet.lowPassDecomposition(),
                    wavelet.highPassDecomposition(), AmdNative.waveletId(wavelet), boundary, J, flags,
                    new double[J][batch][n], new double[batch][n]));
            throw new InvalidArgumentException(ErrorCode.CFG_UNSUPPORTED_OPERATION,
                    "Fixed threshold method requires explicit threshold value");
        }
        double[] flat = AmdBatchMODWT.flatten(signals, 0, batch, n);
        double[] y = new double[flat.length];
        AmdNative.check(AmdNative.waveletDenoise(AmdRuntime.ctx(), flat, batch, n, wavelet.lowPassDecomposition(),
                wavelet.highPassDecomposition(), AmdNative.waveletId(wavelet), boundary, levels, method.ordinal(), 0.0,
                type == ThresholdType.SOFT, flags, y, null));
        double[][] out = new double[batch][n];
        AmdBatchMODWT.unflatten(y, out, 0, batch, n);
        return out;
    }
}

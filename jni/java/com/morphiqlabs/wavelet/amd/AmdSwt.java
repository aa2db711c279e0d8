package com.morphiqlabs.wavelet.amd;

import com.morphiqlabs.wavelet.api.BoundaryMode;
import com.morphiqlabs.wavelet.api.Wavelet;

/**
 * MI355X drop-in for core/swt/VectorWaveSwtAdapter.java's denoising entry points (:532-574):
 * {@code denoise(signal, levels)} = forward -> universal soft threshold sigma * sqrt(2 ln N),
 * sigma = median(|d_1|) / 0.6745 (MutableMultiLevelMODWTResult.java:83-114) -> inverse; and
 * {@code denoise(signal, levels, threshold, soft)} with a fixed threshold on every detail level.  The whole
 * pipeline is one engine call (forward, exact median, threshold fused into the inverse's detail loads);
 * the batch form runs every signal in that one call.  EXACT accumulation by default: the reference's
 * output and threshold bit for bit ({@link AmdRuntime}).
 *
 * <p>Not built or run in this repository (no JDK in its build image): INTEGRATION.md section 2.
 */
public final class AmdSwt {
    private final Wavelet wavelet;
    private final BoundaryMode boundaryMode;
    private final int boundary;

    /** VectorWaveSwtAdapter(Wavelet, BoundaryMode) (:122-138). */
    public AmdSwt(Wavelet wavelet, BoundaryMode boundaryMode) {
        if (wavelet == null) throw new NullPointerException("wavelet cannot be null");
        if (boundaryMode == null) throw new NullPointerException("boundaryMode cannot be null");
        this.wavelet = wavelet;
        this.boundaryMode = boundaryMode;
        this.boundary = AmdNative.boundary(boundaryMode);
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

    /** denoise(signal, levels) (:532-534): universal soft threshold. */
    public double[] denoise(double[] signal, int levels) {
        return denoise(signal, levels, -1, true);
    }

    /** denoise(signal, levels, threshold, soft) (:546-574): threshold < 0 selects the universal threshold. */
    public double[] denoise(double[] signal, int levels, double threshold, boolean soft) {
        if (signal == null) throw new NullPointerException("signal cannot be null");
        return denoiseBatch(new double[][] {signal}, levels, threshold, soft)[0];
    }

    /** Every row as {@link #denoise(double[], int, double, boolean)}, one engine call for the batch. */
    public double[][] denoiseBatch(double[][] signals, int levels, double threshold, boolean soft) {
        final int n = AmdMultiLevelMODWT.equalRows(signals);
        double[][] y = new double[signals.length][n];
        AmdNative.check(AmdNative.swtDenoiseAoS(AmdRuntime.ctx(), signals, wavelet.lowPassDecomposition(),
                wavelet.highPassDecomposition(), AmdNative.waveletId(wavelet), boundary, levels, threshold, soft,
                AmdNative.FLAG_VALIDATE | AmdRuntime.FMA, y));
        return y;
    }
}

"""GPU parity of WaveletDenoiser (core/denoising/WaveletDenoiser.java) through the C ABI.

Thresholds are compared bit for bit with the CPU restatement (oracle/vw_oracle.c vwo_wavelet_denoise, which
runs the reference's O(n^2) SURE search); denoised signals bit for bit in EXACT mode, except levels that
the reference computes by FFT (FftHeuristics region: 1e-12, as test_fft_switch_region).
"""
import numpy as np
import pytest

from oracle import oracle as O
import vectorwave_amd as vw
from vectorwave_amd.denoise import ThresholdMethod as M, ThresholdType as TT
from vectorwave_amd.errors import InvalidStateException
from vectorwave_amd.wavelets import Coiflet, Daubechies, Haar, Symlet

pytestmark = pytest.mark.gpu

METHODS = [M.UNIVERSAL, M.SURE, M.MINIMAX, M.BAYES]


def noisy(B, n, seed, quant=None):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / n
    x = np.sin(2 * np.pi * 3 * t)[None, :] + 0.4 * rng.standard_normal((B, n))
    if quant:
        x = np.round(x * quant) / quant  # exact ties among the coefficients
    return x


def lohi(w):
    return w.lowPassDecomposition(), w.highPassDecomposition()


def fft_region(w, n, J):
    if n < 1024:
        return False
    return any(n / 8 < O.upsample_scale(w.lowPassDecomposition(), j).size <= n // 2 for j in range(1, J + 1))


@pytest.mark.parametrize("method", METHODS, ids=lambda m: m.name)
@pytest.mark.parametrize("boundary", [O.PERIODIC, O.SYMMETRIC, O.ZERO_PADDING], ids=["P", "S", "Z"])
@pytest.mark.parametrize("w,n,levels", [(Haar.INSTANCE, 64, 0), (Daubechies.DB4, 129, 0), (Daubechies.DB4, 1000, 4),
                                         (Symlet.SYM8, 512, 3), (Coiflet.COIF3, 4096, 5), (Haar.INSTANCE, 33, 2)],
                         ids=lambda v: getattr(v, "name", lambda: str(v))() if hasattr(v, "name") else str(v))
def test_denoise_matches_restatement(engine, method, boundary, w, n, levels):
    x = noisy(3, n, n + levels)
    den = vw.WaveletDenoiser(w, vw.BoundaryMode(boundary))
    for soft in (TT.SOFT, TT.HARD):
        if levels == 0:
            y, thr = den.denoise(x, method, soft, return_thresholds=True)
        else:
            y, thr = den.denoiseMultiLevel(x, levels, method, soft, return_thresholds=True)
        approx = boundary == O.PERIODIC and levels > 0 and fft_region(w, n, levels)
        for b in range(3):
            y_ref, t_ref = O.wavelet_denoise(x[b], *lohi(w), boundary, levels, int(method), soft=soft == TT.SOFT,
                                             wavelet_id=w.wavelet_id)
            if approx:
                np.testing.assert_allclose(thr[:, b], t_ref, rtol=1e-12, atol=0)
                np.testing.assert_allclose(y[b], y_ref, rtol=0, atol=1e-12)
            else:
                assert np.array_equal(thr[:, b], t_ref), (thr[:, b], t_ref)
                assert np.array_equal(y[b], y_ref), np.max(np.abs(y[b] - y_ref))


@pytest.mark.parametrize("quant", [None, 8, 1])
def test_sure_ties_and_near_ties(engine, quant):
    """Quantised signals give exact ties among |d| (runs in the sorted keys) and flat risk curves
    (several candidates re-evaluated exactly); quant=1 leaves few distinct values."""
    w = Daubechies.DB4
    x = noisy(6, 2048, 11, quant)
    x[4] = 0.0          # all-zero row: sigma 0, every risk 0
    x[5] = 5.0          # constant row
    den = vw.WaveletDenoiser(w, vw.BoundaryMode.PERIODIC)
    for levels in (0, 4):
        if levels:
            y, thr = den.denoiseMultiLevel(x, levels, M.SURE, TT.SOFT, return_thresholds=True)
        else:
            y, thr = den.denoise(x, M.SURE, TT.SOFT, return_thresholds=True)
        for b in range(6):
            y_ref, t_ref = O.wavelet_denoise(x[b], *lohi(w), O.PERIODIC, levels, O.SURE, wavelet_id=w.wavelet_id)
            assert np.array_equal(thr[:, b], t_ref), (b, levels, thr[:, b], t_ref)
            assert np.array_equal(y[b], y_ref)


def test_sure_max_length(engine):
    w = Haar.INSTANCE
    x = noisy(2, 16384, 5)
    y, thr = vw.WaveletDenoiser(w, vw.BoundaryMode.PERIODIC).denoise(x, M.SURE, return_thresholds=True)
    for b in range(2):
        y_ref, t_ref = O.wavelet_denoise(x[b], *lohi(w), O.PERIODIC, 0, O.SURE)
        assert thr[0, b] == t_ref[0]
        assert np.array_equal(y[b], y_ref)
    with pytest.raises(NotImplementedError):
        vw.WaveletDenoiser(w, vw.BoundaryMode.PERIODIC).denoise(noisy(1, 16385, 1), M.SURE)


def test_denoise_fixed_and_device_batch(engine):
    import torch
    w = Symlet.SYM4
    x = noisy(64, 1024, 2)
    den = vw.WaveletDenoiser(w, vw.BoundaryMode.SYMMETRIC)
    for T in (0.0, 0.3, -0.2):  # a negative fixed threshold shrinks nothing and grows |c| (scalar path :570-581)
        for t in (TT.SOFT, TT.HARD):
            y = den.denoiseFixed(x, T, t)
            for b in (0, 63):
                assert np.array_equal(y[b], O.wavelet_denoise(x[b], *lohi(w), O.SYMMETRIC, 0, O.FIXED, T,
                                                               soft=t == TT.SOFT)[0])
    xd = torch.tensor(x, device="cuda")
    yd = den.denoiseMultiLevel(xd, 4, M.BAYES, TT.SOFT)
    assert yd.is_cuda
    yh = den.denoiseMultiLevel(x, 4, M.BAYES, TT.SOFT)
    assert np.array_equal(yd.cpu().numpy(), yh)


def test_denoiser_errors(engine):
    den = vw.WaveletDenoiser(Daubechies.DB4, vw.BoundaryMode.PERIODIC)
    x = noisy(1, 256, 1)[0]
    with pytest.raises(TypeError):
        den.denoise(None, M.UNIVERSAL)
    with pytest.raises(vw.InvalidSignalException):
        den.denoise(np.zeros(0), M.UNIVERSAL)
    bad = x.copy()
    bad[17] = np.nan
    with pytest.raises(vw.InvalidSignalException):
        den.denoise(bad, M.UNIVERSAL)
    with pytest.raises(vw.InvalidSignalException):
        den.denoiseMultiLevel(np.array([1.0, 2.0, np.inf, 4.0] * 16), 2, M.SURE, TT.SOFT)
    for lv in (0, -1):
        with pytest.raises(vw.InvalidArgumentException):
            den.denoiseMultiLevel(x, lv, M.UNIVERSAL, TT.SOFT)
    with pytest.raises(vw.InvalidArgumentException):
        den.denoiseMultiLevel(np.zeros(8), 10, M.UNIVERSAL, TT.SOFT)   # WaveletDenoiserTest.java:168-169
    with pytest.raises(vw.InvalidArgumentException):
        den.denoise(x, M.FIXED)
    with pytest.raises(vw.InvalidArgumentException):
        den.denoiseMultiLevel(x, 2, M.FIXED, TT.SOFT)
    # WaveletDenoiserTest.testEdgeCases :203-223
    assert den.denoise(np.array([1.0, 2.0]), M.UNIVERSAL).shape == (2,)
    assert np.all(np.isfinite(den.denoise(np.full(64, 5.0), M.UNIVERSAL)))
    assert np.array_equal(den.denoise(np.zeros(32), M.UNIVERSAL), np.zeros(32))


def test_bayes_reduces_noise_variance(engine):
    # WaveletDenoiserBayesTest.testBayesThresholdingWithNoisySignal :36-56
    rng = np.random.default_rng(7)
    n = 256
    clean = np.sin(2 * np.pi * np.arange(n) / 32)
    x = clean + 0.5 * rng.standard_normal(n)
    y = vw.WaveletDenoiser(Haar.INSTANCE, vw.BoundaryMode.PERIODIC).denoise(x, M.BAYES)
    assert np.var(y - clean) <= np.var(x - clean) * 1.1


# ---- MODWTStreamingDenoiser (core/modwt/streaming/MODWTStreamingDenoiser.java) ------------------------
@pytest.mark.parametrize("est", ["MAD", "STD", "FIXED"])
@pytest.mark.parametrize("mult", [1.0, 1.5])
@pytest.mark.parametrize("method", ["UNIVERSAL", "MINIMAX", "SURE"])
@pytest.mark.parametrize("blk,win", [(256, 1024), (512, 100)], ids=["window-fills", "stratified"])
def test_streaming_denoiser_bit_exact(engine, est, mult, method, blk, win):
    from vectorwave_amd import MODWTStreamingDenoiser as SD
    from vectorwave_amd.denoise import ThresholdMethod, ThresholdType
    w = vw.get_wavelet("db4")
    m = ThresholdMethod[method]
    sd = (SD.builder().wavelet(w).boundaryMode(vw.BoundaryMode.PERIODIC).bufferSize(blk)
          .thresholdType(ThresholdType.SOFT).thresholdMethod(m).thresholdMultiplier(mult)
          .noiseEstimation(SD.NoiseEstimation[est]).noiseWindowSize(win).build())
    ref = O.StreamingDenoiserRestatement(w.lowPassDecomposition(), w.highPassDecomposition(), O.PERIODIC,
                                         w.wavelet_id, int(m), True, mult, est, win)
    got_blocks = []
    sd.subscribe(got_blocks.append)
    x = O.java_random_signal(blk * 4, 77) + np.sin(np.arange(blk * 4) * 0.05)
    for k in range(4):
        blockx = x[k * blk:(k + 1) * blk]
        y = sd.denoise(blockx)
        y_ref = ref.denoise(blockx)
        np.testing.assert_array_equal(y, y_ref)
        assert sd.getEstimatedNoiseLevel() == ref.level
    assert sd.getSamplesProcessed() == 4 * blk and len(got_blocks) == 4
    sd.close()
    assert sd.isClosed()
    with pytest.raises(InvalidStateException):
        sd.denoise(x[:blk])


@pytest.mark.parametrize("est", ["MAD", "FIXED"])
def test_streaming_denoiser_long_window_and_block(engine, est):
    """MAD over a noise window / block longer than 16384 samples (the centered median's
    register-keyed limit) -- the deviations go through the workspace, the result stays bit-exact."""
    from vectorwave_amd import MODWTStreamingDenoiser as SD
    from vectorwave_amd.denoise import ThresholdMethod, ThresholdType
    w = vw.get_wavelet("db4")
    blk, win = 20480, 20000
    sd = (SD.builder().wavelet(w).boundaryMode(vw.BoundaryMode.PERIODIC).bufferSize(blk)
          .thresholdType(ThresholdType.SOFT).thresholdMethod(ThresholdMethod.UNIVERSAL).thresholdMultiplier(1.5)
          .noiseEstimation(SD.NoiseEstimation[est]).noiseWindowSize(win).build())
    ref = O.StreamingDenoiserRestatement(w.lowPassDecomposition(), w.highPassDecomposition(), O.PERIODIC,
                                         w.wavelet_id, int(ThresholdMethod.UNIVERSAL), True, 1.5, est, win)
    x = O.java_random_signal(blk * 2, 91) + np.sin(np.arange(blk * 2) * 0.01)
    for k in range(2):
        blockx = x[k * blk:(k + 1) * blk]
        np.testing.assert_array_equal(sd.denoise(blockx), ref.denoise(blockx))
        assert sd.getEstimatedNoiseLevel() == ref.level
    sd.close()


def test_median_centered_long_rows(engine):
    import torch
    from ctypes import c_void_p
    B, n = 3, 40001
    v = torch.tensor(np.stack([O.java_random_signal(n, 5 + b) for b in range(B)]), device="cuda")
    c = torch.tensor([0.1, -0.25, 0.0], dtype=torch.float64, device="cuda")
    out = torch.empty(B, dtype=torch.float64, device="cuda")
    engine.bind_torch_stream()
    P = lambda t: c_void_p(t.data_ptr())  # noqa: E731
    assert engine.lib.vw_median_f64(engine.ctx, P(v), B, n, P(c), 0, P(out)) == 0
    torch.cuda.synchronize()
    vh, ch = v.cpu().numpy(), c.cpu().numpy()
    for b in range(B):
        assert out[b].item() == O.java_median(np.abs(vh[b] - ch[b]))


def test_streaming_denoiser_builder_validation(engine):
    from vectorwave_amd import MODWTStreamingDenoiser as SD
    for bad in (lambda b: b.bufferSize(0), lambda b: b.noiseWindowSize(-1), lambda b: b.thresholdMultiplier(0),
                lambda b: b.wavelet(None)):
        with pytest.raises(vw.InvalidArgumentException):
            bad(SD.builder())
    with pytest.raises(vw.InvalidArgumentException):
        SD.builder().build().denoise(np.zeros(0))

"""GPU parity: the HIP path (through the C ABI) against the CPU restatement of vectorwave-core.

Bar: bit-exact in the default EXACT mode (separate multiply/add in the reference's order) for every
index/bookkeeping path; FFT-region levels (the reference uses an FFT there) and the FMA variant
within 1e-12 * max|x|; fp32 within 1e-5 * max|x| * J (no fp32 path exists in the reference).
"""
import math
import os

import numpy as np
import pytest

from oracle import oracle as O
import vectorwave_amd as vw
from vectorwave_amd import _native as nat
from vectorwave_amd.wavelets import Coiflet, Daubechies, Haar, Symlet

pytestmark = pytest.mark.gpu

H = Haar.INSTANCE
WAVELETS = [H, Daubechies.DB2, Symlet.SYM3, Daubechies.DB4, Coiflet.COIF2, Daubechies.DB8, Symlet.SYM8,
            Coiflet.COIF3, Coiflet.COIF5, Daubechies.DB6, Symlet.SYM4]
BOUNDARIES = [O.PERIODIC, O.SYMMETRIC, O.ZERO_PADDING]


def signals(B, n, seed):
    return np.stack([O.java_random_signal(n, seed + b) for b in range(B)])


def lohi(w):
    return w.lowPassDecomposition(), w.highPassDecomposition()


def exact(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape
    if not np.array_equal(a, b):
        i = np.unravel_index(np.argmax(np.abs(a - b)), a.shape)
        raise AssertionError(f"not bit-exact: max |diff| = {np.max(np.abs(a - b)):.3e} at {i}")


# ---- multi-level forward / inverse ----------------------------------------------------------------
@pytest.mark.parametrize("w", WAVELETS, ids=lambda w: w.name())
@pytest.mark.parametrize("boundary", BOUNDARIES, ids=["P", "S", "Z"])
@pytest.mark.parametrize("n", [64, 129, 512, 4096])
def test_multilevel_forward_inverse_bit_exact(engine, w, boundary, n):
    L = w.filter_length
    J = min(6, O.max_levels(n, L))
    if J < 1:
        pytest.skip("no level fits")
    if boundary == O.PERIODIC and n >= 1024 and any(
            O.upsample_scale(w.lowPassDecomposition(), j).size > n / 8 and not (O.upsample_scale(w.lowPassDecomposition(), j).size > n // 2)
            for j in range(1, J + 1)):
        pytest.skip("FFT region: covered by test_fft_switch_region")
    x = signals(3, n, 7)
    tx = vw.MultiLevelMODWTTransform(w, vw.BoundaryMode(boundary))
    res = tx.decompose(x, J)
    det, app = res.details_array, res.approximation_array
    for b in range(3):
        d_ref, a_ref = O.decompose(x[b], *lohi(w), boundary, J)
        exact(det[:, b, :], d_ref)
        exact(app[b], a_ref)
        y_ref = O.reconstruct(d_ref, a_ref, w.lowPassReconstruction(), w.highPassReconstruction(), boundary,
                              w.wavelet_id)
        exact(tx.reconstruct(vw.MultiLevelMODWTResult(d_ref[:, None, :].copy(), a_ref[None, :].copy()))[0], y_ref)
    y = tx.reconstruct(res)
    for b in range(3):
        d_ref, a_ref = O.decompose(x[b], *lohi(w), boundary, J)
        exact(y[b], O.reconstruct(d_ref, a_ref, w.lowPassReconstruction(), w.highPassReconstruction(), boundary,
                                  w.wavelet_id))


@pytest.mark.parametrize("n,w,J", [(1500, Daubechies.DB4, 6), (2048, Daubechies.DB4, 8), (3000, Symlet.SYM8, 7)])
def test_fft_switch_region(engine, n, w, J):
    # MultiLevelMODWTTransform PERIODIC levels with N/8 < L_j <= N/2 use the FFT branch (zero-padded to
    # nextPow2(N)); the engine computes that convolution directly.  Tolerance: FFT rounding.
    x = signals(2, n, 3)
    res = vw.MultiLevelMODWTTransform(w, vw.BoundaryMode.PERIODIC).decompose(x, J)
    for b in range(2):
        d_ref, a_ref = O.decompose(x[b], *lohi(w), O.PERIODIC, J)
        np.testing.assert_allclose(res.details_array[:, b, :], d_ref, rtol=0, atol=1e-12)
        np.testing.assert_allclose(res.approximation_array[b], a_ref, rtol=0, atol=1e-12)


def test_reconstruct_partial(engine):
    w = Daubechies.DB4
    x = signals(2, 512, 5)
    tx = vw.MultiLevelMODWTTransform(w, vw.BoundaryMode.PERIODIC)
    res = tx.decompose(x, 5)
    lo, hi = w.lowPassReconstruction(), w.highPassReconstruction()
    for b in range(2):
        d, a = O.decompose(x[b], *lohi(w), O.PERIODIC, 5)
        # reconstructFromLevel(3): details of levels 1-2 zeroed
        exact(tx.reconstructFromLevel(res, 3)[b], O.reconstruct(d, a, lo, hi, O.PERIODIC, detail_mask=0b11100))
        # reconstructLevels(2, 3): approx zeroed (J=5 > 3), details 2..3 only
        exact(tx.reconstructLevels(res, 2, 3)[b],
              O.reconstruct(d, a, lo, hi, O.PERIODIC, detail_mask=0b00110, approx_zero=True))
        exact(tx.reconstructLevels(res, 4, 5)[b], O.reconstruct(d, a, lo, hi, O.PERIODIC, detail_mask=0b11000))


def test_level_cap_and_errors(engine):
    tx = vw.MultiLevelMODWTTransform(Daubechies.DB4, vw.BoundaryMode.PERIODIC)
    x = np.zeros(4096)
    with pytest.raises(vw.InvalidArgumentException):
        tx.decompose(x, 10)  # cap 9 (calculateMaxLevels loop bound)
    with pytest.raises(vw.InvalidArgumentException):
        tx.decompose(np.zeros(100), 5)
    bad = np.ones(256)
    bad[77] = np.nan
    with pytest.raises(vw.InvalidSignalException) as ei:
        tx.decompose(bad, 3)
    assert ei.value.index == 77
    with pytest.raises(vw.InvalidSignalException):
        tx.decompose(np.zeros(0), 1)


# ---- single level (MODWTTransform) --------------------------------------------------------------------
@pytest.mark.parametrize("w", [H, Daubechies.DB4, Daubechies.DB8, Coiflet.COIF5], ids=lambda w: w.name())
@pytest.mark.parametrize("boundary", BOUNDARIES, ids=["P", "S", "Z"])
@pytest.mark.parametrize("n", [1, 4, 7, 9, 64, 1000])
def test_single_level_bit_exact(engine, w, boundary, n):
    x = signals(4, n, 11)
    tx = vw.MODWTTransform(w, vw.BoundaryMode(boundary))
    r = tx.forwardBatch(x)
    for b in range(4):
        a_ref, d_ref = O.modwt_forward(x[b], *lohi(w), boundary)
        exact(r[b].approximationCoeffs(), a_ref)
        exact(r[b].detailCoeffs(), d_ref)
        exact(tx.inverse(r[b]), O.modwt_inverse(a_ref, d_ref, w.lowPassReconstruction(), w.highPassReconstruction(),
                                               boundary))
    ys = tx.inverseBatch(r)
    opt = len(r) >= 4 and n >= 64
    for b in range(4):
        a_ref, d_ref = O.modwt_forward(x[b], *lohi(w), boundary)
        exact(ys[b], O.modwt_inverse(a_ref, d_ref, w.lowPassReconstruction(), w.highPassReconstruction(), boundary,
                                     batch_optimized=opt))


def test_known_answers_on_device(engine):
    # MODWTPercivalWaldenValidationTest.java:73 and TimeReversedFilterTest.java:42-49
    tx = vw.MODWTTransform(H, vw.BoundaryMode.PERIODIC)
    r = tx.forward(np.array([1.0, 2.0, 3.0, 4.0]))
    np.testing.assert_allclose(r.approximationCoeffs(), [2.5, 1.5, 2.5, 3.5], atol=1e-10)
    np.testing.assert_allclose(tx.inverse(r), [1.0, 2.0, 3.0, 4.0], atol=1e-10)


# ---- batch facade ----------------------------------------------------------------------------------
def test_batch_facade(engine):
    x = signals(5, 256, 31)
    a = vw.BatchMODWT.singleLevelAoS(H, x)
    for b in range(5):
        ra, rd = O.batch_single(x[b], *lohi(H), True)
        exact(a.approx[b], ra)
        exact(a.detail[b], rd)
    w = Daubechies.DB4
    m = vw.BatchMODWT.multiLevelAoS(w, x, 4)
    for b in range(5):
        d, ap = O.decompose(x[b], *lohi(w), O.PERIODIC, 4, core=False)
        exact(m.detailPerLevel[:, b, :], d)
        exact(m.finalApprox[b], ap)
    y = vw.BatchMODWT.inverseMultiLevelAoS(w, m.detailPerLevel, m.finalApprox)
    for b in range(5):
        d, ap = O.decompose(x[b], *lohi(w), O.PERIODIC, 4, core=False)
        exact(y[b], O.reconstruct(d, ap, w.lowPassReconstruction(), w.highPassReconstruction(), O.PERIODIC))
    # no level cap in the facade (BatchMODWT.java:90-111): J=10 on N=8192 db4 is allowed
    m10 = vw.BatchMODWT.multiLevelAoS(w, signals(2, 8192, 1), 10)
    d, ap = O.decompose(signals(2, 8192, 1)[1], *lohi(w), O.PERIODIC, 10, core=False)
    exact(m10.detailPerLevel[:, 1, :], d)


# ---- SWT denoise -------------------------------------------------------------------------------------
@pytest.mark.parametrize("boundary", BOUNDARIES, ids=["P", "S", "Z"])
@pytest.mark.parametrize("n", [1024, 1025, 4096])
def test_swt_denoise_bit_exact(engine, boundary, n):
    w = Symlet.SYM8
    J = 4
    rng = np.random.default_rng(n)
    t = np.arange(n) / n
    x = np.stack([np.sin(2 * math.pi * 3 * t) + 0.5 * np.sin(2 * math.pi * 37 * t) + 0.2 * rng.standard_normal(n)
                  for _ in range(3)])
    swt = vw.VectorWaveSwtAdapter(w, vw.BoundaryMode(boundary))
    y, thr = swt.denoise(x, J, return_thresholds=True)
    for b in range(3):
        y_ref, t_ref = O.swt_denoise(x[b], *lohi(w), boundary, J, wavelet_id=w.wavelet_id)
        assert thr[b] == t_ref
        exact(y[b], y_ref)
    y2 = swt.denoise(x, J, 0.05, False)  # fixed hard threshold
    for b in range(3):
        exact(y2[b], O.swt_denoise(x[b], *lohi(w), boundary, J, 0.05, False, wavelet_id=w.wavelet_id)[0])


def test_noise_sigma_exact(engine):
    rng = np.random.default_rng(1)
    for n in (1, 2, 5, 1024, 1025, 16384, 20001):
        c = rng.standard_normal((3, n))
        c[0, : n // 3] = 0.0  # duplicates
        sig = vw.VectorWaveSwtAdapter(H).estimateNoiseSigma(c)
        for b in range(3):
            assert sig[b] == O.noise_sigma(c[b]), n


def _sigma_cases(n, rng):
    """Distributions that stress the selection kernel: ties, a single value, sub-normals, ranges spanning
    the exponent range, keys a few ulps apart (many refinement passes), non-finite keys."""
    one_ulp = np.spacing(1.0)
    return {
        "zeros": np.zeros(n),
        "const": np.full(n, -3.25),
        "two_values": np.where(rng.random(n) < 0.5, 1.0, 2.0),
        "subnormal": rng.standard_normal(n) * 1e-310,
        "wide": np.where(rng.random(n) < 0.5, 1e300, 1e-300) * rng.random(n),
        "ulps": 1.0 + rng.integers(0, 5000, n) * one_ulp,
        "ulps_narrow": 1.0 + rng.integers(0, 3, n) * one_ulp,
        "outlier": np.concatenate([rng.standard_normal(n - 1) * 1e-12, [1e308]]),
        "geometric": np.exp2(-rng.integers(0, 1000, n).astype(np.float64)),
        "inf": np.where(np.arange(n) % 7 == 0, np.inf, rng.standard_normal(n)),
        "nan": np.where(np.arange(n) % 3 == 0, np.nan, rng.standard_normal(n)),
        "signed_zero": np.where(rng.random(n) < 0.6, -0.0, 0.0) + (np.arange(n) % 11 == 0) * 1.5,
    }


@pytest.mark.parametrize("n", [2, 7, 1000, 4096, 16383, 16384, 16385])
def test_noise_sigma_adversarial(engine, n):
    rng = np.random.default_rng(n)
    cases = _sigma_cases(n, rng)
    c = np.stack(list(cases.values()))
    sig = vw.VectorWaveSwtAdapter(H).estimateNoiseSigma(c)
    for b, name in enumerate(cases):
        ref = O.noise_sigma(c[b])
        assert np.array_equal(np.float64(sig[b]), np.float64(ref), equal_nan=True), (name, n, sig[b], ref)


def test_swt_mutable_threshold_and_extract(engine):
    w = Daubechies.DB4
    x = signals(2, 512, 2)
    swt = vw.VectorWaveSwtAdapter(w)
    res = swt.forward(x, 4)
    swt.applyUniversalThreshold(res, True)
    for b in range(2):
        d, a = O.swt_forward(x[b], *lohi(w), O.PERIODIC, 4)
        T = O.universal_threshold(O.noise_sigma(d[0]), 512)
        for j in range(4):
            exact(res.getDetailCoeffsAtLevel(j + 1)[b], O.threshold(d[j], T, True))
    e = swt.extractLevel(x, 4, 2)
    for b in range(2):
        d, a = O.swt_forward(x[b], *lohi(w), O.PERIODIC, 4)
        exact(e[b], O.reconstruct(d, a, w.lowPassReconstruction(), w.highPassReconstruction(), O.PERIODIC,
                                  detail_mask=0b0010, approx_zero=True))


# ---- streaming -------------------------------------------------------------------------------------
@pytest.mark.parametrize("boundary", [O.ZERO_PADDING, O.SYMMETRIC], ids=["Z", "S"])
@pytest.mark.parametrize("blk,J", [(256, 3), (12000, 5)])   # 12000 > fused capacity: per-level path + sweeps
def test_streaming_blocks_match_whole_signal(engine, boundary, blk, J):
    w = Daubechies.DB4
    nb = 4 if blk <= 4096 else 2
    x = signals(2, blk * nb, 8)
    st = vw.BatchStreamingMODWT(w, vw.BoundaryMode(boundary), J)
    outs = [st.processMultiLevel(x[:, k * blk:(k + 1) * blk]) for k in range(nb)]
    for b in range(2):
        d_ref, a_ref = O.decompose(x[b], *lohi(w), boundary, J)
        got_d = np.concatenate([o.detailPerLevel[:, b, :] for o in outs], axis=1)
        got_a = np.concatenate([o.finalApprox[b] for o in outs])
        if boundary == O.ZERO_PADDING:
            exact(got_d, d_ref)
            exact(got_a, a_ref)
        else:  # history carries the left context; the first block mirrors like the whole signal
            exact(got_d, d_ref)
            exact(got_a, a_ref)
    tail = st.flushMultiLevel(st.getMinFlushTailLength())
    assert tail.finalApprox.shape == (2, st.getMinFlushTailLength())
    st.close()


@pytest.mark.parametrize("boundary", [O.ZERO_PADDING, O.SYMMETRIC], ids=["Z", "S"])
@pytest.mark.parametrize("w,blk,J", [(Daubechies.DB4, 256, 3), (Symlet.SYM8, 1000, 2), (H, 64, 4),
                                     (Daubechies.DB4, 12000, 5)], ids=["db4-256", "sym8-1000", "haar-64", "db4-12000"])
def test_streaming_history_and_flush_values(engine, boundary, w, blk, J):
    # BatchStreamingMODWT ZERO/SYMMETRIC: every block and the flush tail (synthetic zeros / reflected
    # history run through every level's history) against the restatement, bit for bit; tail lengths
    # up to getMinFlushTailLength(), single-level flush too
    x = signals(2, blk * 3, 17)
    st = vw.BatchStreamingMODWT(w, vw.BoundaryMode(boundary), J)
    refs = [O.StreamRestatement(*lohi(w), boundary, J) for _ in range(2)]
    for k in range(3):
        out = st.processMultiLevel(x[:, k * blk:(k + 1) * blk])
        for b in range(2):
            d_ref, a_ref = refs[b].process(x[b, k * blk:(k + 1) * blk])
            exact(out.detailPerLevel[:, b, :], d_ref)
            exact(out.finalApprox[b], a_ref)
    m = st.getMinFlushTailLength()
    assert m == (w.filter_length - 1)
    for tl in sorted({1, m // 2 or 1, m}):
        tail = st.flushMultiLevel(tl)
        for b in range(2):
            d_ref, a_ref = refs[b].flush(tl)
            exact(tail.detailPerLevel[:, b, :], d_ref)
            exact(tail.finalApprox[b], a_ref)
    with pytest.raises(vw.InvalidArgumentException):
        st.flushMultiLevel(m + 1)
    st.close()
    s1 = vw.BatchStreamingMODWT(w, vw.BoundaryMode(boundary), 1)
    r1 = O.StreamRestatement(*lohi(w), boundary, 1)
    s1.processSingleLevel(x[:1, :blk])
    r1.process(x[0, :blk])
    t1 = s1.flushSingleLevel(w.filter_length - 1)
    d_ref, a_ref = r1.flush(w.filter_length - 1)
    exact(t1.detail[0], d_ref[0])
    exact(t1.approx[0], a_ref)
    s1.close()


# ---- FMA and fp32 variants --------------------------------------------------------------------------
def test_fma_variant_within_tolerance(engine):
    w = Daubechies.DB4
    x = signals(4, 4096, 13)
    res = vw.MultiLevelMODWTTransform(w, vw.BoundaryMode.PERIODIC, fma=True).decompose(x, 6)
    y = vw.MultiLevelMODWTTransform(w, vw.BoundaryMode.PERIODIC, fma=True).reconstruct(res)
    for b in range(4):
        d, a = O.decompose(x[b], *lohi(w), O.PERIODIC, 6)
        np.testing.assert_allclose(res.details_array[:, b, :], d, rtol=0, atol=1e-12)
        np.testing.assert_allclose(y[b], O.reconstruct(d, a, w.lowPassReconstruction(), w.highPassReconstruction(),
                                                       O.PERIODIC), rtol=0, atol=1e-12)


@pytest.mark.parametrize("case", [
    ("db4", O.PERIODIC, 4096, 6, "f64", nat.FLAG_FMA, None),
    ("db4", O.PERIODIC, 4096, 6, "f64", 0, "2"),          # EXACT on two buffers -> persistent, bit-exact
    ("db4", O.SYMMETRIC, 4096, 5, "f64", nat.FLAG_FMA, None),
    ("db4", O.ZERO_PADDING, 4096, 4, "f64", nat.FLAG_FMA, None),
    ("sym8", O.PERIODIC, 4096, 6, "f64", nat.FLAG_FMA, None),
    ("db4", O.PERIODIC, 1024, 3, "f64", nat.FLAG_FMA, "2"),
    ("coif5", O.PERIODIC, 8192, 6, "f32", nat.FLAG_FMA, None),
], ids=lambda c: f"{c[0]}-{c[1]}-{c[2]}-J{c[3]}-{c[4]}-{'fma' if c[5] else 'exact'}")
def test_forward_persistent_matches_per_signal_kernel(engine, case):
    """k_forward_persist (a workgroup walks several signals; the next row arrives by LDS-DMA during the
    last level) against k_forward_fused (one signal per workgroup): identical arithmetic, so identical
    bits, over a batch larger than the resident grid (every workgroup handles >= 2 signals)."""
    import torch
    wname, boundary, n, J, dt, flags, buf = case
    w = {"db4": Daubechies.DB4, "sym8": Symlet.SYM8, "coif5": Coiflet.COIF5}[wname]
    B = 1100 if n <= 4096 else 700
    dtype = torch.float64 if dt == "f64" else torch.float32
    x = torch.empty((B, n), dtype=dtype, device="cuda")
    engine.fill_uniform(x, 5)
    outs = []
    for nv in (4, 8, 2):
        for persist in (0, 1):
            opts = dict(VW_FWD_PERSIST=persist, VW_NV=nv) if nv != 2 else dict(VW_FWD_PERSIST=persist, VW_FWD_NV=2)
            if buf:
                opts["VW_FWD_BUF"] = int(buf)
            with engine.options(**opts):
                outs.append(engine.forward(x, *lohi(w), w.wavelet_id, boundary, J, flags))
            torch.cuda.synchronize()
    for d_, a_ in outs[2:]:  # the NV = 8 / NV = 2 kernels (half / twice the threads) compute the same bits
        assert torch.equal(d_, outs[0][0]) and torch.equal(a_, outs[0][1])
    outs = outs[:2]
    (d0, a0), (d1, a1) = outs
    assert torch.equal(d0, d1) and torch.equal(a0, a1)
    xh = x.double().cpu().numpy()
    tol = 1e-12 if dt == "f64" else 1e-5 * float(x.abs().max().item()) * J
    for b in (0, 511, 512, B - 1):
        d_ref, a_ref = O.decompose(xh[b], *lohi(w), boundary, J)
        got_d, got_a = d1[:, b, :].double().cpu().numpy(), a1[b].double().cpu().numpy()
        if dt == "f64" and not flags:
            exact(got_d, d_ref)
            exact(got_a, a_ref)
        else:
            np.testing.assert_allclose(got_d, d_ref, rtol=0, atol=tol)
            np.testing.assert_allclose(got_a, a_ref, rtol=0, atol=tol)


def test_fp32_path(engine):
    import torch
    w = Coiflet.COIF5
    x64 = signals(3, 8192, 17)
    x = torch.tensor(x64, dtype=torch.float32, device="cuda")
    det, app = engine.forward(x, *lohi(w), w.wavelet_id, O.PERIODIC, 6, 0)
    y = engine.inverse(det, app, w.lowPassReconstruction(), w.highPassReconstruction(), w.wavelet_id, O.PERIODIC, 6,
                       nat.FLAG_CORE_LEVELS)
    tol = 1e-5 * float(np.max(np.abs(x64))) * 6
    for b in range(3):
        d, a = O.decompose(x64[b], *lohi(w), O.PERIODIC, 6, core=False)
        np.testing.assert_allclose(det[:, b, :].double().cpu().numpy(), d, rtol=0, atol=tol)
        np.testing.assert_allclose(app[b].double().cpu().numpy(), a, rtol=0, atol=tol)
        np.testing.assert_allclose(y[b].double().cpu().numpy(),
                                   O.reconstruct(d, a, w.lowPassReconstruction(), w.highPassReconstruction(),
                                                 O.PERIODIC), rtol=0, atol=tol)


# ---- tiled (long-signal) path ---------------------------------------------------------------------------
def test_tiled_path_bit_exact(engine):
    # levels with spacing >= 16 run as column sweeps (N % s != 0 exercises wraps across residues)
    with engine.options(VW_FORCE_TILED=1):
        for w, boundary, n, J in [(Daubechies.DB4, O.PERIODIC, 10000, 6), (Daubechies.DB8, O.SYMMETRIC, 5000, 4),
                                  (Symlet.SYM8, O.ZERO_PADDING, 9000, 5), (Daubechies.DB8, O.SYMMETRIC, 7001, 6),
                                  (Coiflet.COIF5, O.PERIODIC, 20000, 6),
                                  (Daubechies.DB4, O.SYMMETRIC, 4099, 8)]:
            x = signals(2, n, 19)
            tx = vw.MultiLevelMODWTTransform(w, vw.BoundaryMode(boundary))
            res = tx.decompose(x, J)
            y = tx.reconstruct(res)
            for b in range(2):
                d, a = O.decompose(x[b], *lohi(w), boundary, J)
                exact(res.details_array[:, b, :], d)
                exact(res.approximation_array[b], a)
                exact(y[b], O.reconstruct(d, a, w.lowPassReconstruction(), w.highPassReconstruction(), boundary,
                                          w.wavelet_id))


@pytest.mark.parametrize("tile", [128, 2048])
def test_multilevel_tiles_bit_exact(engine, tile):
    # long PERIODIC signals run groups of levels per tile (vw_capi.cpp level_groups): odd N (scalar
    # I/O), N not a multiple of the tile, tiles shorter than the reach (wraps through the halo), and
    # the SWT denoise thresholds applied on the detail loads; EXACT mode is bit-exact
    with engine.options(VW_FORCE_TILED=1, VW_MULTI_TILE=tile):
        for w, n, J in [(Daubechies.DB4, 10000, 6), (Daubechies.DB8, 30001, 8), (H, 5000, 9),
                        (Coiflet.COIF5, 20000, 5), (Symlet.SYM8, 4097, 6)]:   # J=7 would enter the FFT region
            x = signals(2, n, 23)
            tx = vw.MultiLevelMODWTTransform(w, vw.BoundaryMode.PERIODIC)
            res = tx.decompose(x, J)
            y = tx.reconstruct(res)
            for b in range(2):
                d, a = O.decompose(x[b], *lohi(w), O.PERIODIC, J)
                exact(res.details_array[:, b, :], d)
                exact(res.approximation_array[b], a)
                exact(y[b], O.reconstruct(d, a, w.lowPassReconstruction(), w.highPassReconstruction(), O.PERIODIC))
        w, n, J = Symlet.SYM8, 12000, 5
        x = signals(2, n, 29)
        y, thr = vw.VectorWaveSwtAdapter(w, vw.BoundaryMode.PERIODIC).denoise(x, J, return_thresholds=True)
        for b in range(2):
            y_ref, t_ref = O.swt_denoise(x[b], *lohi(w), O.PERIODIC, J, wavelet_id=w.wavelet_id)
            assert thr[b] == t_ref
            exact(y[b], y_ref)


@pytest.mark.parametrize("opts", [dict(VW_MULTI_PAD=0), dict(VW_MULTI_INV_TILE=1792), dict(VW_MULTI_INV_TILE=1024),
                                  dict(VW_MULTI_INV_TILE=512, VW_MULTI_TILE=512), dict(VW_MULTI_NI=4),
                                  dict(VW_MULTI_NI=4, VW_MULTI_TILE=1024), dict(VW_MULTI_NI=8)],
                         ids=lambda d: ",".join(f"{k}={v}" for k, v in d.items()))
def test_multilevel_inverse_padded_layout(engine, opts):
    """k_inverse_multi's padded LDS layout at the register-blocked levels (VW_MULTI_PAD, default on), its own
    tile (VW_MULTI_INV_TILE) and its outputs per thread (VW_MULTI_NI: 8, or 4 on the largest tile whose levels
    fit, with the NV = 4 pad layouts): EXACT bit-exact vs the restatement; FMA and fp32 identical bits to the
    default configuration (the same per-output operation sequence, only LDS addresses move)."""
    import torch
    with engine.options(VW_FORCE_TILED=1):
        for w, n, J in [(Daubechies.DB8, 1 << 15, 9), (Daubechies.DB4, 12288, 8), (Symlet.SYM8, 1 << 14, 6)]:
            x = signals(2, n, 37)
            tx = vw.MultiLevelMODWTTransform(w, vw.BoundaryMode.PERIODIC)
            res = tx.decompose(x, J)
            with engine.options(**opts):
                y = tx.reconstruct(res)
            for b in range(2):
                d, a = O.decompose(x[b], *lohi(w), O.PERIODIC, J)
                exact(y[b], O.reconstruct(d, a, w.lowPassReconstruction(), w.highPassReconstruction(), O.PERIODIC))
        for w, n, J, dt in [(Daubechies.DB8, 1 << 15, 10, torch.float64), (Coiflet.COIF5, 1 << 15, 7, torch.float32)]:
            x = torch.empty((3, n), dtype=dt, device="cuda")
            engine.fill_uniform(x, 8)
            rl, rh = w.lowPassReconstruction(), w.highPassReconstruction()
            d1, a1 = engine.forward(x, *lohi(w), w.wavelet_id, O.PERIODIC, J, nat.FLAG_FMA)
            y0 = engine.inverse(d1, a1, rl, rh, w.wavelet_id, O.PERIODIC, J, nat.FLAG_FMA)
            with engine.options(**opts):
                y1 = engine.inverse(d1, a1, rl, rh, w.wavelet_id, O.PERIODIC, J, nat.FLAG_FMA)
            torch.cuda.synchronize()
            assert torch.equal(y0, y1), (w.name(), dt)


@pytest.mark.parametrize("ni", [4, 8])
def test_multilevel_inverse_outputs_per_thread_edges(engine, ni):
    """k_inverse_multi at NI = 4 (default for fp64: its own tile, 1792 samples for db8) and NI = 8 on the shapes
    the tile choice touches: a partial last tile (N not a multiple of either tile), L = 30 (coif5: its reach moves
    the NI = 4 tile down further), levels past the group (J = 8 at N = 16384, the deepest below the FFT region,
    L_J <= N/8, where the reference switches to an FFT) and the SWT denoise thresholds applied on the detail
    loads.  EXACT bit-exact vs the restatement."""
    with engine.options(VW_FORCE_TILED=1, VW_MULTI_NI=ni):
        for w, n, J in [(Daubechies.DB8, 3 * 1792 + 500, 5), (Coiflet.COIF5, 12000, 4), (Daubechies.DB8, 1 << 14, 8)]:
            x = signals(2, n, 53)
            tx = vw.MultiLevelMODWTTransform(w, vw.BoundaryMode.PERIODIC)
            res = tx.decompose(x, J)
            y = tx.reconstruct(res)
            for b in range(2):
                d, a = O.decompose(x[b], *lohi(w), O.PERIODIC, J)
                exact(y[b], O.reconstruct(d, a, w.lowPassReconstruction(), w.highPassReconstruction(), O.PERIODIC))
        w, n, J = Daubechies.DB8, 9000, 5
        x = signals(2, n, 59)
        y, thr = vw.VectorWaveSwtAdapter(w, vw.BoundaryMode.PERIODIC).denoise(x, J, return_thresholds=True)
        for b in range(2):
            y_ref, t_ref = O.swt_denoise(x[b], *lohi(w), O.PERIODIC, J, wavelet_id=w.wavelet_id)
            assert thr[b] == t_ref
            exact(y[b], y_ref)


# ---- alternative fused inverse kernels (selected by policy or option) ------------------------------------
@pytest.mark.parametrize("opts", [dict(VW_INV_BUF=1), dict(VW_INV_BUF=2), dict(VW_NV=8), dict(VW_INV_BUF=1, VW_NV=8),
                                  dict(VW_INV_NV=2), dict(VW_INV_NV=2, VW_INV_BUF=1), dict(VW_INV_NV=2, VW_INV_BUF=2)],
                         ids=lambda d: ",".join(f"{k}={v}" for k, v in d.items()))
@pytest.mark.parametrize("fma", [False, True], ids=["exact", "fma"])
def test_inverse_kernel_variants_bit_exact(engine, opts, fma):
    # every variant computes the reference's sums in the reference's order: EXACT bit-exact, FMA equal
    # to the default FMA kernel (same per-output operation sequence)
    cases = [(Daubechies.DB4, 4096, 6, 8), (Daubechies.DB4, 4096, 9, 3), (Symlet.SYM8, 4096, 8, 3),
             (H, 2048, 7, 4), (Daubechies.DB8, 1024, 5, 5), (Coiflet.COIF5, 8192, 6, 2)]
    for w, n, J, B in cases:
        x = signals(B, n, 41)
        tx = vw.MultiLevelMODWTTransform(w, vw.BoundaryMode.PERIODIC, fma=fma)
        res = tx.decompose(x, J)
        y0 = tx.reconstruct(res)
        with engine.options(**opts):
            y1 = tx.reconstruct(res)
            y2 = vw.VectorWaveSwtAdapter(w, vw.BoundaryMode.PERIODIC, fma=fma).denoise(x, J)
        y2_ref = vw.VectorWaveSwtAdapter(w, vw.BoundaryMode.PERIODIC, fma=fma).denoise(x, J)
        exact(y1, y0)
        exact(y2, y2_ref)
        if not fma:
            for b in range(B):
                d, a = res.details_array[:, b, :], res.approximation_array[b]
                exact(y1[b], O.reconstruct(d, a, w.lowPassReconstruction(), w.highPassReconstruction(), O.PERIODIC))


def test_long_block_db8_j10(engine):
    # config 4 shape on a short batch: 2^17-sample PERIODIC block, db8, J=10 (BatchMODWT semantics)
    w = Daubechies.DB8
    n = 1 << 17
    x = O.fill_uniform(n, 42).reshape(1, n)
    m = vw.BatchMODWT.multiLevelAoS(w, x, 10)
    y = vw.BatchMODWT.inverseMultiLevelAoS(w, m.detailPerLevel, m.finalApprox)
    assert np.max(np.abs(y - x)) < 1e-8   # truncated DB8 taps limit PR (SURVEY.md key fact 5)
    # bit-exact spot check of the first levels against the restatement
    d, a = O.decompose(x[0], *lohi(w), O.PERIODIC, 2, core=False)
    m2 = vw.BatchMODWT.multiLevelAoS(w, x, 2)
    exact(m2.detailPerLevel[:, 0, :], d)


# ---- device-resident path at the headline size --------------------------------------------------
def test_headline_device_resident_properties(engine):
    import torch
    w = Daubechies.DB4
    B, n, J = 4096, 4096, 6
    x = torch.empty((B, n), dtype=torch.float64, device="cuda")
    engine.fill_uniform(x, 42)
    # generator parity with the restatement
    exact(x[17].cpu().numpy(), O.fill_uniform(n, 42, 17 * n))
    det, app = engine.forward(x, *lohi(w), w.wavelet_id, O.PERIODIC, J, 0)
    y = engine.inverse(det, app, w.lowPassReconstruction(), w.highPassReconstruction(), w.wavelet_id, O.PERIODIC, J,
                       nat.FLAG_CORE_LEVELS)
    torch.cuda.synchronize()
    err = (y - x).abs().max().item()
    assert err < 1e-9, err   # DB4 taps are truncated: PR ~5e-11 (SURVEY.md key fact 5)
    # energy: sum_j ||d_j||^2 + ||a_J||^2 == ||x||^2 per signal (orthogonal MODWT)
    ex = (x * x).sum(1)
    et = (det * det).sum((0, 2)) + (app * app).sum(1)
    assert ((et - ex).abs() / ex).max().item() < 1e-9
    # rows spot-checked bit for bit against the restatement
    for b in (0, 1234, 4095):
        d, a = O.decompose(x[b].cpu().numpy(), *lohi(w), O.PERIODIC, J)
        exact(det[:, b, :].cpu().numpy(), d)
        exact(app[b].cpu().numpy(), a)


# ---- SoA facade (BatchSIMDMODWT) -----------------------------------------------------------------------
@pytest.mark.parametrize("B,n", [(3, 1000), (130, 67), (64, 64), (1, 5)])
def test_soa_layout_round_trip(engine, B, n):
    import torch
    x = signals(B, n, 3)
    soa = vw.BatchSIMDMODWT.convertToSoA(x)
    exact(soa, x.T.reshape(-1))                              # convertToSoA :282-292: index t*B + b
    exact(vw.BatchSIMDMODWT.convertFromSoA(soa, B, n), x)     # convertFromSoA :299-308
    xd = torch.tensor(x, device="cuda")
    sd = vw.BatchSIMDMODWT.convertToSoA(xd)
    assert sd.is_cuda
    exact(sd.cpu().numpy(), x.T.reshape(-1))


@pytest.mark.parametrize("w", [H, Daubechies.DB2, Daubechies.DB4, Symlet.SYM8], ids=lambda w: w.name())
def test_soa_single_and_multilevel_match_restatement(engine, w):
    B, n = 5, 256
    x = signals(B, n, 21)
    soa = x.T.reshape(-1).copy()
    sa, sd = vw.BatchSIMDMODWT.batchMODWTSoA(soa, w, B, n)
    for b in range(B):
        ra, rd = O.batch_single(x[b], *lohi(w), w is H)
        exact(sa.reshape(n, B)[:, b], ra)
        exact(sd.reshape(n, B)[:, b], rd)
    J = 4
    sdet, sapp = vw.BatchSIMDMODWT.batchMultiLevelMODWTSoA(soa, w, B, n, J)
    assert sdet.shape == (J, n * B)
    for b in range(B):
        d, a = O.decompose(x[b], *lohi(w), O.PERIODIC, J, core=False)
        exact(sdet.reshape(J, n, B)[:, :, b], d)
        exact(sapp.reshape(n, B)[:, b], a)


# ---- core Flow-API streaming (MODWTStreamingTransform) --------------------------------------------------
class _Collect:
    def __init__(self):
        self.items, self.done = [], False

    def onNext(self, r):
        self.items.append(r)

    def onComplete(self):
        self.done = True


@pytest.mark.parametrize("w,buf", [(Daubechies.DB4, 64), (H, 16), (Symlet.SYM8, 100)], ids=["db4", "haar", "sym8"])
@pytest.mark.parametrize("boundary", [O.PERIODIC, O.SYMMETRIC], ids=["P", "S"])
def test_streaming_transform_windows(engine, w, buf, boundary):
    """MODWTStreamingTransformImpl: windows of bufferSize overlapping by L-1 (:188-218), flush zero-pads the
    rest (:228-252); chunks of any size (one batched device call per process())."""
    rng = np.random.default_rng(buf)
    x = rng.standard_normal(1000)
    st = vw.MODWTStreamingTransform.create(w, vw.BoundaryMode(boundary), buf)
    sub = _Collect()
    st.subscribe(sub)
    pos = 0
    for n in (1, 7, buf - 1, 3 * buf + 5, 250, 1):
        st.process(x[pos:pos + n])
        pos += n
    st.process(x[pos:])
    st.close()
    L = len(w.lowPassDecomposition())
    hop = buf - (L - 1)
    starts = list(range(0, len(x) - buf + 1, hop))
    rem = len(x) - (starts[-1] + hop)
    assert sub.done and len(sub.items) == len(starts) + (1 if rem > 0 else 0)
    for r, s0 in zip(sub.items, starts):
        a, d = O.modwt_forward(x[s0:s0 + buf], *lohi(w), boundary)
        exact(r.approximationCoeffs(), a)
        exact(r.detailCoeffs(), d)
    if rem > 0:
        tail = np.zeros(buf)
        tail[:rem] = x[len(x) - rem:]
        a, d = O.modwt_forward(tail, *lohi(w), boundary)
        exact(sub.items[-1].approximationCoeffs(), a)
    assert st.getStatistics().getSamplesProcessed() == len(x)
    with pytest.raises(vw.InvalidStateException):
        st.process(x[:4])


def test_streaming_multilevel_blocks(engine):
    """MultiLevelMODWTStreamingTransform: non-overlapping blocks, one result per level, approximation
    only at the last level (:133-166, :238-240)."""
    w, buf, J = Daubechies.DB4, 128, 3
    x = np.random.default_rng(5).standard_normal(3 * buf + 40)
    st = vw.MODWTStreamingTransform.createMultiLevel(w, vw.BoundaryMode.PERIODIC, buf, J)
    got = []
    st.subscribe(got.append)
    st.process(x[:100])
    st.process(x[100:])
    st.flush()
    blocks = [x[k * buf:(k + 1) * buf] for k in range(3)] + [np.concatenate([x[3 * buf:], np.zeros(buf - 40)])]
    assert len(got) == 4 * J
    for k, blk in enumerate(blocks):
        d, a = O.decompose(blk, *lohi(w), O.PERIODIC, J)
        for j in range(J):
            r = got[k * J + j]
            exact(r.detailCoeffs(), d[j])
            assert r.approximationCoeffs().size == (buf if j == J - 1 else 0)
        exact(got[k * J + J - 1].approximationCoeffs(), a)
    with pytest.raises(vw.InvalidArgumentException):
        vw.MODWTStreamingTransform.createMultiLevel(w, vw.BoundaryMode.PERIODIC, buf, 0)
    with pytest.raises(vw.InvalidArgumentException):
        vw.MODWTStreamingTransform.create(w, vw.BoundaryMode.PERIODIC, 4)  # bufferSize < filter length


def test_forward_strided_rows_ldx(engine):
    """vw_modwt_forward_f64 with ldx > N (rows of a wider buffer, e.g. a strided JNI view): the
    persistent forward's row DMA and the per-signal kernels address row b at x + b*ldx."""
    import ctypes
    import torch
    w = Daubechies.DB4
    B, N, J, pad = 600, 4096, 6, 64
    big = torch.empty((B, N + pad), dtype=torch.float64, device="cuda")
    engine.fill_uniform(big, 9)
    x = big[:, :N].contiguous()
    lib = nat.load()
    for flags in (nat.FLAG_FMA, 0):
        det = torch.empty((J, B, N), dtype=torch.float64, device="cuda")
        app = torch.empty((B, N), dtype=torch.float64, device="cuda")
        st = lib.vw_modwt_forward_f64(engine.ctx, ctypes.c_void_p(big.data_ptr()), B, N, N + pad,
                                      nat.taps_array(w.lowPassDecomposition()), nat.taps_array(w.highPassDecomposition()),
                                      8, w.wavelet_id, O.PERIODIC, J, flags, ctypes.c_void_p(det.data_ptr()),
                                      ctypes.c_void_p(app.data_ptr()))
        assert st == 0
        d2, a2 = engine.forward(x, w.lowPassDecomposition(), w.highPassDecomposition(), w.wavelet_id, O.PERIODIC, J,
                                flags)
        torch.cuda.synchronize()
        assert torch.equal(det, d2) and torch.equal(app, a2)


# ---- register-blocked PERIODIC kernels (long filters, vw_device.h k_forward_blk / k_inverse_blk) --------
@pytest.mark.parametrize("case", [("sym8", 16384, 8, "f64", 3), ("sym8", 4096, 8, "f64", 5), ("db8", 4096, 6, "f64", 5),
                                  ("coif5", 8192, 6, "f32", 6), ("coif5", 4096, 5, "f64", 3), ("db6", 2048, 7, "f64", 4)],
                         ids=lambda c: f"{c[0]}-{c[1]}-J{c[2]}-{c[3]}")
@pytest.mark.parametrize("fma", [False, True], ids=["exact", "fma"])
def test_blocked_kernels_match_default(engine, case, fma):
    # the blocked kernels run every output's taps in the same order as the one-vector-per-tap kernels:
    # identical bits (EXACT and FMA), and EXACT equals the restatement
    import torch
    wname, n, J, dt, B = case
    w = vw.get_wavelet(wname)
    dtype = torch.float64 if dt == "f64" else torch.float32
    x = torch.from_numpy(O.fill_uniform(B * n, 9).reshape(B, n)).to(dtype).cuda()
    flags = nat.FLAG_FMA if fma else 0
    out = {}
    # 8: the blocked forward at NV = 8 too (1024-thread workgroups; VW_BLK_FWD8)
    for blk in (0, 2, 8):
        with engine.options(VW_BLK=min(blk, 2), VW_BLK_FWD8=int(blk == 8)):
            d, a = engine.forward(x, *lohi(w), w.wavelet_id, O.PERIODIC, J, flags)
            y = engine.inverse(d, a, w.lowPassReconstruction(), w.highPassReconstruction(), w.wavelet_id, O.PERIODIC,
                               J, flags)
            torch.cuda.synchronize()
            out[blk] = (d, a, y)
    for v in (2, 8):
        for t0, t1 in zip(out[0], out[v]):
            assert torch.equal(t0, t1), v
    if dt == "f64" and not fma:
        d, a, y = (t.cpu().numpy() for t in out[2])
        xh = x.cpu().numpy()
        for b in (0, B - 1):
            d_ref, a_ref = O.decompose(xh[b], *lohi(w), O.PERIODIC, J, core=False)
            exact(d[:, b, :], d_ref)
            exact(a[b], a_ref)
            exact(y[b], O.reconstruct(d_ref, a_ref, w.lowPassReconstruction(), w.highPassReconstruction(), O.PERIODIC))
    if wname == "sym8" and n == 16384 and not fma:
        # the config-3 denoise through the blocked kernels: thresholds and outputs bit-exact
        y2, thr = vw.VectorWaveSwtAdapter(w, vw.BoundaryMode.PERIODIC).denoise(x.cpu().numpy(), J, return_thresholds=True)
        for b in (0, B - 1):
            y_ref, t_ref = O.swt_denoise(x[b].cpu().numpy(), *lohi(w), O.PERIODIC, J, wavelet_id=w.wavelet_id)
            assert thr[b] == t_ref
            exact(y2[b], y_ref)


# ---- non-finite inputs on the unvalidated batch path ------------------------------------------------------
def test_batch_nonfinite_inputs_match_the_reference(engine):
    """BatchMODWT.multiLevelAoS has no finite check (BatchMODWT.java:201-212) and multiplies the zero taps of
    the upsampled filters (BatchSIMDMODWT.java:400-404), so a non-finite sample turns every output whose
    window reaches it through a zero tap into NaN (0 * Inf).  The facade sets VW_FLAG_REF_NONFINITE: such
    rows are recomputed with the reference's full-tap loops, so NaN masks, +-Inf and every finite value are
    identical (more cases: tests/test_gpu_nonfinite.py).  L_j > N + 1 raises like Java's negative index."""
    w = Daubechies.DB4
    n, J = 512, 4
    x = signals(3, n, 51)
    x[0, 100] = np.inf
    x[1, 7] = np.nan
    x[2, 300] = -np.inf
    x[2, 301] = np.inf
    m = vw.BatchMODWT.multiLevelAoS(w, x, J)
    for b in range(3):
        d_ref, a_ref = O.decompose(x[b], *lohi(w), O.PERIODIC, J, core=False)
        for got, ref in ((m.detailPerLevel[:, b, :], d_ref), (m.finalApprox[b], a_ref)):
            assert np.array_equal(np.isnan(got), np.isnan(ref))
            assert np.array_equal(got[~np.isnan(got)].view(np.int64), ref[~np.isnan(ref)].view(np.int64))
            assert np.isnan(ref).any()  # the non-finite sample reaches the outputs through the zero taps
    with pytest.raises(IndexError):
        vw.BatchMODWT.multiLevelAoS(w, signals(1, 64, 3), 5)   # L_5 = 7*16+1 = 113 > 65

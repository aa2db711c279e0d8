"""Streaming deep-level kernels (vw_deep.hip k_forward_deep / k_inverse_deep): the PERIODIC levels of
long signals past the multi-level tile group, one launch each way, streamed along the decimated
coordinate with per-level LDS rings.  EXACT: bit-exact against the restatement of vectorwave-core
(MultiLevelMODWTTransform.java:243-251 forward, :339-349 / :576-589 inverse); FMA: identical bits to
the column sweeps they replace (same per-output operation sequence, VW_DEEP=0 A/B).  Shapes cover
several groups / segments, residue blocks, fp32 (C = 16), masked details, zero approximation, the
fused denoise thresholds, and an N the deep path must decline (N % P != 0)."""
import numpy as np
import pytest

from oracle import oracle as O
import vectorwave_amd as vw
from vectorwave_amd import _native as nat
from vectorwave_amd.wavelets import Coiflet, Daubechies, Haar, Symlet

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def deep_on(engine):
    """Every test here runs the deep kernels whatever the default policy (VW_DEEP=1)."""
    engine.set_option("VW_DEEP", 1)
    yield
    engine.set_option("VW_DEEP", -1)


def _rows(B, n, seed):
    return np.stack([O.java_random_signal(n, seed + b) for b in range(B)])


def lohi(w):
    return w.lowPassDecomposition(), w.highPassDecomposition()


def lohi_r(w):
    return w.lowPassReconstruction(), w.highPassReconstruction()


@pytest.mark.parametrize("w,n,J,B", [(Daubechies.DB8, 1 << 15, 10, 2), (Haar.INSTANCE, 1 << 13, 12, 3),
                                     (Daubechies.DB4, 1 << 14, 10, 2), (Symlet.SYM8, 1 << 16, 9, 1),
                                     (Daubechies.DB8, 30000, 6, 2)],
                         ids=["db8-2^15-J10", "haar-2^13-J12", "db4-2^14-J10", "sym8-2^16-J9", "db8-30000-declined"])
def test_deep_forward_inverse_bit_exact(engine, w, n, J, B):
    x = _rows(B, n, 5)
    d, a = engine.forward(x, *lohi(w), w.wavelet_id, O.PERIODIC, J, 0)        # BatchMODWT semantics (no cap)
    y = engine.inverse(d, a, *lohi_r(w), w.wavelet_id, O.PERIODIC, J, 0)
    for b in range(B):
        d_ref, a_ref = O.decompose(x[b], *lohi(w), O.PERIODIC, J, core=False)
        assert np.array_equal(d[:, b, :], d_ref), b
        assert np.array_equal(a[b], a_ref), b
        assert np.array_equal(y[b], O.reconstruct(d_ref, a_ref, *lohi_r(w), O.PERIODIC)), b


@pytest.mark.parametrize("w,n,J,dt", [(Daubechies.DB8, 1 << 16, 10, "f64"), (Coiflet.COIF5, 1 << 15, 8, "f32"),
                                      (Daubechies.DB4, 1 << 17, 12, "f32")])
def test_deep_matches_column_sweeps(engine, w, n, J, dt):
    """FMA and fp32: the deep kernels and the column sweeps compute every output with the same operation
    sequence, so their bits agree (VW_DEEP=0 restores the sweeps)."""
    import torch
    tdt = torch.float64 if dt == "f64" else torch.float32
    x = torch.empty((3, n), dtype=tdt, device="cuda")
    engine.fill_uniform(x, 9)
    for flags in (0, nat.FLAG_FMA):
        d1, a1 = engine.forward(x, *lohi(w), w.wavelet_id, O.PERIODIC, J, flags)
        y1 = engine.inverse(d1, a1, *lohi_r(w), w.wavelet_id, O.PERIODIC, J, flags)
        with engine.options(VW_DEEP=0):
            d0, a0 = engine.forward(x, *lohi(w), w.wavelet_id, O.PERIODIC, J, flags)
            y0 = engine.inverse(d1, a1, *lohi_r(w), w.wavelet_id, O.PERIODIC, J, flags)
        torch.cuda.synchronize()
        assert torch.equal(d1, d0) and torch.equal(a1, a0), (w.name(), dt, flags)
        assert torch.equal(y1, y0), (w.name(), dt, flags)


@pytest.mark.parametrize("lds", [40, 160])
def test_deep_group_split_and_segments(engine, lds):
    """A small LDS budget splits levels 6..10 into several deep groups (more launches, same bits); one
    long block (B = 1) is cut into many segments, each with its own warm-up."""
    w = Daubechies.DB8
    n, J = 1 << 20, 10
    x = O.fill_uniform(n, 42).reshape(1, n)
    with engine.options(VW_DEEP_LDS=lds):
        d, a = engine.forward(x, *lohi(w), w.wavelet_id, O.PERIODIC, J, 0)
        y = engine.inverse(d, a, *lohi_r(w), w.wavelet_id, O.PERIODIC, J, 0)
    d_ref, a_ref = O.decompose(x[0], *lohi(w), O.PERIODIC, J, core=False)
    assert np.array_equal(d[:, 0, :], d_ref)
    assert np.array_equal(a[0], a_ref)
    assert np.array_equal(y[0], O.reconstruct(d_ref, a_ref, *lohi_r(w), O.PERIODIC))


def test_deep_partial_reconstruction(engine):
    """reconstructFromLevel / reconstructLevels on a long signal: masked details and a zero approximation
    through the deep inverse (MultiLevelMODWTTransform.java:361-446)."""
    w = Daubechies.DB8
    n, J = 1 << 15, 9
    x = _rows(2, n, 13)
    d, a = engine.forward(x, *lohi(w), w.wavelet_id, O.PERIODIC, J, 0)
    for mask, az in [(0b111000000, False), (0b011110000, True), (0b000001111, False)]:
        y = engine.inverse(d, a, *lohi_r(w), w.wavelet_id, O.PERIODIC, J, 0, detail_mask=mask, approx_zero=az)
        for b in range(2):
            y_ref = O.reconstruct(d[:, b, :], a[b], *lohi_r(w), O.PERIODIC, detail_mask=mask, approx_zero=az)
            assert np.array_equal(y[b], y_ref), (mask, az, b)


def test_deep_denoise_thresholds(engine):
    """SWT universal-threshold denoise on long signals: the per-signal threshold is applied on the detail
    loads of the deep inverse as in the fused kernels (MutableMultiLevelMODWTResult.java:97-114)."""
    w = Symlet.SYM8
    n, J = 1 << 15, 8
    x = _rows(2, n, 29)
    y, thr = vw.VectorWaveSwtAdapter(w, vw.BoundaryMode.PERIODIC).denoise(x, J, return_thresholds=True)
    for b in range(2):
        y_ref, t_ref = O.swt_denoise(x[b], *lohi(w), O.PERIODIC, J, wavelet_id=w.wavelet_id)
        assert thr[b] == t_ref
        assert np.array_equal(y[b], y_ref)

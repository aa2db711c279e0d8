"""Chained inverse column sweeps (vw_device.h k_inverse_sweep2 / k_inverse_sweep3): two or three deep
PERIODIC inverse levels in one launch, the intermediate approximations handed from one level's column
sweep to the next through LDS rings (VW_SWEEP2 = 2: pairs only, 3: triples where they qualify).
EXACT: bit-exact against the restatement of vectorwave-core (MultiLevelMODWTTransform.java:339-349,
:576-589); FMA and fp32: identical bits to one column sweep per level (VW_SWEEP2=0), since every output
is the same operation sequence.  Shapes cover triples, pairs of 64- and 32-residue groups, a lone sweep
level, N not a power of two (partial u-chunks), short and long filters (KA = 8 / 16), small chunks,
masked details, a zero approximation and the fused denoise thresholds."""
import numpy as np
import pytest

from oracle import oracle as O
import vectorwave_amd as vw
from vectorwave_amd import _native as nat
from vectorwave_amd.wavelets import Coiflet, Daubechies, Haar, Symlet

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def short_classes(engine):
    """The small shapes here have short residue classes, which the default policy leaves to one sweep per
    level (VW_SWEEP2_MINB = 64 blocks): admit them so the kernels' edge cases run at test sizes."""
    engine.set_option("VW_SWEEP2_MINB", 1)
    yield
    engine.set_option("VW_SWEEP2_MINB", -1)


def _rows(B, n, seed):
    return np.stack([O.java_random_signal(n, seed + b) for b in range(B)])


def lohi(w):
    return w.lowPassDecomposition(), w.highPassDecomposition()


def lohi_r(w):
    return w.lowPassReconstruction(), w.highPassReconstruction()


@pytest.mark.parametrize("w,n,J,B", [(Daubechies.DB8, 1 << 15, 10, 2), (Haar.INSTANCE, 1 << 14, 12, 2),
                                     (Symlet.SYM8, 1 << 16, 9, 1), (Daubechies.DB4, 3 << 14, 10, 2),
                                     (Coiflet.COIF5, 1 << 17, 9, 1)],
                         ids=["db8-2^15-J10", "haar-2^14-J12", "sym8-2^16-J9", "db4-3x2^14-J10", "coif5-2^17-J9"])
def test_pair_inverse_bit_exact(engine, w, n, J, B):
    x = _rows(B, n, 7)
    d, a = engine.forward(x, *lohi(w), w.wavelet_id, O.PERIODIC, J, 0)        # BatchMODWT semantics (no cap)
    for g in (3, 2):
        with engine.options(VW_SWEEP2=g):
            y = engine.inverse(d, a, *lohi_r(w), w.wavelet_id, O.PERIODIC, J, 0)
        for b in range(B):
            y_ref = O.reconstruct(d[:, b, :], a[b], *lohi_r(w), O.PERIODIC)
            assert np.array_equal(y[b], y_ref), (g, b)


@pytest.mark.parametrize("opts", [{"VW_SWEEP2": 3}, {"VW_SWEEP2": 2}, {"VW_SWEEP2": 3, "VW_SWEEP2_KA": 16},
                                  {"VW_SWEEP2": 3, "VW_SWEEP2_UC": 32}, {"VW_SWEEP2": 2, "VW_SWEEP2_UC": 4096}],
                         ids=["triple", "pair", "ka16", "uc32", "pair-uc4096"])
@pytest.mark.parametrize("w,n,J,dt", [(Daubechies.DB8, 1 << 16, 10, "f64"), (Coiflet.COIF5, 1 << 16, 9, "f32"),
                                      (Daubechies.DB4, 3 << 15, 11, "f32"), (Haar.INSTANCE, 1 << 15, 13, "f64")])
def test_pair_matches_single_sweeps(engine, opts, w, n, J, dt):
    import torch
    tdt = torch.float64 if dt == "f64" else torch.float32
    x = torch.empty((3, n), dtype=tdt, device="cuda")
    engine.fill_uniform(x, 11)
    for flags in (0, nat.FLAG_FMA):
        d, a = engine.forward(x, *lohi(w), w.wavelet_id, O.PERIODIC, J, flags)
        with engine.options(**opts):
            y1 = engine.inverse(d, a, *lohi_r(w), w.wavelet_id, O.PERIODIC, J, flags)
        with engine.options(VW_SWEEP2=0):
            y0 = engine.inverse(d, a, *lohi_r(w), w.wavelet_id, O.PERIODIC, J, flags)
        torch.cuda.synchronize()
        assert torch.equal(y1, y0), (w.name(), dt, flags, opts)


def test_pair_partial_reconstruction(engine):
    """reconstructFromLevel / reconstructLevels: masked details on either level of a pair and a zero
    approximation (MultiLevelMODWTTransform.java:361-446)."""
    w = Daubechies.DB8
    n, J = 1 << 15, 10
    x = _rows(2, n, 17)
    d, a = engine.forward(x, *lohi(w), w.wavelet_id, O.PERIODIC, J, 0)
    with engine.options(VW_SWEEP2=3):
        for mask, az in [(0b1000000000, False), (0b0110000000, True), (0b0101010101, False), (0, False)]:
            y = engine.inverse(d, a, *lohi_r(w), w.wavelet_id, O.PERIODIC, J, 0, detail_mask=mask, approx_zero=az)
            for b in range(2):
                y_ref = O.reconstruct(d[:, b, :], a[b], *lohi_r(w), O.PERIODIC, detail_mask=mask, approx_zero=az)
                assert np.array_equal(y[b], y_ref), (mask, az, b)


def test_pair_denoise_thresholds(engine):
    """SWT universal-threshold denoise on long signals: each level's per-signal threshold is applied on
    that level's detail loads inside the pair (MutableMultiLevelMODWTResult.java:97-114)."""
    w = Symlet.SYM8
    n, J = 1 << 16, 9
    x = _rows(2, n, 31)
    with engine.options(VW_SWEEP2=3):
        y, thr = vw.VectorWaveSwtAdapter(w, vw.BoundaryMode.PERIODIC).denoise(x, J, return_thresholds=True)
    for b in range(2):
        y_ref, t_ref = O.swt_denoise(x[b], *lohi(w), O.PERIODIC, J, wavelet_id=w.wavelet_id)
        assert thr[b] == t_ref
        assert np.array_equal(y[b], y_ref)


def test_default_policy_triple_on_long_blocks(engine):
    """The default policy (VW_SWEEP2_MINB = 64) on a 2^18-sample db8 block: levels (10,9,8) as a triple of
    64-residue groups, (7,6) as a pair of 32-residue groups; bit-exact against the restatement."""
    w = Daubechies.DB8
    n, J = 1 << 18, 10
    x = _rows(1, n, 3)
    d, a = engine.forward(x, *lohi(w), w.wavelet_id, O.PERIODIC, J, 0)
    with engine.options(VW_SWEEP2_MINB=-1):
        y = engine.inverse(d, a, *lohi_r(w), w.wavelet_id, O.PERIODIC, J, 0)
    assert np.array_equal(y[0], O.reconstruct(d[:, 0, :], a[0], *lohi_r(w), O.PERIODIC))

"""GPU parity of the headline configuration in the mode the bench reports.

BASELINE.json configs[1]: db4, J = 6, 4096 x 4096 fp64, PERIODIC, forward + inverse, the default kernel
policy -- at B = 4096 > 2 signals per CU that is k_forward_persist (512 resident workgroups, each walking
8 signals with the next row arriving by LDS-DMA) and k_inverse_seq (vw_capi.cpp inverse_impl policy).
Rows are picked across the batch and across resident workgroups: b and b + 512 are walked by the same
persistent workgroup, b and b + 1 by neighbours on different CUs / XCDs.

Bars: FMA (the bench's accumulation) within 1e-12 of the restatement of vectorwave-core
(MultiLevelMODWTTransform.java:243-251 forward, :339-349 / :576-589 inverse) for details, approximation
and the reconstruction; EXACT bit-exact for forward AND inverse rows.
"""
import numpy as np
import pytest

from oracle import oracle as O
from vectorwave_amd import _native as nat
from vectorwave_amd.wavelets import Daubechies

pytestmark = pytest.mark.gpu

B, N, J = 4096, 4096, 6
ROWS = (0, 1, 255, 511, 512, 1023, 2047, 2048, 3071, 4094, 4095)
TOL = 1e-12   # north_star: fp64 max-abs error < 1e-12 vs vectorwave-core


@pytest.fixture(scope="module")
def headline(engine):
    import torch
    x = torch.empty((B, N), dtype=torch.float64, device="cuda")
    engine.fill_uniform(x, 42)   # the bench's input (bench.py Workload)
    torch.cuda.synchronize()
    return x


def _run(engine, x, flags):
    import torch
    w = Daubechies.DB4
    det, app = engine.forward(x, w.lowPassDecomposition(), w.highPassDecomposition(), w.wavelet_id, O.PERIODIC, J,
                              flags)
    y = engine.inverse(det, app, w.lowPassReconstruction(), w.highPassReconstruction(), w.wavelet_id, O.PERIODIC, J,
                       flags)
    torch.cuda.synchronize()
    return det, app, y


def _oracle(xrow):
    w = Daubechies.DB4
    d, a = O.decompose(xrow, w.lowPassDecomposition(), w.highPassDecomposition(), O.PERIODIC, J)
    y = O.reconstruct(d, a, w.lowPassReconstruction(), w.highPassReconstruction(), O.PERIODIC, w.wavelet_id)
    return d, a, y


def test_headline_fma_rows_within_1e12(engine, headline):
    det, app, y = _run(engine, headline, nat.FLAG_FMA)
    w = Daubechies.DB4
    worst = 0.0
    for b in ROWS:
        xr = headline[b].cpu().numpy()
        d_ref, a_ref, y_ref = _oracle(xr)
        gd, ga, gy = det[:, b, :].cpu().numpy(), app[b].cpu().numpy(), y[b].cpu().numpy()
        np.testing.assert_allclose(gd, d_ref, rtol=0, atol=TOL)
        np.testing.assert_allclose(ga, a_ref, rtol=0, atol=TOL)
        np.testing.assert_allclose(gy, y_ref, rtol=0, atol=TOL)
        # the inverse alone, on the kernel's own FMA coefficients
        y_own = O.reconstruct(gd, ga, w.lowPassReconstruction(), w.highPassReconstruction(), O.PERIODIC)
        np.testing.assert_allclose(gy, y_own, rtol=0, atol=TOL)
        worst = max(worst, float(np.max(np.abs(gy - y_ref))), float(np.max(np.abs(gd - d_ref))))
    assert worst < TOL
    # whole batch: perfect reconstruction of the truncated db4 taps (SURVEY.md key fact 5)
    assert (y - headline).abs().max().item() < 1e-9


def test_headline_exact_rows_bit_exact(engine, headline):
    det, app, y = _run(engine, headline, 0)
    for b in ROWS:
        d_ref, a_ref, y_ref = _oracle(headline[b].cpu().numpy())
        assert np.array_equal(det[:, b, :].cpu().numpy(), d_ref), f"forward row {b}"
        assert np.array_equal(app[b].cpu().numpy(), a_ref), f"approx row {b}"
        assert np.array_equal(y[b].cpu().numpy(), y_ref), f"inverse row {b}"


def test_headline_fma_batch_checksum(engine, headline):
    """A size-independent property over all 4096 rows: the reconstruction of the FMA chain equals the
    EXACT chain's within 1e-12 everywhere (both paths are checked row-wise against the oracle above)."""
    _, _, y_f = _run(engine, headline, nat.FLAG_FMA)
    _, _, y_e = _run(engine, headline, 0)
    assert (y_f - y_e).abs().max().item() < TOL

"""Matrix-core fp32 kernels (vectorwave_amd/csrc/vw_mfma.hip, VW_MFMA): the FMA path's PERIODIC convolutions as
Toeplitz products on v_mfma_f32_16x16x4_f32.

Each output is accumulated tap by tap in the reference's order with one rounding per tap (the B operand is
read so that k ascends with the tap index), i.e. the VALU FMA kernels' sums: the test asks for the same bits
as VW_MFMA=0 and, independently, the fp32 bar of the FMA path against the fp64 restatement,
1e-5 * max|x| * J (the reference has no fp32 path).  Reference loops restated:
BatchSIMDMODWT.java:384-424 (forward), MultiLevelMODWTTransform.java:576-589 (K4 inverse).
"""
import numpy as np
import pytest

from oracle import oracle as O
import vectorwave_amd as vw
from vectorwave_amd import _native as nat

pytestmark = pytest.mark.gpu


def lohi(w):
    return w.lowPassDecomposition(), w.highPassDecomposition()


def run(engine, x, w, J, mfma, mask=0xFFFFFFFF, approx_zero=False):
    with engine.options(VW_MFMA=mfma):
        d, a = engine.forward(x, *lohi(w), w.wavelet_id, O.PERIODIC, J, nat.FLAG_FMA)
        y = engine.inverse(d, a, w.lowPassReconstruction(), w.highPassReconstruction(), w.wavelet_id, O.PERIODIC, J,
                           nat.FLAG_FMA, detail_mask=mask, approx_zero=approx_zero)
    import torch
    torch.cuda.synchronize()
    return d.cpu().numpy(), a.cpu().numpy(), y.cpu().numpy()


@pytest.mark.parametrize("case", [("coif5", 8192, 6, 5), ("coif5", 4096, 5, 3), ("coif5", 2048, 3, 9),
                                  ("db8", 8192, 8, 3), ("sym8", 2048, 7, 4)],
                         ids=lambda c: f"{c[0]}-{c[1]}-J{c[2]}")
def test_mfma_matches_valu_fma_and_the_restatement(engine, case):
    import torch
    wname, n, J, B = case
    w = vw.get_wavelet(wname)
    x = torch.from_numpy(O.fill_uniform(B * n, 17).reshape(B, n)).float().cuda()
    d0, a0, y0 = run(engine, x, w, J, 0)
    d1, a1, y1 = run(engine, x, w, J, 3)
    tol = 1e-5 * float(x.abs().max()) * J
    for name, p, q in (("details", d0, d1), ("approx", a0, a1), ("y", y0, y1)):
        assert np.max(np.abs(p - q)) <= tol, name
    assert np.array_equal(d0, d1) and np.array_equal(a0, a1), "forward: not the VALU FMA kernels' bits"
    assert np.array_equal(y0, y1), "inverse: not the VALU FMA kernels' bits"
    xh = x.double().cpu().numpy()
    for b in (0, B - 1):
        d_ref, a_ref = O.decompose(xh[b], *lohi(w), O.PERIODIC, J, core=False)
        assert np.max(np.abs(d1[:, b, :] - d_ref)) <= tol and np.max(np.abs(a1[b] - a_ref)) <= tol
        y_ref = O.reconstruct(d_ref, a_ref, w.lowPassReconstruction(), w.highPassReconstruction(), O.PERIODIC)
        assert np.max(np.abs(y1[b] - y_ref)) <= tol


def test_mfma_inverse_masks(engine):
    # reconstructFromLevel / reconstructLevels shapes: masked details, zero approximation
    import torch
    w, n, J, B = vw.Coiflet.COIF5, 8192, 6, 3
    x = torch.from_numpy(O.fill_uniform(B * n, 5).reshape(B, n)).float().cuda()
    for mask, az in ((0b111100, False), (0b000011, True), (0, False)):
        _, _, y0 = run(engine, x, w, J, 0, mask, az)
        _, _, y1 = run(engine, x, w, J, 3, mask, az)
        assert np.array_equal(y0, y1), (mask, az)


def test_mfma_config5_batch_rows(engine):
    # the coif5 J=6 8192-sample rows of config 5 through the default policy's switch, a batch of 64
    import torch
    w, n, J, B = vw.Coiflet.COIF5, 8192, 6, 64
    x = torch.empty((B, n), dtype=torch.float32, device="cuda")
    engine.fill_uniform(x, 42)
    d1, a1, y1 = run(engine, x, w, J, 3)
    xh = x.double().cpu().numpy()
    tol = 1e-5 * float(np.abs(xh).max()) * J
    for b in (0, 31, 63):
        d_ref, a_ref = O.decompose(xh[b], *lohi(w), O.PERIODIC, J, core=False)
        assert np.max(np.abs(d1[:, b, :] - d_ref)) <= tol and np.max(np.abs(a1[b] - a_ref)) <= tol
    assert np.max(np.abs(y1 - xh)) <= 1e-3  # perfect reconstruction within fp32 / coif5's truncated taps

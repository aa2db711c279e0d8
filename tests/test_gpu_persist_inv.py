"""Persistent two-region inverse (vw_device.h k_inverse_persist, VW_INV_PERSIST=1): rows by LDS-DMA with
their periodic right halo, the resident grid walking the batch, next signal's a_J / d_J loaded during
level 1.  Per output it runs the same operation sequence as k_inverse_seq (approximation taps, then
detail taps, l ascending -- MultiLevelMODWTTransform.java:576-589), so:
  * EXACT: bit-exact against the restatement of vectorwave-core on sampled rows;
  * EXACT, FMA and fp32: every row bit-identical to the one-signal-per-workgroup kernel (VW_INV_PERSIST=0)
    on the same coefficients -- batches below, at and above the resident grid (2 workgroups per CU),
    so rows b and b + grid share a persistent workgroup.
"""
import numpy as np
import pytest

from oracle import oracle as O
from vectorwave_amd import _native as nat
from vectorwave_amd.wavelets import Daubechies, Haar

pytestmark = pytest.mark.gpu


def _inverse(engine, torch, det, app, w, J, flags, persist, nv2=False):
    from ctypes import c_void_p
    P = lambda t: c_void_p(t.data_ptr())  # noqa: E731
    f32 = det.dtype == torch.float32
    _, B, N = det.shape
    y = torch.empty((B, N), dtype=det.dtype, device="cuda")
    lo, hi = w.lowPassReconstruction(), w.highPassReconstruction()
    engine.set_option("VW_INV_PERSIST", 1 if persist else 0)
    engine.set_option("VW_INV_NV", 2 if nv2 else -1)
    try:
        fn = engine.lib.vw_modwt_inverse_f32 if f32 else engine.lib.vw_modwt_inverse_f64
        st = fn(engine.ctx, P(det), P(app), B, N, nat.taps_array(lo), nat.taps_array(hi), len(lo), w.wavelet_id,
                nat.PERIODIC, J, 0xFFFFFFFF, 0, flags, P(y))
        assert st == 0, nat.last_error()
    finally:
        engine.set_option("VW_INV_PERSIST", -1)
        engine.set_option("VW_INV_NV", -1)
    torch.cuda.synchronize()
    return y


def _coeffs(engine, torch, w, B, N, J, dtype, seed=42):
    from ctypes import c_void_p
    P = lambda t: c_void_p(t.data_ptr())  # noqa: E731
    x = torch.empty((B, N), dtype=dtype, device="cuda")
    engine.fill_uniform(x, seed)
    det = torch.empty((J, B, N), dtype=dtype, device="cuda")
    app = torch.empty((B, N), dtype=dtype, device="cuda")
    lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
    fn = engine.lib.vw_modwt_forward_f32 if dtype == torch.float32 else engine.lib.vw_modwt_forward_f64
    engine.bind_torch_stream()
    assert fn(engine.ctx, P(x), B, N, N, nat.taps_array(lo), nat.taps_array(hi), len(lo), w.wavelet_id, nat.PERIODIC,
              J, 0, P(det), P(app)) == 0, nat.last_error()
    torch.cuda.synchronize()
    return x, det, app


CASES = [  # wavelet, B, N, J: below / at / above the resident grid (512 on 256 CUs), short and long rows
    (Daubechies.DB4, 4096, 4096, 6),   # the headline shape: 8 signals per workgroup
    (Daubechies.DB4, 1300, 4096, 6),   # uneven walk
    (Daubechies.DB4, 512, 4096, 6),    # one signal per workgroup (the 8-GPU shard)
    (Daubechies.DB4, 3, 1024, 7),
    (Haar.INSTANCE, 700, 512, 8),
    (Daubechies.DB2, 600, 2048, 4),
    (Daubechies.DB4, 37, 512, 4),      # the smallest row of whole-wave slabs; halo rounded to 64 vectors
]


@pytest.mark.parametrize("w,B,N,J", CASES, ids=[f"{c[0].name()}-B{c[1]}-N{c[2]}-J{c[3]}" for c in CASES])
@pytest.mark.parametrize("flags", [0, nat.FLAG_FMA], ids=["exact", "fma"])
def test_persist_inverse_identical_to_per_signal_kernel(engine, w, B, N, J, flags):
    import torch
    x, det, app = _coeffs(engine, torch, w, B, N, J, torch.float64)
    y_ref = _inverse(engine, torch, det, app, w, J, flags, persist=False)
    y = _inverse(engine, torch, det, app, w, J, flags, persist=True)
    assert torch.equal(y, y_ref), float((y - y_ref).abs().max())
    if B * N >= 1 << 20:   # NV = 2 form (1024-thread workgroups) on the larger shapes
        y2 = _inverse(engine, torch, det, app, w, J, flags, persist=True, nv2=True)
        assert torch.equal(y2, y_ref), float((y2 - y_ref).abs().max())
    if flags == 0:   # EXACT: the restatement of vectorwave-core, rows across persistent workgroups
        dh, ah, yh = det.cpu().numpy(), app.cpu().numpy(), y.cpu().numpy()
        for b in sorted({0, B - 1, min(B - 1, 512), min(B - 1, 1024 + 3)}):
            yr = O.reconstruct(dh[:, b, :], ah[b], w.lowPassReconstruction(), w.highPassReconstruction(), O.PERIODIC)
            assert np.array_equal(yh[b], yr), b
        assert float((y - x).abs().max()) < 1e-8   # perfect reconstruction (truncated published taps)


def test_persist_inverse_f32(engine):
    import torch
    w = Daubechies.DB4
    B, N, J = 900, 8192, 6
    _, det, app = _coeffs(engine, torch, w, B, N, J, torch.float32)
    for flags in (0, nat.FLAG_FMA):
        y_ref = _inverse(engine, torch, det, app, w, J, flags, persist=False)
        y = _inverse(engine, torch, det, app, w, J, flags, persist=True)
        assert torch.equal(y, y_ref), float((y - y_ref).abs().max())


def test_persist_declines_outside_its_contract(engine):
    # SYMMETRIC, masked details and thresholds keep the per-signal kernels; results unchanged
    import torch
    from ctypes import c_void_p
    w = Daubechies.DB4
    B, N, J = 64, 1024, 4
    _, det, app = _coeffs(engine, torch, w, B, N, J, torch.float64)
    P = lambda t: c_void_p(t.data_ptr())  # noqa: E731
    lo, hi = w.lowPassReconstruction(), w.highPassReconstruction()
    outs = []
    for persist in (0, 1):
        engine.set_option("VW_INV_PERSIST", persist)
        y = torch.empty((B, N), dtype=torch.float64, device="cuda")
        assert engine.lib.vw_modwt_inverse_f64(engine.ctx, P(det), P(app), B, N, nat.taps_array(lo),
                                               nat.taps_array(hi), len(lo), w.wavelet_id, nat.PERIODIC, J, 0b1010, 0,
                                               0, P(y)) == 0
        outs.append(y)
    engine.set_option("VW_INV_PERSIST", -1)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("B", [4096, 700, 512])
def test_persistent_forward_register_prefetch_identical(engine, B):
    """k_forward_persist with the next row prefetched into registers from level 1 (VW_FWD_PF=1) instead of
    DMA'd during level J: the same outputs bit for bit (EXACT and FMA), every row."""
    import torch
    from ctypes import c_void_p
    w = Daubechies.DB4
    N, J = 4096, 6
    P = lambda t: c_void_p(t.data_ptr())  # noqa: E731
    x = torch.empty((B, N), dtype=torch.float64, device="cuda")
    engine.fill_uniform(x, 3)
    lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
    engine.bind_torch_stream()
    for flags in (0, nat.FLAG_FMA):
        outs = []
        for pf in (0, 1):
            det = torch.empty((J, B, N), dtype=torch.float64, device="cuda")
            app = torch.empty((B, N), dtype=torch.float64, device="cuda")
            with engine.options(VW_FWD_PF=pf):
                assert engine.lib.vw_modwt_forward_f64(engine.ctx, P(x), B, N, N, nat.taps_array(lo),
                                                       nat.taps_array(hi), len(lo), w.wavelet_id, nat.PERIODIC, J,
                                                       flags, P(det), P(app)) == 0, nat.last_error()
            outs.append((det, app))
        torch.cuda.synchronize()
        assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    if B == 700:   # EXACT rows across persistent workgroups against the restatement
        d, a = outs[0]
        for b in (0, 699):
            d_ref, a_ref = O.decompose(x[b].cpu().numpy(), lo, hi, O.PERIODIC, J, core=False)
            assert np.abs(d[:, b].cpu().numpy() - d_ref).max() <= 1e-12

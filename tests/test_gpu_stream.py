"""Streaming multi-level forward (vw_device.h k_forward_stream, VW_FWD_STREAM=1): levels of a long
PERIODIC signal streamed in chunks, each level's input history in an LDS ring, a warm-up of the group's
reach before every segment.  Per output it runs the reference's tap order with both filters from one read
(ScalarOps.java:700-723), like every other forward kernel, so:
  * EXACT: bit-exact against the restatement of vectorwave-core;
  * EXACT / FMA / fp32: every level and the approximation bit-identical to the default per-level path
    (multi-level tiles + streaming deep levels) on the same input.
Shapes: one and several segments per signal (batches below the CU count split signals), groups cut by
the LDS budget (the remaining levels run on the per-level path), short and long filters."""
import numpy as np
import pytest

from oracle import oracle as O
import vectorwave_amd as vw
from vectorwave_amd.wavelets import Coiflet, Daubechies, Haar, Symlet

pytestmark = pytest.mark.gpu


def _run(engine, torch, w, x, J, fma, stream):
    with engine.options(VW_FWD_STREAM=1 if stream else 0):
        m = vw.BatchMODWT.multiLevelAoS(w, x, J, fma=fma)
    torch.cuda.synchronize()
    return m.detailPerLevel, m.finalApprox


CASES = [  # wavelet, B, N, J
    (Daubechies.DB8, 2, 1 << 20, 10),   # config 4's block: levels 1-8 streamed, 9-10 deep
    (Daubechies.DB8, 3, 1 << 18, 10),   # several segments per signal (3 signals << 256 CUs)
    (Daubechies.DB4, 5, 1 << 16, 9),
    (Haar.INSTANCE, 1, 1 << 15, 12),
    (Symlet.SYM8, 2, 1 << 17, 8),
    (Coiflet.COIF5, 1, 1 << 17, 6),     # L = 30: the LDS budget cuts the group
]


@pytest.mark.parametrize("w,B,N,J", CASES, ids=[f"{c[0].name()}-B{c[1]}-N{c[2]}-J{c[3]}" for c in CASES])
@pytest.mark.parametrize("fma", [False, True], ids=["exact", "fma"])
def test_stream_identical_to_per_level_path(engine, w, B, N, J, fma):
    import torch
    x = torch.empty((B, N), dtype=torch.float64, device="cuda")
    engine.fill_uniform(x, 11)
    d0, a0 = _run(engine, torch, w, x, J, fma, stream=False)
    d1, a1 = _run(engine, torch, w, x, J, fma, stream=True)
    for j in range(J):
        assert torch.equal(d0[j], d1[j]), (j + 1, float((d0[j] - d1[j]).abs().max()))
    assert torch.equal(a0, a1)
    if not fma and N <= 1 << 18:   # EXACT: the restatement of vectorwave-core, last signal
        lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
        d_ref, a_ref = O.decompose(x[B - 1].cpu().numpy(), lo, hi, O.PERIODIC, J, core=False)
        assert np.array_equal(d1[:, B - 1].cpu().numpy(), d_ref)
        assert np.array_equal(a1[B - 1].cpu().numpy(), a_ref)


def test_stream_f32(engine):
    import torch
    w = Daubechies.DB8
    x = torch.empty((4, 1 << 18), dtype=torch.float32, device="cuda")
    engine.fill_uniform(x, 5)
    for fma in (False, True):
        d0, a0 = _run(engine, torch, w, x, 10, fma, stream=False)
        d1, a1 = _run(engine, torch, w, x, 10, fma, stream=True)
        assert torch.equal(d0, d1) and torch.equal(a0, a1)


# ---- streaming inverse (vw_device.h k_inverse_stream, VW_INV_STREAM = 512 | 1024 threads): the finest
# levels streamed right to left, approximation and detail rings per level.  Per output the K4 order
# (approximation taps, then detail taps, t + l ascending; MultiLevelMODWTTransform.java:576-589), so every
# output is bit-identical to the per-level path (multi-level tiles + chained sweeps) and, in EXACT mode,
# to the restatement of vectorwave-core.
INV_CASES = [  # wavelet, B, N, J
    (Daubechies.DB8, 2, 1 << 20, 10),   # config 4's block
    (Daubechies.DB8, 3, 1 << 18, 10),   # several segments per signal
    (Daubechies.DB4, 5, 1 << 16, 9),
    (Haar.INSTANCE, 1, 1 << 15, 12),
    (Symlet.SYM8, 2, 1 << 17, 8),
    (Coiflet.COIF5, 1, 1 << 17, 6),
]


@pytest.mark.parametrize("threads", [512, 1024])
@pytest.mark.parametrize("w,B,N,J", INV_CASES, ids=[f"{c[0].name()}-B{c[1]}-N{c[2]}-J{c[3]}" for c in INV_CASES])
@pytest.mark.parametrize("fma", [False, True], ids=["exact", "fma"])
def test_inverse_stream_identical_to_per_level_path(engine, w, B, N, J, fma, threads):
    import torch
    x = torch.empty((B, N), dtype=torch.float64, device="cuda")
    engine.fill_uniform(x, 13)
    m = vw.BatchMODWT.multiLevelAoS(w, x, J, fma=fma)
    y0 = vw.BatchMODWT.inverseMultiLevelAoS(w, m.detailPerLevel, m.finalApprox, fma=fma)
    with engine.options(VW_INV_STREAM=threads):
        y1 = vw.BatchMODWT.inverseMultiLevelAoS(w, m.detailPerLevel, m.finalApprox, fma=fma)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1), float((y0 - y1).abs().max())
    if not fma and N <= 1 << 18:
        d = m.detailPerLevel[:, B - 1].cpu().numpy()
        a = m.finalApprox[B - 1].cpu().numpy()
        y_ref = O.reconstruct(d, a, w.lowPassReconstruction(), w.highPassReconstruction(), O.PERIODIC, w.wavelet_id)
        assert np.array_equal(y1[B - 1].cpu().numpy(), y_ref)


def test_inverse_stream_f32(engine):
    import torch
    w = Daubechies.DB8
    x = torch.empty((4, 1 << 18), dtype=torch.float32, device="cuda")
    engine.fill_uniform(x, 5)
    for fma in (False, True):
        m = vw.BatchMODWT.multiLevelAoS(w, x, 10, fma=fma)
        y0 = vw.BatchMODWT.inverseMultiLevelAoS(w, m.detailPerLevel, m.finalApprox, fma=fma)
        with engine.options(VW_INV_STREAM=512):
            y1 = vw.BatchMODWT.inverseMultiLevelAoS(w, m.detailPerLevel, m.finalApprox, fma=fma)
        torch.cuda.synchronize()
        assert torch.equal(y0, y1)

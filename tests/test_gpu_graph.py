"""Captured steps (vw_capture_begin / vw_capture_end / vw_graph_launch) and dtype safety of the
device entry points.  A recorded graph replays exactly the calls it recorded: outputs are
bit-identical to direct calls; calls that must synchronize are refused while capturing."""
import numpy as np
import pytest

from oracle import oracle as O
import vectorwave_amd as vw
from vectorwave_amd import _native as nat
from vectorwave_amd.errors import InvalidStateException
from vectorwave_amd.wavelets import Daubechies, Symlet

pytestmark = pytest.mark.gpu


def _bufs(torch, B, N, J, dt=None):
    dt = dt or torch.float64
    x = torch.empty((B, N), dtype=dt, device="cuda")
    return x, torch.empty((J, B, N), dtype=dt, device="cuda"), torch.empty((B, N), dtype=dt, device="cuda"), \
        torch.empty((B, N), dtype=dt, device="cuda")


@pytest.mark.parametrize("w,B,N,J", [(Daubechies.DB4, 64, 4096, 6), (Daubechies.DB8, 2, 1 << 16, 8)],
                         ids=["fused", "multilevel-tiles"])
def test_graph_replay_bit_identical(engine, w, B, N, J):
    import torch
    from ctypes import c_void_p
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        x, det, app, y = _bufs(torch, B, N, J)
        engine.fill_uniform(x, 42)
        lo, hi = nat.taps_array(w.lowPassDecomposition()), nat.taps_array(w.highPassDecomposition())
        lib, ctx = engine.lib, engine.ctx
        P = lambda t: c_void_p(t.data_ptr())  # noqa: E731

        def step():
            assert lib.vw_modwt_forward_f64(ctx, P(x), B, N, N, lo, hi, len(lo), w.wavelet_id, 0, J, 0,
                                            P(det), P(app)) == 0
            assert lib.vw_modwt_inverse_f64(ctx, P(det), P(app), B, N, lo, hi, len(lo), w.wavelet_id, 0, J,
                                            0xFFFFFFFF, 0, 0, P(y)) == 0

        step()
        torch.cuda.synchronize()
        d0, a0, y0 = det.clone(), app.clone(), y.clone()
        g = engine.capture(step)
        for t in (det, app, y):
            t.fill_(float("nan"))
        g.launch(3)
        torch.cuda.synchronize()
        assert torch.equal(det, d0) and torch.equal(app, a0) and torch.equal(y, y0)
        g.close()
    xh = x.cpu().numpy()
    d_ref, a_ref = O.decompose(xh[B - 1], w.lowPassDecomposition(), w.highPassDecomposition(), O.PERIODIC, J,
                               core=False)
    assert np.array_equal(d0[:, B - 1].cpu().numpy(), d_ref)
    assert np.array_equal(a0[B - 1].cpu().numpy(), a_ref)


def test_capture_refuses_synchronizing_calls(engine):
    import torch
    from ctypes import byref, c_void_p
    w = Daubechies.DB4
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        x, det, app, _ = _bufs(torch, 4, 512, 3)
        engine.bind_torch_stream()
        lo, hi = nat.taps_array(w.lowPassDecomposition()), nat.taps_array(w.highPassDecomposition())
        lib, ctx = engine.lib, engine.ctx
        assert lib.vw_capture_begin(ctx) == 0
        st = lib.vw_modwt_forward_f64(ctx, c_void_p(x.data_ptr()), 4, 512, 512, lo, hi, len(lo), w.wavelet_id, 0, 3,
                                      nat.FLAG_VALIDATE, c_void_p(det.data_ptr()), c_void_p(app.data_ptr()))
        assert st == 10  # VW_ERR_STATE
        # a host-memory (JNI-shaped) call is refused before it stages anything: the capture
        # stays valid and ends cleanly
        xh, dh, ah = np.zeros((4, 512)), np.empty((3, 4, 512)), np.empty((4, 512))
        for fn, args in ((lib.vw_modwt_forward_f64, (c_void_p(xh.ctypes.data), 4, 512, 512, lo, hi, len(lo),
                                                     w.wavelet_id, 0, 3, nat.FLAG_HOST_MEMORY,
                                                     c_void_p(dh.ctypes.data), c_void_p(ah.ctypes.data))),
                         (lib.vw_modwt_inverse_f64, (c_void_p(dh.ctypes.data), c_void_p(ah.ctypes.data), 4, 512,
                                                     lo, hi, len(lo), w.wavelet_id, 0, 3, 0xFFFFFFFF, 0,
                                                     nat.FLAG_HOST_MEMORY, c_void_p(xh.ctypes.data)))):
            assert fn(ctx, *args) == 10
            assert "captured" in nat.last_error()
        assert lib.vw_capture_begin(ctx) == 10  # already capturing
        g = c_void_p()
        assert lib.vw_capture_end(ctx, byref(g)) == 0
        assert lib.vw_graph_destroy(g) == 0
    # the null stream cannot be captured
    engine.bind_torch_stream()
    if torch.cuda.current_stream().cuda_stream == 0:
        with pytest.raises(InvalidStateException):
            engine.capture(lambda: None)


def test_f32_tensor_into_f64_only_entry_points(engine):
    # the f64-only entry points convert an f32 tensor instead of reading it as f64
    import torch
    w = Symlet.SYM8
    x64 = torch.from_numpy(O.fill_uniform(2 * 2048, 42).reshape(2, 2048)).cuda()
    x32 = x64.float()
    ref = x32.double()
    swt = vw.VectorWaveSwtAdapter(w, vw.BoundaryMode.PERIODIC)
    assert torch.equal(swt.denoise(x32, 4), swt.denoise(ref, 4))
    assert torch.equal(swt.estimateNoiseSigma(x32), swt.estimateNoiseSigma(ref))
    tx = vw.MODWTTransform(w, vw.BoundaryMode.PERIODIC)
    r32, r64 = tx.forward(x32[0]), tx.forward(ref[0])
    assert torch.equal(r32.approximationCoeffs(), r64.approximationCoeffs())
    # threshold_inplace on a non-contiguous view writes back in place
    c = torch.from_numpy(O.fill_uniform(4 * 64, 7).reshape(64, 4)).cuda().t()  # [4, 64], non-contiguous
    expect = c.clone().contiguous()
    thr = torch.full((4,), 0.3, dtype=torch.float64, device="cuda")
    engine.threshold_inplace(expect, thr, True)
    engine.threshold_inplace(c, thr, True)
    assert torch.equal(c, expect)


def test_timing_inside_captured_graph(engine):
    # launches recorded with timing enabled carry their own event nodes: one replay of a K-step graph
    # reports K launches per family with positive durations (bench.py's timed region)
    import torch
    from ctypes import c_void_p
    w = Daubechies.DB4
    B, N, J, K = 32, 4096, 6, 5
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        x, det, app, y = _bufs(torch, B, N, J)
        engine.fill_uniform(x, 1)
        lo, hi = nat.taps_array(w.lowPassDecomposition()), nat.taps_array(w.highPassDecomposition())
        lib, ctx = engine.lib, engine.ctx
        P = lambda t: c_void_p(t.data_ptr())  # noqa: E731

        def step():
            assert lib.vw_modwt_forward_f64(ctx, P(x), B, N, N, lo, hi, len(lo), w.wavelet_id, 0, J, nat.FLAG_FMA,
                                            P(det), P(app)) == 0
            assert lib.vw_modwt_inverse_f64(ctx, P(det), P(app), B, N, lo, hi, len(lo), w.wavelet_id, 0, J,
                                            0xFFFFFFFF, 0, nat.FLAG_FMA, P(y)) == 0

        step()
        engine.reset_timing()
        engine.enable_timing(True)
        g = engine.capture(lambda: [step() for _ in range(K)])
        g.launch(1)
        torch.cuda.synchronize()
        for fam in ("forward", "inverse"):
            ms, n = engine.kernel_time(fam)
            assert n == K and ms > 0, (fam, ms, n)
        engine.enable_timing(False)
        engine.reset_timing()
        g.close()
        assert float((y - x).abs().max()) < 1e-9


def test_capture_of_allocating_engine_calls_keeps_storage(engine):
    """Engine.forward inside capture() allocates its outputs; the Graph keeps them (and the
    contiguous copy of a strided input) alive, so replays never write into storage the caching
    allocator has handed to other tensors.  Graph.result holds fn()'s outputs, rewritten per replay."""
    import torch
    w = Daubechies.DB4
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        xs = torch.empty((8, 2 * 1024), dtype=torch.float64, device="cuda")
        engine.fill_uniform(xs, 3)
        x = xs[:, ::2]   # strided: _prep makes a contiguous copy inside the capture
        lohi = (w.lowPassDecomposition(), w.highPassDecomposition())
        d0, a0 = engine.forward(x, *lohi, w.wavelet_id, O.PERIODIC, 4, 0)
        g = engine.capture(lambda: engine.forward(x, *lohi, w.wavelet_id, O.PERIODIC, 4, 0))
        det, app = g.result
        # churn the allocator: new tensors of the same sizes, filled with a sentinel
        others = [torch.full_like(det, 7.0) for _ in range(4)] + [torch.full_like(app, 7.0) for _ in range(4)]
        det.fill_(float("nan"))
        g.launch(2)
        torch.cuda.synchronize()
        assert all(bool((o == 7.0).all()) for o in others), "a replay wrote into another tensor's storage"
        assert torch.equal(det, d0) and torch.equal(app, a0)
        g.close()


def test_capture_exception_destroys_partial_graph(engine):
    import torch
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        x = torch.zeros((2, 256), dtype=torch.float64, device="cuda")
        w = Daubechies.DB4

        def boom():
            engine.forward(x, w.lowPassDecomposition(), w.highPassDecomposition(), w.wavelet_id, O.PERIODIC, 2, 0)
            raise KeyError("inside capture")

        with pytest.raises(KeyError):
            engine.capture(boom)
        # the context is usable again (not left capturing)
        d, a = engine.forward(x, w.lowPassDecomposition(), w.highPassDecomposition(), w.wavelet_id, O.PERIODIC, 2, 0)
        torch.cuda.synchronize()
        assert bool((d == 0).all())


def test_graph_outliving_its_context(engine):
    """vw_ctx_destroy invalidates the context's live graphs; launching one then fails with
    VW_ERR_STATE and destroying it is safe (no use of the freed context)."""
    import torch
    from ctypes import byref, c_void_p
    lib = engine.lib
    ctx = c_void_p()
    assert lib.vw_ctx_create(0, byref(ctx)) == 0
    s = torch.cuda.Stream()
    assert lib.vw_ctx_set_stream(ctx, c_void_p(s.cuda_stream)) == 0
    x = torch.empty((4, 512), dtype=torch.float64, device="cuda")
    x.fill_(1.0)
    det = torch.empty((2, 4, 512), dtype=torch.float64, device="cuda")
    app = torch.empty((4, 512), dtype=torch.float64, device="cuda")
    w = Daubechies.DB4
    lo, hi = nat.taps_array(w.lowPassDecomposition()), nat.taps_array(w.highPassDecomposition())
    P = lambda t: c_void_p(t.data_ptr())  # noqa: E731
    torch.cuda.synchronize()
    assert lib.vw_capture_begin(ctx) == 0
    assert lib.vw_modwt_forward_f64(ctx, P(x), 4, 512, 512, lo, hi, 8, w.wavelet_id, 0, 2, 0, P(det), P(app)) == 0
    g = c_void_p()
    assert lib.vw_capture_end(ctx, byref(g)) == 0
    assert lib.vw_graph_launch(g, 2) == 0
    assert lib.vw_ctx_synchronize(ctx) == 0
    assert lib.vw_ctx_destroy(ctx) == 0
    assert lib.vw_graph_launch(g, 1) == 10   # VW_ERR_STATE
    assert lib.vw_graph_destroy(g) == 0


def test_graph_of_long_centered_median_goes_stale_when_scratch_grows(engine):
    # the centred median of rows longer than the register path (N > 16384) uses a
    # per-context scratch; growing it frees the old one, so a graph that recorded the old address must
    # refuse to replay (VW_ERR_STATE) instead of touching freed memory
    import torch
    from ctypes import c_void_p
    eng = vw.Engine(0)
    try:
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            eng.bind_torch_stream()
            lib, ctx = eng.lib, eng.ctx
            P = lambda t: c_void_p(t.data_ptr())  # noqa: E731
            x = torch.from_numpy(O.fill_uniform(20000, 42).reshape(1, 20000)).cuda()
            cen = torch.zeros(1, dtype=torch.float64, device="cuda")
            out = torch.empty(1, dtype=torch.float64, device="cuda")

            def med():
                assert lib.vw_median_f64(ctx, P(x), 1, 20000, P(cen), 0, P(out)) == 0, nat.last_error()
            med()   # sizes the scratch outside the capture
            torch.cuda.synchronize()
            ref = float(np.median(np.abs(x.cpu().numpy())))
            assert out.item() == ref
            g = eng.capture(med)
            g.launch(1)
            torch.cuda.synchronize()
            assert out.item() == ref
            big = torch.from_numpy(O.fill_uniform(3 * 40000, 7).reshape(3, 40000)).cuda()
            cb = torch.zeros(3, dtype=torch.float64, device="cuda")
            ob = torch.empty(3, dtype=torch.float64, device="cuda")
            assert lib.vw_median_f64(ctx, P(big), 3, 40000, P(cb), 0, P(ob)) == 0, nat.last_error()
            torch.cuda.synchronize()
            assert np.array_equal(ob.cpu().numpy(), np.median(np.abs(big.cpu().numpy()), axis=1))
            assert lib.vw_graph_launch(g.handle, 1) == 10   # VW_ERR_STATE: the scratch moved
            g.close()
    finally:
        eng.close()

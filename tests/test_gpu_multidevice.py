"""In-process multi-context execution and the C ABI's thread-safety contract.

The reference's transforms are thread-safe (ConcurrentHashMap filter caches,
core/modwt/MultiLevelMODWTTransform.java:137-138) and are exercised concurrently by
vectorwave-extensions/src/test/java/com/morphiqlabs/wavelet/parallel/ConcurrentExecutionIntegrationTest.java.
Here: one batch split over several contexts (std::thread per context inside
vw_modwt_forward_multi_f64), several host threads on one context, and one Python thread per context
on device tensors.  A one-GPU box maps every context onto cuda:0.
"""
import threading

import numpy as np
import pytest

from oracle import oracle as O
import vectorwave_amd as vw
from vectorwave_amd import _native as nat
from vectorwave_amd.wavelets import Daubechies, Symlet

pytestmark = pytest.mark.gpu


def _rows(B, n, seed):
    return np.stack([O.java_random_signal(n, seed + b) for b in range(B)])


@pytest.mark.parametrize("nctx,B", [(2, 37), (3, 3), (4, 2), (2, 1)])
def test_sharded_batch_two_contexts_bit_exact(engine, nctx, B):
    w = Daubechies.DB4
    n, J = 1024, 5
    x = _rows(B, n, 11)
    with vw.DeviceGroup([0] * nctx) as g:
        det, app = g.forward(x, w, J)
        y = g.inverse(det, app, w)
        assert len(g.blocks(B)) == min(nctx, B)
    for b in range(B):
        d_ref, a_ref = O.decompose(x[b], w.lowPassDecomposition(), w.highPassDecomposition(), O.PERIODIC, J,
                                   core=False)
        assert np.array_equal(det[:, b, :], d_ref), b
        assert np.array_equal(app[b], a_ref), b
        y_ref = O.reconstruct(d_ref, a_ref, w.lowPassReconstruction(), w.highPassReconstruction(), O.PERIODIC)
        assert np.array_equal(y[b], y_ref), b
    # identical to the single-context call
    d1, a1 = engine.forward(x, w.lowPassDecomposition(), w.highPassDecomposition(), w.wavelet_id, O.PERIODIC, J, 0)
    assert np.array_equal(d1, det) and np.array_equal(a1, app)


def test_sharded_errors_name_the_block(engine):
    w = Daubechies.DB4
    x = _rows(4, 256, 3)
    x[3, 17] = np.nan
    lib = nat.load()
    with vw.DeviceGroup([0, 0]) as g:
        with pytest.raises(vw.InvalidSignalException) as ei:
            # validated (core) semantics: the bad row sits in block 1
            det = np.empty((2, 4, 256))
            app = np.empty((4, 256))
            from ctypes import c_void_p
            from vectorwave_amd.engine import _check
            _check(lib.vw_modwt_forward_multi_f64(g._ctxs, 2, x.ctypes.data_as(c_void_p), 4, 256, 256,
                                                  nat.taps_array(w.lowPassDecomposition()),
                                                  nat.taps_array(w.highPassDecomposition()), 8, w.wavelet_id,
                                                  O.PERIODIC, 2, nat.FLAG_HOST_MEMORY | nat.FLAG_VALIDATE,
                                                  det.ctypes.data_as(c_void_p), app.ctypes.data_as(c_void_p)))
        assert ei.value.index == 17
        msg = nat.last_error()
        # the block, its global rows, and the signal counted from row 0 of the whole batch
        assert "block 1 (rows 2..3)" in msg and "(signal 3)" in msg, msg
        # device memory is refused (each block must be staged through its own context)
        st = lib.vw_modwt_forward_multi_f64(g._ctxs, 2, x.ctypes.data_as(c_void_p), 4, 256, 256,
                                            nat.taps_array(w.lowPassDecomposition()),
                                            nat.taps_array(w.highPassDecomposition()), 8, w.wavelet_id, O.PERIODIC,
                                            2, 0, det.ctypes.data_as(c_void_p), app.ctypes.data_as(c_void_p))
        assert st == 7   # VW_ERR_ARG


def test_four_threads_hammer_one_context(engine):
    """ConcurrentExecutionIntegrationTest's pattern on one context: 4 host threads, each with its own
    host batch, forward + inverse 10 times through the host-memory path; every result bit-identical
    to the single-threaded one (calls are serialized by the context's mutex, staging reused)."""
    cases = [(Daubechies.DB4, 2048, 6), (Symlet.SYM8, 1000, 4), (Daubechies.DB8, 4096, 5), (Daubechies.DB4, 333, 3)]
    inputs = [_rows(5, n, 100 + k) for k, (_, n, _) in enumerate(cases)]
    expect = []
    for (w, n, J), x in zip(cases, inputs):
        d, a = engine.forward(x, w.lowPassDecomposition(), w.highPassDecomposition(), w.wavelet_id, O.PERIODIC, J, 0)
        y = engine.inverse(d, a, w.lowPassReconstruction(), w.highPassReconstruction(), w.wavelet_id, O.PERIODIC, J,
                           0)
        expect.append((d, a, y))
    errors = []

    def worker(k):
        try:
            w, n, J = cases[k]
            for _ in range(10):
                d, a = engine.forward(inputs[k], w.lowPassDecomposition(), w.highPassDecomposition(), w.wavelet_id,
                                      O.PERIODIC, J, 0)
                y = engine.inverse(d, a, w.lowPassReconstruction(), w.highPassReconstruction(), w.wavelet_id,
                                   O.PERIODIC, J, 0)
                e = expect[k]
                if not (np.array_equal(d, e[0]) and np.array_equal(a, e[1]) and np.array_equal(y, e[2])):
                    errors.append(f"thread {k}: result differs")
                    return
        except Exception as ex:  # pragma: no cover
            errors.append(f"thread {k}: {ex!r}")

    th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errors, errors


def test_device_tensors_one_thread_per_context(engine):
    """vw_modwt_forward/inverse_multi_dev_f64: each context works on its own device
    buffers (uneven shards, an empty one), no staging; bit-exact vs the restatement in EXACT mode and
    within 1e-12 with FMA; the inverse round trip too."""
    import torch
    w = Daubechies.DB4
    n, J = 4096, 6
    rows = [64, 37, 0]
    with vw.DeviceGroup([0, 0, 0]) as g:
        xs, off = [], 0
        for r in rows:
            x = torch.empty((r, n), dtype=torch.float64, device="cuda")
            if r:
                engine.fill_uniform(x, 42, offset=off * n)
            off += r
            xs.append(x)
        torch.cuda.synchronize()
        for fma in (False, True):
            outs = g.forward_device(xs, w, J, fma=fma)
            ys = g.inverse_device(outs, w, fma=fma)
            for k, ((d, a), y) in enumerate(zip(outs, ys)):
                assert d.shape == (J, rows[k], n) and y.shape == (rows[k], n)
                for b in ({0, rows[k] - 1} if rows[k] else ()):
                    xr = xs[k][b].cpu().numpy()
                    d_ref, a_ref = O.decompose(xr, w.lowPassDecomposition(), w.highPassDecomposition(), O.PERIODIC,
                                               J, core=False)
                    y_ref = O.reconstruct(d_ref, a_ref, w.lowPassReconstruction(), w.highPassReconstruction(),
                                          O.PERIODIC)
                    if fma:
                        assert np.abs(d[:, b].cpu().numpy() - d_ref).max() <= 1e-12
                        assert np.abs(y[b].cpu().numpy() - y_ref).max() <= 1e-12
                    else:
                        assert np.array_equal(d[:, b].cpu().numpy(), d_ref)
                        assert np.array_equal(a[b].cpu().numpy(), a_ref)
                        assert np.array_equal(y[b].cpu().numpy(), y_ref)
        # the device path refuses the host flag, and the host path still refuses device memory
        lib = nat.load()
        from ctypes import c_int64, c_void_p
        ptrs = (c_void_p * 3)(*[x.data_ptr() for x in xs])
        rr = (c_int64 * 3)(*rows)
        st = lib.vw_modwt_forward_multi_dev_f64(g._ctxs, 3, ptrs, rr, n, n, nat.taps_array(w.lowPassDecomposition()),
                                                nat.taps_array(w.highPassDecomposition()), 8, w.wavelet_id,
                                                O.PERIODIC, J, nat.FLAG_HOST_MEMORY, ptrs, ptrs)
        assert st == 7   # VW_ERR_ARG
        # inverse_device checks every shard before any launch: wrong dtype, mismatched rows,
        # a different N on one shard, a host tensor -- InvalidArgumentException, nothing enqueued
        from vectorwave_amd.errors import InvalidArgumentException
        good = g.forward_device(xs, w, J)
        bad_cases = [
            [(good[0][0].float(), good[0][1].float())] + good[1:],
            [(good[0][0], good[0][1][:-1])] + good[1:],
            good[:1] + [(good[1][0][..., :-8].contiguous(), good[1][1][..., :-8].contiguous())] + good[2:],
            good[:2] + [(good[2][0].cpu(), good[2][1].cpu())],
            [(good[0][0][0], good[0][1])] + good[1:],
        ]
        for parts in bad_cases:
            with pytest.raises(InvalidArgumentException):
                g.inverse_device(parts, w)

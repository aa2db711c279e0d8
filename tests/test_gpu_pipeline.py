"""Pipelined round trips (vw_pipeline_*, include/vectorwave_amd.h): step i = forward of buffer set i mod R
on one context's stream, then its inverse on another's, the steps issued by the engine from C++.  Every
set's outputs must equal the single-call results: the restatement bit for bit in EXACT mode, within
1e-12 with FMA (north_star), for every set and for f32 within the SURVEY.md §8d fp32 bar."""
from ctypes import byref, c_void_p

import numpy as np
import pytest

from oracle import oracle as O
import vectorwave_amd as vw
from vectorwave_amd import _native as nat
from vectorwave_amd.wavelets import Daubechies

pytestmark = pytest.mark.gpu


def _sets(torch, eng, R, B, N, J, dt):
    sets = []
    for r in range(R):
        x = torch.empty((B, N), dtype=dt, device="cuda")
        eng.fill_uniform(x, 100 + r)   # a different input per set: each step must use its own set
        sets.append({"x": x, "det": torch.full((J, B, N), float("nan"), dtype=dt, device="cuda"),
                     "app": torch.full((B, N), float("nan"), dtype=dt, device="cuda"),
                     "y": torch.full((B, N), float("nan"), dtype=dt, device="cuda")})
    return sets


def _create(lib, ef, ei, sets, esz, B, N, w, J, flags):
    R = len(sets)
    arr = lambda k: (c_void_p * R)(*[s[k].data_ptr() for s in sets])  # noqa: E731
    lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
    p = c_void_p()
    st = lib.vw_pipeline_create(ef.ctx, ei.ctx, esz, R, arr("x"), arr("det"), arr("app"), arr("y"), B, N,
                                nat.taps_array(lo), nat.taps_array(hi), len(lo), w.wavelet_id, nat.PERIODIC, J,
                                flags, byref(p))
    return st, p


@pytest.mark.parametrize("fma,f32", [(False, False), (True, False), (True, True)], ids=["exact", "fma", "f32"])
def test_pipeline_matches_restatement_every_set(engine, fma, f32):
    import torch
    w = Daubechies.DB4
    B, N, J, R = 48, 4096, 6, 3
    dt = torch.float32 if f32 else torch.float64
    ef, ei = vw.Engine(0), vw.Engine(0)
    sF, sI = torch.cuda.Stream(), torch.cuda.Stream()
    try:
        with torch.cuda.stream(sI):
            ei.bind_torch_stream()
        with torch.cuda.stream(sF):
            ef.bind_torch_stream()
            sets = _sets(torch, ef, R, B, N, J, dt)
        torch.cuda.synchronize()
        lib = ef.lib
        st, p = _create(lib, ef, ei, sets, 4 if f32 else 8, B, N, w, J, nat.FLAG_FMA if fma else 0)
        assert st == 0, nat.last_error()
        try:
            assert lib.vw_pipeline_last_set(p) == -1
            # 7 steps in two runs (the second run continues the set rotation), then a join
            assert lib.vw_pipeline_run(p, 4) == 0, nat.last_error()
            assert lib.vw_pipeline_run(p, 3) == 0, nat.last_error()
            assert lib.vw_pipeline_last_set(p) == 6 % R
            assert lib.vw_pipeline_join(p) == 0
            torch.cuda.synchronize()
        finally:
            assert lib.vw_pipeline_destroy(p) == 0
        lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
        for r, s in enumerate(sets):
            for b in (0, B - 1):
                xr = s["x"][b].double().cpu().numpy()
                d_ref, a_ref = O.decompose(xr, lo, hi, O.PERIODIC, J, core=False)
                y_ref = O.reconstruct(d_ref, a_ref, w.lowPassReconstruction(), w.highPassReconstruction(),
                                      O.PERIODIC)
                got = [(s["det"][:, b].double().cpu().numpy(), d_ref), (s["app"][b].double().cpu().numpy(), a_ref),
                       (s["y"][b].double().cpu().numpy(), y_ref)]
                for g, ref in got:
                    if f32:
                        np.testing.assert_allclose(g, ref, rtol=0, atol=1e-5 * float(np.abs(xr).max()) * J)
                    elif fma:
                        np.testing.assert_allclose(g, ref, rtol=0, atol=1e-12)
                    else:
                        assert np.array_equal(g, ref), f"set {r} row {b}"
    finally:
        ef.close()
        ei.close()


def test_pipeline_refuses_bad_arguments_and_dies_with_its_context(engine):
    import torch
    w = Daubechies.DB4
    B, N, J = 4, 512, 3
    ef, ei = vw.Engine(0), vw.Engine(0)
    try:
        sets = _sets(torch, engine, 2, B, N, J, torch.float64)
        torch.cuda.synchronize()
        lib = ef.lib
        for flags in (nat.FLAG_SYNC, nat.FLAG_HOST_MEMORY, nat.FLAG_VALIDATE):
            st, _ = _create(lib, ef, ei, sets, 8, B, N, w, J, flags)
            assert st == 7, flags   # VW_ERR_ARG
        st, _ = _create(lib, ef, ei, sets, 2, B, N, w, J, 0)
        assert st == 7
        st, p = _create(lib, ef, ei, sets, 8, B, N, w, J, 0)
        assert st == 0
        assert lib.vw_pipeline_run(p, 3) == 0
        assert lib.vw_pipeline_join(p) == 0
        ei.close()                               # destroying a context kills the pipeline
        assert lib.vw_pipeline_run(p, 1) == 10   # VW_ERR_STATE
        assert lib.vw_pipeline_join(p) == 10
        assert lib.vw_pipeline_destroy(p) == 0
    finally:
        ef.close()
        if ei.ctx:
            ei.close()

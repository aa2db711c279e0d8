"""Committed golden vectors (tests/golden/modwt_fixtures.npz, made by tests/golden/make_fixtures.py):
{haar, db4, db8, sym8, coif5} x {periodic, symmetric, zero} x N in {7, 64, 129, 512}, J <= 3, two
signals per case.

CPU: the restatement still reproduces every vector bit for bit (pins the oracle against drift).
GPU: the HIP engine, through the C-ABI, reproduces them bit for bit in EXACT mode (forward from x;
inverse from the fixture's coefficients) and within 1e-12 in FMA mode.
"""
import os

import numpy as np
import pytest

from vectorwave_amd import get_wavelet
from vectorwave_amd import _native as nat

PATH = os.path.join(os.path.dirname(__file__), "golden", "modwt_fixtures.npz")
BOUND = {"periodic": 0, "symmetric": 1, "zero": 2}  # VW_PERIODIC / VW_SYMMETRIC / VW_ZERO_PADDING


def _cases():
    with np.load(PATH, allow_pickle=False) as z:
        names = [str(c) for c in z["cases"]]
    return names


def _load(name):
    with np.load(PATH, allow_pickle=False) as z:
        return {k: z[f"{name}_{k}"] for k in ("x", "details", "approx", "y")}


def _parse(name):
    wn, bn, n, j = name.split("_")
    return get_wavelet(wn), BOUND[bn], int(n[1:]), int(j[1:])


CASES = _cases()


def test_fixture_matrix_complete():
    assert len(CASES) >= 40
    assert {c.split("_")[1] for c in CASES} == set(BOUND)


@pytest.mark.parametrize("name", CASES)
def test_oracle_reproduces_fixture(name):
    from oracle import oracle as O

    w, bc, n, J = _parse(name)
    f = _load(name)
    lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
    for b in range(f["x"].shape[0]):
        d, a = O.decompose(f["x"][b], lo, hi, bc, J)
        np.testing.assert_array_equal(d, f["details"][:, b, :])
        np.testing.assert_array_equal(a, f["approx"][b])
        np.testing.assert_array_equal(O.reconstruct(d, a, lo, hi, bc, w.wavelet_id), f["y"][b])


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_engine_matches_fixture(engine, name):
    w, bc, n, J = _parse(name)
    f = _load(name)
    lo, hi = w.lowPassDecomposition(), w.highPassDecomposition()
    det, app = engine.forward(f["x"], lo, hi, w.wavelet_id, bc, J, nat.FLAG_CORE_LEVELS)
    np.testing.assert_array_equal(det, f["details"])
    np.testing.assert_array_equal(app, f["approx"])
    y = engine.inverse(f["details"], f["approx"], lo, hi, w.wavelet_id, bc, J, nat.FLAG_CORE_LEVELS)
    np.testing.assert_array_equal(y, f["y"])
    # FMA accumulation: the north_star tolerance
    det2, app2 = engine.forward(f["x"], lo, hi, w.wavelet_id, bc, J, nat.FLAG_FMA)
    assert np.max(np.abs(det2 - f["details"])) < 1e-12
    assert np.max(np.abs(app2 - f["approx"])) < 1e-12
    y2 = engine.inverse(f["details"], f["approx"], lo, hi, w.wavelet_id, bc, J, nat.FLAG_FMA)
    assert np.max(np.abs(y2 - f["y"])) < 1e-12

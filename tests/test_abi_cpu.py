"""CPU-side checks of the C ABI: the library loads, exports every symbol include/vectorwave_amd.h declares,
host-only bookkeeping matches the restatement, and argument errors map to the reference's error codes.
No compute call is made (no GPU here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from oracle import oracle as O
from vectorwave_amd import _native as nat
from vectorwave_amd import errors

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "vectorwave_amd.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"VW_API\s+[\w\s\*]+?\b(vw_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = nat.load()
    syms = declared_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # the ctypes signature table covers the header exactly
    assert sorted(nat.SIGNATURES) == syms


def test_gfx950_code_object_present():
    data = open(nat.LIB_PATH, "rb").read()
    assert b"gfx950" in data


@pytest.mark.parametrize("n", [1, 2, 7, 8, 9, 63, 64, 100, 129, 512, 1000, 4096, 16384, 65536, 1 << 20])
@pytest.mark.parametrize("L", [2, 4, 6, 8, 12, 16, 18, 30])
def test_max_levels_matches_restatement(n, L):
    assert nat.load().vw_max_levels(n, L) == O.max_levels(n, L)


@pytest.mark.parametrize("L,level", [(2, 1), (8, 6), (16, 10), (30, 6), (16, 8)])
def test_upsampled_length(L, level):
    assert nat.load().vw_upsampled_length(L, level) == len(O.upsample_scale([1.0] * L, level))


def test_version_string():
    assert b"gfx950" in nat.load().vw_version()


def test_null_context_maps_to_npe():
    lib = nat.load()
    lo = nat.taps_array([0.5, 0.5])
    st = lib.vw_modwt_forward_f64(None, None, 1, 4, 4, lo, lo, 2, 0, 0, 1, 0, None, None)
    assert st == errors.VW_ERR_NULL
    assert "null" in nat.last_error()
    with pytest.raises(TypeError):
        errors.raise_for_status(st, nat.last_error())


def test_status_to_exception_mapping():
    with pytest.raises(errors.InvalidSignalException) as e:
        errors.raise_for_status(errors.VW_ERR_NONFINITE, "nan", 5)
    assert e.value.index == 5 and e.value.error_code == errors.ErrorCode.VAL_NON_FINITE_VALUES
    with pytest.raises(errors.InvalidArgumentException) as e:
        errors.raise_for_status(errors.VW_ERR_LEVEL, "lvl")
    assert e.value.error_code == errors.ErrorCode.CFG_INVALID_DECOMPOSITION_LEVEL
    with pytest.raises(errors.InvalidArgumentException) as e:
        errors.raise_for_status(errors.VW_ERR_TOO_LARGE, "big")
    assert e.value.error_code == errors.ErrorCode.VAL_TOO_LARGE
    with pytest.raises(errors.InvalidSignalException):
        errors.raise_for_status(errors.VW_ERR_EMPTY, "empty")
    with pytest.raises(NotImplementedError):
        errors.raise_for_status(errors.VW_ERR_UNSUPPORTED, "x")


def test_product_package_does_not_import_oracle():
    pkg = os.path.join(ROOT, "vectorwave_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in txt.replace("restatement", ""), f


def test_wavelet_taps_match_reference_literals():
    from vectorwave_amd.wavelets import Coiflet, Daubechies, Haar, Symlet
    import math
    assert Haar.INSTANCE.lowPassDecomposition() == [1.0 / math.sqrt(2)] * 2
    assert Daubechies.DB4.lowPassDecomposition()[0] == 0.2303778133088964
    assert len(Coiflet.COIF5.lowPassDecomposition()) == 30
    assert len(Symlet.SYM8.lowPassDecomposition()) == 16
    for w in (Daubechies.DB4, Daubechies.DB8, Symlet.SYM8, Coiflet.COIF5):
        h = w.lowPassDecomposition()
        assert abs(sum(h) - math.sqrt(2)) < 1e-6
        g = w.highPassDecomposition()
        assert g == [(1 if i % 2 == 0 else -1) * h[len(h) - 1 - i] for i in range(len(h))]


# The reference's own tap pins: vectorwave-core/src/test/java/com/morphiqlabs/wavelet/api/
# NewWaveletsTest.java:161-197 (value, index, tolerance exactly as asserted there).
@pytest.mark.parametrize("name,idx,value,tol", [
    ("DB6", 0, 0.1115407433501094, 1e-15), ("DB6", 1, 0.4946238903984530, 1e-15),
    ("DB6", 2, 0.7511339080210954, 1e-15), ("DB6", 11, -0.0010773010853085, 1e-15),
    ("SYM10", 0, 0.0007701598091030, 1e-15), ("SYM10", 14, 0.0057649120335782, 1e-15),
    ("SYM10", 19, -0.0004593294205334, 1e-15),
    ("COIF5", 0, -0.0000000960401011, 1e-15), ("COIF5", 19, 0.7742936228603274, 1e-10),
    ("COIF5", 29, -0.0002120818620675, 1e-10),
])
def test_reference_tap_pins(name, idx, value, tol):
    from vectorwave_amd.wavelets import Coiflet, Daubechies, Symlet
    w = {"DB6": Daubechies.DB6, "SYM10": Symlet.SYM10, "COIF5": Coiflet.COIF5}[name]
    taps = w.lowPassDecomposition()
    assert len(taps) == {"DB6": 12, "SYM10": 20, "COIF5": 30}[name]
    assert abs(taps[idx] - value) <= tol

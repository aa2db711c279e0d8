"""The JNI glue (jni/vectorwave_amd_jni.c) driven through a fake JNIEnv (tests/jni_harness), no JDK needed.

This proves the glue's own logic -- row gathering / scattering, the chunking of AoS batches (built here with
VW_JNI_CHUNK_BYTES = 64 KiB so every batch below spans several chunks and ends in a partial one), the signal
base of chunked error messages, the exceptions it raises for malformed arguments, and its local-reference
and pending-exception discipline -- by comparing every native against the direct C-ABI call on the same
data.  It does not prove JNI ABI compatibility with a real JVM.
Reference call sites: BatchMODWT.java:90-178 (AoS batches), BatchStreamingMODWT.java:55-275 (streams),
VectorWaveSwtAdapter.java:532-645 (denoise, noise sigma), MODWTOptimizer.java:12-84 (flat arrays).
"""
import ctypes
import os
import subprocess
from ctypes import c_double, c_int, c_long, c_ubyte, c_void_p

import numpy as np
import pytest

from oracle import oracle as O
from vectorwave_amd import _native as nat
from vectorwave_amd.wavelets import Daubechies, Symlet

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "jni_harness")
LIB = os.path.join(HERE, "libvw_jni_harness.so")
CHUNK_BYTES = 65536  # tests/jni_harness/Makefile CHUNK
PFX = "Java_com_morphiqlabs_wavelet_amd_AmdNative_"
IAE = "java/lang/IllegalArgumentException"
NPE = "java/lang/NullPointerException"
HOST = nat.FLAG_HOST_MEMORY | nat.FLAG_SYNC

# native name -> (restype, argument types after (JNIEnv*, jclass)); o = a Java object
o, i, l, d, z = c_void_p, c_int, c_long, c_double, c_ubyte
NATIVES = {
    "ctxCreate": (l, [i]), "ctxDestroy": (i, [l]), "maxLevels": (i, [l, i]), "lastError": (o, []),
    "lastErrorIndex": (l, []),
    "modwt1Forward": (i, [l, o, i, i, o, o, i, i, o, o]),
    "modwt1Inverse": (i, [l, o, o, i, i, o, o, i, i, o]),
    "modwtForward": (i, [l, o, i, i, o, o, i, i, i, i, o, o]),
    "modwtInverse": (i, [l, o, o, i, i, o, o, i, i, i, i, z, i, o]),
    "modwtForwardMulti": (i, [o, o, i, i, o, o, i, i, i, i, o, o]),
    "swtDenoise": (i, [l, o, i, i, o, o, i, i, i, d, z, i, o, o]),
    "waveletDenoise": (i, [l, o, i, i, o, o, i, i, i, i, d, z, i, o, o]),
    "noiseSigma": (i, [l, o, i, i, o]),
    "modwtForwardDirect": (i, [l, o, i, i, o, o, i, i, i, i, o, o]),
    "modwtInverseDirect": (i, [l, o, o, i, i, o, o, i, i, i, i, o]),
    "modwtForwardAoS": (i, [l, o, o, o, i, i, i, i, o, o]),
    "modwtInverseAoS": (i, [l, o, o, o, o, i, i, i, o]),
    "swtDenoiseAoS": (i, [l, o, o, o, i, i, i, d, z, i, o]),
    "streamCreate": (l, [l, o, o, i, i]), "streamDestroy": (i, [l]), "streamHistoryLength": (l, [l, i]),
    "streamProcessAoS": (i, [l, o, o, o]), "streamFlushAoS": (i, [l, i, o, o]),
}


def _harness():
    srcs = [os.path.join(HERE, f) for f in ("harness.c", "jni.h", "Makefile")]
    srcs.append(os.path.join(HERE, "..", "..", "jni", "vectorwave_amd_jni.c"))
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(s) for s in srcs):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)  # normally built by __graft_entry__.build()
    L = ctypes.CDLL(LIB)
    for name, (res, args) in {"h_env": (o, []), "h_doubles": (o, [o, i]), "h_longs": (o, [o, i]),
                              "h_objects": (o, [i]), "h_set": (None, [o, i, o]), "h_direct": (o, [o, l]),
                              "h_free": (None, [o]), "h_string": (ctypes.c_char_p, [o]),
                              "h_pending": (ctypes.c_char_p, []), "h_clear": (None, []), "h_misuse": (i, []),
                              "h_live_refs": (l, []), "h_peak_refs": (l, []),
                              "h_reset_counts": (None, [])}.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    for name, (res, args) in NATIVES.items():
        f = getattr(L, PFX + name)
        f.restype, f.argtypes = res, [o, o] + args
    return L


@pytest.fixture(scope="module")
def jni():
    return Jni(_harness())


class Jni:
    """Java-side objects over numpy memory (kept alive here) and checked native calls."""

    def __init__(self, L):
        self.L, self.env, self.keep, self.objs = L, L.h_env(), [], []

    def _o(self, obj):
        self.objs.append(obj)
        return obj

    def doubles(self, a):
        """double[] over `a`'s memory (a 1-D contiguous float64 array; results written there)."""
        assert a.dtype == np.float64 and a.flags.c_contiguous and a.ndim == 1
        self.keep.append(a)
        return self._o(self.L.h_doubles(a.ctypes.data, len(a)))

    def rows(self, m):
        """double[][] whose rows are m's rows (None entries stay null)."""
        arr = self._o(self.L.h_objects(len(m)))
        for k, r in enumerate(m):
            self.L.h_set(arr, k, None if r is None else self.doubles(r))
        return arr

    def planes(self, cube):
        arr = self._o(self.L.h_objects(len(cube)))
        for k, m in enumerate(cube):
            self.L.h_set(arr, k, None if m is None else self.rows(m))
        return arr

    def longs(self, a):
        a = np.ascontiguousarray(a, dtype=np.int64)
        self.keep.append(a)
        return self._o(self.L.h_longs(a.ctypes.data, len(a)))

    def direct(self, a):
        self.keep.append(a)
        return self._o(self.L.h_direct(a.ctypes.data, a.nbytes))

    def call(self, name, *args, expect=None):
        """Native call; checks the JNI discipline, returns (status, pending exception text or None)."""
        self.L.h_clear()
        self.L.h_reset_counts()
        st = getattr(self.L, PFX + name)(self.env, None, *args)
        pend = self.L.h_pending()
        pend = pend.decode() if pend else None
        assert self.L.h_misuse() == 0, f"{name}: JNI call made with an exception pending / on a wrong object"
        assert self.L.h_live_refs() == 0, f"{name}: leaked {self.L.h_live_refs()} local references"
        assert self.L.h_peak_refs() <= 16, f"{name}: {self.L.h_peak_refs()} live local references (JNI: 16)"
        if expect is not None:
            assert pend is not None and pend.startswith(expect[0]) and expect[1] in pend, (name, st, pend)
        return st, pend

    def raw(self, name, *args):
        """A native whose result is not a status (handles, lengths): a fresh call, as a JVM makes it after the
        previous native's exception was thrown."""
        self.L.h_clear()
        return getattr(self.L, PFX + name)(self.env, None, *args)

    def last_error(self):
        self.L.h_clear()
        s = getattr(self.L, PFX + "lastError")(self.env, None)
        return self.L.h_string(s).decode()


def signals(B, n, seed):
    return np.stack([O.java_random_signal(n, seed + b) for b in range(B)])


def taps(w):
    return np.array(w.lowPassDecomposition()), np.array(w.highPassDecomposition())


def chunk_rows(per_row_doubles, B):
    return max(1, min(B, CHUNK_BYTES // (per_row_doubles * 8)))


# ---- argument errors the glue raises itself (no engine call: runs without a GPU, ctx = 0) ------------------
def test_malformed_aos_arguments_raise_their_own_exceptions(jni):
    lo, hi = taps(Daubechies.DB4)
    J, n = 3, 256
    x = signals(4, n, 1)
    det = np.zeros((J, 4, n))
    app = np.zeros((4, n))
    args = lambda xo, do, ao: (0, xo, jni.doubles(lo), jni.doubles(hi), 4, 0, J, 0, do, ao)  # noqa: E731
    ragged = [x[0], x[1][:100], x[2], x[3]]
    st, _ = jni.call("modwtForwardAoS", *args(jni.rows(ragged), jni.planes(det), jni.rows(app)),
                     expect=(IAE, "all signals must be non-null and same length"))
    assert st == 7
    jni.call("modwtForwardAoS", *args(jni.rows([x[0], None, x[2], x[3]]), jni.planes(det), jni.rows(app)),
             expect=(IAE, "non-null"))
    jni.call("modwtForwardAoS", *args(None, jni.planes(det), jni.rows(app)), expect=(IAE, "non-null and non-empty"))
    jni.call("modwtForwardAoS", *args(jni.rows(x), jni.planes(det[:2]), jni.rows(app)),
             expect=(IAE, "one plane per level"))
    jni.call("modwtForwardAoS", *args(jni.rows(x), jni.planes([det[0], det[1][:3], det[2]]), jni.rows(app)),
             expect=(IAE, "detailPerLevel[L] must be non-null and length=batch"))
    jni.call("modwtForwardAoS", *args(jni.rows(x), jni.planes([det[0], None, det[2]]), jni.rows(app)),
             expect=(IAE, "detailPerLevel[L]"))
    jni.call("modwtForwardAoS", *args(jni.rows(x), jni.planes(det), jni.rows(app[:3])),
             expect=(IAE, "one row per signal"))
    jni.call("modwtForwardAoS", 0, jni.rows(x), jni.doubles(lo), jni.doubles(hi[:5]), 4, 0, J, 0, jni.planes(det),
             jni.rows(app), expect=(IAE, "filter taps"))
    jni.call("modwtForwardAoS", 0, jni.rows(x), None, jni.doubles(hi), 4, 0, J, 0, jni.planes(det), jni.rows(app),
             expect=(NPE, "taps"))
    # inverse: a short detail plane, a ragged approximation row, the output's row count
    y = np.zeros((4, n))
    jni.call("modwtInverseAoS", 0, jni.planes([det[0], det[1][:3], det[2]]), jni.rows(app), jni.doubles(lo),
             jni.doubles(hi), 4, 0, 0, jni.rows(y), expect=(IAE, "detailPerLevel[L]"))
    jni.call("modwtInverseAoS", 0, jni.planes(det), jni.rows([app[0], app[1][:9], app[2], app[3]]), jni.doubles(lo),
             jni.doubles(hi), 4, 0, 0, jni.rows(y), expect=(IAE, "same length"))
    jni.call("modwtInverseAoS", 0, jni.planes(det), jni.rows(app), jni.doubles(lo), jni.doubles(hi), 4, 0, 0,
             jni.rows(y[:2]), expect=(IAE, "one row per signal"))
    jni.call("swtDenoiseAoS", 0, jni.rows(x), jni.doubles(lo), jni.doubles(hi), 4, 0, J, -1.0, 1, 0,
             jni.rows(y[:1]), expect=(IAE, "one row per signal"))


def test_malformed_flat_and_direct_arguments(jni):
    lo, hi = taps(Daubechies.DB4)
    x, a, dd = np.zeros(64), np.zeros(64), np.zeros(63)
    jni.call("modwt1Forward", 0, jni.doubles(x), 1, 64, jni.doubles(lo), jni.doubles(hi), 0, 0, jni.doubles(a),
             jni.doubles(dd), expect=(IAE, "shorter than B * N"))
    jni.call("modwt1Forward", 0, jni.doubles(x), 0, 64, jni.doubles(lo), jni.doubles(hi), 0, 0, jni.doubles(a),
             jni.doubles(a), expect=(IAE, "must be > 0"))
    jni.call("modwtForward", 0, jni.doubles(x), 1, 64, jni.doubles(lo), jni.doubles(hi), 4, 0, 2, 0,
             jni.doubles(np.zeros(100)), jni.doubles(a), expect=(IAE, "levels * B * N"))
    jni.call("modwtForward", 0, None, 1, 64, jni.doubles(lo), jni.doubles(hi), 4, 0, 2, 0,
             jni.doubles(np.zeros(128)), jni.doubles(a), expect=(NPE, "cannot be null"))
    # a heap double[] where a direct ByteBuffer is required
    jni.call("modwtForwardDirect", 0, jni.doubles(x), 1, 64, jni.doubles(lo), jni.doubles(hi), 4, 0, 2, 0,
             jni.direct(np.zeros(128)), jni.direct(np.zeros(64)), expect=(IAE, "direct"))
    jni.call("noiseSigma", 0, jni.doubles(x), 2, 64, jni.doubles(np.zeros(2)), expect=(IAE, "shorter"))
    st, pend = jni.call("maxLevels", 4096, 8)
    assert st == nat.load().vw_max_levels(4096, 8) and pend is None


# ---- every native against the direct C-ABI call (GPU) ----------------------------------------------------
def cabi_forward(engine, x, w, boundary, J, flags):
    B, n = x.shape
    det, app = np.empty((J, B, n)), np.empty((B, n))
    lo, hi = nat.taps_array(w.lowPassDecomposition()), nat.taps_array(w.highPassDecomposition())
    st = engine.lib.vw_modwt_forward_f64(engine.ctx, x.ctypes.data, B, n, n, lo, hi, len(w.lowPassDecomposition()),
                                         w.wavelet_id, boundary, J, flags | HOST, det.ctypes.data, app.ctypes.data)
    assert st == 0, nat.last_error()
    return det, app


def cabi_inverse(engine, det, app, w, boundary, flags, mask=0xFFFFFFFF, approx_zero=0):
    J, B, n = det.shape
    y = np.empty((B, n))
    lo, hi = nat.taps_array(w.lowPassDecomposition()), nat.taps_array(w.highPassDecomposition())
    st = engine.lib.vw_modwt_inverse_f64(engine.ctx, det.ctypes.data, app.ctypes.data, B, n, lo, hi,
                                         len(w.lowPassDecomposition()), w.wavelet_id, boundary, J, mask, approx_zero,
                                         flags | HOST, y.ctypes.data)
    assert st == 0, nat.last_error()
    return y


def ctx_of(engine):
    return ctypes.cast(engine.ctx, c_void_p).value


@pytest.mark.gpu
@pytest.mark.parametrize("boundary", [O.PERIODIC, O.SYMMETRIC], ids=["P", "S"])
@pytest.mark.parametrize("flags", [0, nat.FLAG_FMA, nat.FLAG_CORE_LEVELS | nat.FLAG_VALIDATE | nat.FLAG_FFT_SWITCH],
                         ids=["batch", "fma", "core"])
def test_aos_forward_inverse_chunks_bit_exact(engine, jni, boundary, flags):
    w, n, J, B = Daubechies.DB4, 512, 4, 7
    cb = chunk_rows((J + 2) * n, B)
    assert cb == 2 and B % cb != 0  # four chunks, the last one partial
    x = signals(B, n, 3)
    lo, hi = taps(w)
    det, app = np.full((J, B, n), -7.0), np.full((B, n), -7.0)
    st, pend = jni.call("modwtForwardAoS", ctx_of(engine), jni.rows(x), jni.doubles(lo), jni.doubles(hi), w.wavelet_id,
                        boundary, J, flags, jni.planes(det), jni.rows(app))
    assert st == 0 and pend is None
    d_ref, a_ref = cabi_forward(engine, x, w, boundary, J, flags)
    assert np.array_equal(det, d_ref) and np.array_equal(app, a_ref)
    y = np.full((B, n), -7.0)
    st, pend = jni.call("modwtInverseAoS", ctx_of(engine), jni.planes(det), jni.rows(app), jni.doubles(lo),
                        jni.doubles(hi), w.wavelet_id, boundary, flags & ~nat.FLAG_VALIDATE, jni.rows(y))
    assert st == 0 and pend is None
    assert np.array_equal(y, cabi_inverse(engine, d_ref, a_ref, w, boundary, flags & ~nat.FLAG_VALIDATE))
    if flags == 0 and boundary == O.PERIODIC:  # and the restatement (BatchMODWT semantics)
        for b in (0, B - 1):
            dr, ar = O.decompose(x[b], lo, hi, O.PERIODIC, J, core=False)
            assert np.array_equal(det[:, b, :], dr) and np.array_equal(app[b], ar)


@pytest.mark.gpu
def test_aos_nonfinite_error_names_the_batch_signal(engine, jni):
    # chunk 2 (rows 4-5) holds the bad sample: the message names signal 5 of the batch, not signal 1 of the chunk
    w, n, J, B = Daubechies.DB4, 512, 4, 7
    x = signals(B, n, 5)
    x[5, 123] = np.nan
    lo, hi = taps(w)
    det, app = np.zeros((J, B, n)), np.zeros((B, n))
    st, pend = jni.call("modwtForwardAoS", ctx_of(engine), jni.rows(x), jni.doubles(lo), jni.doubles(hi), w.wavelet_id,
                        0, J, nat.FLAG_CORE_LEVELS | nat.FLAG_VALIDATE, jni.planes(det), jni.rows(app))
    assert st == 3 and pend is None  # VW_ERR_NONFINITE -> AmdNative.check -> InvalidSignalException
    msg = jni.last_error()
    assert "signal 5" in msg and "index 123" in msg, msg
    assert jni.raw("lastErrorIndex") == 123


@pytest.mark.gpu
@pytest.mark.parametrize("soft", [1, 0], ids=["soft", "hard"])
def test_aos_swt_denoise_chunks_bit_exact(engine, jni, soft):
    w, n, J, B = Symlet.SYM8, 2048, 4, 5
    assert chunk_rows(2 * n, B) == 2
    x = signals(B, n, 11)
    lo, hi = taps(w)
    y = np.zeros((B, n))
    st, pend = jni.call("swtDenoiseAoS", ctx_of(engine), jni.rows(x), jni.doubles(lo), jni.doubles(hi), w.wavelet_id,
                        0, J, -1.0, soft, 0, jni.rows(y))
    assert st == 0 and pend is None
    y_ref, t_ref = np.empty((B, n)), np.empty(B)
    st = engine.lib.vw_swt_denoise_f64(engine.ctx, x.ctypes.data, B, n, n, nat.taps_array(lo), nat.taps_array(hi), 16,
                                       w.wavelet_id, 0, J, -1.0, soft, HOST, y_ref.ctypes.data, t_ref.ctypes.data)
    assert st == 0 and np.array_equal(y, y_ref)
    # the flat form with its thresholds
    yf, tf = np.zeros(B * n), np.zeros(B)
    st, _ = jni.call("swtDenoise", ctx_of(engine), jni.doubles(x.reshape(-1).copy()), B, n, jni.doubles(lo),
                     jni.doubles(hi), w.wavelet_id, 0, J, -1.0, soft, 0, jni.doubles(yf), jni.doubles(tf))
    assert st == 0 and np.array_equal(yf.reshape(B, n), y_ref) and np.array_equal(tf, t_ref)


@pytest.mark.gpu
def test_flat_natives_match_the_c_abi(engine, jni):
    w, n, J, B = Daubechies.DB4, 1024, 3, 3
    x = signals(B, n, 21)
    lo, hi = taps(w)
    flat = x.reshape(-1).copy()
    # single level (MODWTOptimizer.forward / inverse, MODWTTransform semantics)
    a, dd = np.zeros(B * n), np.zeros(B * n)
    st, _ = jni.call("modwt1Forward", ctx_of(engine), jni.doubles(flat), B, n, jni.doubles(lo), jni.doubles(hi), 1,
                     nat.FLAG_VALIDATE, jni.doubles(a), jni.doubles(dd))
    assert st == 0
    for b in range(B):
        ar, dr = O.modwt_forward(x[b], lo, hi, O.SYMMETRIC)
        assert np.array_equal(a.reshape(B, n)[b], ar) and np.array_equal(dd.reshape(B, n)[b], dr)
    y1 = np.zeros(B * n)
    st, _ = jni.call("modwt1Inverse", ctx_of(engine), jni.doubles(a), jni.doubles(dd), B, n, jni.doubles(lo),
                     jni.doubles(hi), 1, 0, jni.doubles(y1))
    assert st == 0
    for b in range(B):
        ref = O.modwt_inverse(a.reshape(B, n)[b], dd.reshape(B, n)[b], lo, hi, O.SYMMETRIC)
        assert np.array_equal(y1.reshape(B, n)[b], ref)
    # multi level, flat, with a detail mask (reconstructFromLevel 2) and a zero approximation
    det, app = np.zeros(J * B * n), np.zeros(B * n)
    st, _ = jni.call("modwtForward", ctx_of(engine), jni.doubles(flat), B, n, jni.doubles(lo), jni.doubles(hi),
                     w.wavelet_id, 0, J, 0, jni.doubles(det), jni.doubles(app))
    assert st == 0
    d_ref, a_ref = cabi_forward(engine, x, w, 0, J, 0)
    assert np.array_equal(det.reshape(J, B, n), d_ref) and np.array_equal(app.reshape(B, n), a_ref)
    for mask, az in ((0b110, 0), (0b011, 1)):
        y = np.zeros(B * n)
        st, _ = jni.call("modwtInverse", ctx_of(engine), jni.doubles(det), jni.doubles(app), B, n, jni.doubles(lo),
                         jni.doubles(hi), w.wavelet_id, 0, J, mask, az, 0, jni.doubles(y))
        assert st == 0
        assert np.array_equal(y.reshape(B, n), cabi_inverse(engine, d_ref, a_ref, w, 0, 0, mask, az))
    # direct buffers (zero-copy path)
    dx, ddet, dapp, dy = flat.copy(), np.zeros(J * B * n), np.zeros(B * n), np.zeros(B * n)
    st, _ = jni.call("modwtForwardDirect", ctx_of(engine), jni.direct(dx), B, n, jni.doubles(lo), jni.doubles(hi),
                     w.wavelet_id, 0, J, 0, jni.direct(ddet), jni.direct(dapp))
    assert st == 0 and np.array_equal(ddet, det) and np.array_equal(dapp, app)
    st, _ = jni.call("modwtInverseDirect", ctx_of(engine), jni.direct(ddet), jni.direct(dapp), B, n, jni.doubles(lo),
                     jni.doubles(hi), w.wavelet_id, 0, J, 0, jni.direct(dy))
    assert st == 0 and np.array_equal(dy.reshape(B, n), cabi_inverse(engine, d_ref, a_ref, w, 0, 0))
    # noise sigma (estimateNoiseSigma) of d_1 per row
    sig = np.zeros(B)
    st, _ = jni.call("noiseSigma", ctx_of(engine), jni.doubles(d_ref[0].reshape(-1).copy()), B, n, jni.doubles(sig))
    assert st == 0 and all(sig[b] == O.noise_sigma(d_ref[0][b]) for b in range(B))
    # WaveletDenoiser (SURE, multi-level) with its per-level thresholds
    yw, tw = np.zeros(B * n), np.zeros(J * B)
    st, _ = jni.call("waveletDenoise", ctx_of(engine), jni.doubles(flat), B, n, jni.doubles(lo), jni.doubles(hi),
                     w.wavelet_id, 0, J, O.SURE, 0.0, 1, 0, jni.doubles(yw), jni.doubles(tw))
    assert st == 0
    for b in range(B):
        y_ref, t_ref = O.wavelet_denoise(x[b], lo, hi, O.PERIODIC, J, O.SURE, wavelet_id=w.wavelet_id)
        assert np.array_equal(yw.reshape(B, n)[b], y_ref) and np.array_equal(tw.reshape(J, B)[:, b], t_ref)


@pytest.mark.gpu
def test_multi_context_native(engine, jni):
    import vectorwave_amd as vw
    w, n, J, B = Daubechies.DB4, 512, 3, 5
    x = signals(B, n, 8)
    lo, hi = taps(w)
    second = vw.Engine(0)
    try:
        det, app = np.zeros(J * B * n), np.zeros(B * n)
        st, _ = jni.call("modwtForwardMulti", jni.longs([ctx_of(engine), ctx_of(second)]),
                         jni.doubles(x.reshape(-1).copy()), B, n, jni.doubles(lo), jni.doubles(hi), w.wavelet_id, 0, J, 0,
                         jni.doubles(det), jni.doubles(app))
        assert st == 0
        d_ref, a_ref = cabi_forward(engine, x, w, 0, J, 0)
        assert np.array_equal(det.reshape(J, B, n), d_ref) and np.array_equal(app.reshape(B, n), a_ref)
    finally:
        second.close()


@pytest.mark.gpu
@pytest.mark.parametrize("boundary", [O.SYMMETRIC, O.ZERO_PADDING], ids=["S", "Z"])
def test_stream_natives_match_the_restatement(engine, jni, boundary):
    # BatchStreamingMODWT (ZERO / SYMMETRIC): history kept on the device across blocks, then the flush
    w, J, B, n = Daubechies.DB4, 3, 3, 256
    lo, hi = taps(w)
    h = jni.raw("streamCreate", ctx_of(engine), jni.doubles(lo), jni.doubles(hi), boundary, J)
    assert h
    try:
        assert [jni.raw("streamHistoryLength", h, j) for j in (1, 2, 3, 4)] == [7, 14, 28, -1]
        refs = [O.StreamRestatement(lo, hi, boundary, J) for _ in range(B)]
        for blk in range(2):
            x = signals(B, n, 100 + 10 * blk)
            det, app = np.zeros((J, B, n)), np.zeros((B, n))
            st, pend = jni.call("streamProcessAoS", h, jni.rows(x), jni.planes(det), jni.rows(app))
            assert st == 0 and pend is None
            for b in range(B):
                dr, ar = refs[b].process(x[b])
                assert np.array_equal(det[:, b, :], dr) and np.array_equal(app[b], ar)
        tail = 7
        det, app = np.zeros((J, B, tail)), np.zeros((B, tail))
        st, pend = jni.call("streamFlushAoS", h, tail, jni.planes(det), jni.rows(app))
        assert st == 0 and pend is None
        for b in range(B):
            dr, ar = refs[b].flush(tail)
            assert np.array_equal(det[:, b, :], dr) and np.array_equal(app[b], ar)
        # the planes must be the configured levels, the flush rows the last block's batch
        jni.call("streamProcessAoS", h, jni.rows(signals(B, n, 1)), jni.planes(np.zeros((2, B, n))),
                 jni.rows(np.zeros((B, n))), expect=(IAE, "configured level"))
        jni.call("streamFlushAoS", h, tail, jni.planes(np.zeros((J, 2, tail))), jni.rows(np.zeros((2, tail))),
                 expect=(IAE, "last block"))
    finally:
        assert jni.raw("streamDestroy", h) == 0

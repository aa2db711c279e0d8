"""ctypes wrapper of the CPU restatement (oracle/vw_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only
as the checker / CPU baseline.  The product (vectorwave_amd/) never imports it.

Every entry point follows one Java loop of the reference (file:line cited in vw_oracle.c).  Also
holds a java.util.Random restatement so tests can reproduce the reference tests' inputs.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from ctypes import POINTER, c_double, c_int, c_longlong, c_uint, c_ulonglong, c_void_p

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "libvw_oracle.so")

PERIODIC, SYMMETRIC, ZERO_PADDING = 0, 1, 2
_dp = POINTER(c_double)


def build() -> str:
    """Compile the restatement (gcc, -ffp-contract=off) if needed."""
    src = os.path.join(_HERE, "vw_oracle.c")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return LIB


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        sig = {
            "vwo_max_levels": (c_int, [c_int, c_int]),
            "vwo_upsampled_length": (c_int, [c_int, c_int]),
            "vwo_upsample_scale": (c_int, [_dp, c_int, c_int, _dp]),
            "vwo_symmetric_index": (c_int, [c_int, c_int]),
            "vwo_circular_conv": (None, [_dp, c_int, _dp, c_int, _dp]),
            "vwo_circular_conv_direct": (None, [_dp, c_int, _dp, c_int, _dp]),
            "vwo_zero_conv": (None, [_dp, c_int, _dp, c_int, _dp]),
            "vwo_symmetric_conv": (None, [_dp, c_int, _dp, c_int, _dp]),
            "vwo_fft_conv": (None, [_dp, c_int, _dp, c_int, _dp]),
            "vwo_should_use_fft": (c_int, [c_int, c_int]),
            "vwo_ml_decompose": (c_int, [_dp, c_int, _dp, _dp, c_int, c_int, c_int, c_int, _dp, _dp,
                                         POINTER(c_longlong)]),
            "vwo_ml_reconstruct": (c_int, [_dp, _dp, c_int, _dp, _dp, c_int, c_int, c_int, c_int, c_uint, c_int, _dp]),
            "vwo_sym_decide": (None, [c_int, c_int, c_int, POINTER(c_int), POINTER(c_int), POINTER(c_int),
                                      POINTER(c_int)]),
            "vwo_compute_tau": (c_int, [c_int, c_int]),
            "vwo_modwt_forward": (c_int, [_dp, c_int, _dp, _dp, c_int, c_int, _dp, _dp, POINTER(c_longlong)]),
            "vwo_modwt_inverse": (c_int, [_dp, _dp, c_int, _dp, _dp, c_int, c_int, c_int, _dp]),
            "vwo_swt_forward": (c_int, [_dp, c_int, _dp, _dp, c_int, c_int, c_int, _dp, _dp]),
            "vwo_sure_risk": (c_double, [_dp, c_int, c_double, c_double]),
            "vwo_sure_threshold": (c_double, [_dp, c_int, c_double]),
            "vwo_minimax_threshold": (c_double, [c_int, c_double]),
            "vwo_bayes_threshold": (c_double, [_dp, c_int, c_double]),
            "vwo_calc_threshold": (c_int, [_dp, c_int, c_double, c_int, _dp]),
            "vwo_wavelet_denoise": (c_int, [_dp, c_int, _dp, _dp, c_int, c_int, c_int, c_int, c_int, c_double, c_int,
                                            _dp, _dp, POINTER(c_longlong)]),
            "vwo_swt_reconstruct_periodic": (None, [_dp, _dp, c_int, _dp, _dp, c_int, c_int, _dp]),
            "vwo_noise_sigma": (c_double, [_dp, c_int]),
            "vwo_universal_threshold": (c_double, [c_double, c_int]),
            "vwo_threshold": (None, [_dp, c_int, c_double, c_int]),
            "vwo_swt_denoise": (c_int, [_dp, c_int, _dp, _dp, c_int, c_int, c_int, c_int, c_double, c_int, _dp, _dp]),
            "vwo_batch_single": (None, [_dp, c_int, _dp, _dp, c_int, c_int, _dp, _dp]),
            "vwo_conv_with_history": (None, [_dp, c_int, _dp, c_int, _dp, _dp, c_int, _dp, _dp]),
            "vwo_batch_fwd_inv": (c_int, [_dp, c_longlong, c_int, _dp, _dp, c_int, c_int, c_int, c_int, _dp]),
            "vwo_batch_denoise": (c_int, [_dp, c_longlong, c_int, _dp, _dp, c_int, c_int, c_int, c_int, c_double,
                                          c_int, _dp]),
            "vwo_fill_uniform": (None, [_dp, c_longlong, c_ulonglong, c_longlong]),
            "vwo_first_nonfinite": (c_longlong, [_dp, c_longlong]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(_dp)


def _arr(x) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x, dtype=np.float64))


class OracleError(Exception):
    def __init__(self, status: int, index: int = -1):
        super().__init__(f"oracle status {status}")
        self.status = status
        self.index = index


def max_levels(n: int, L: int) -> int:
    return lib().vwo_max_levels(n, L)


def upsample_scale(base, level: int) -> np.ndarray:
    base = _arr(base)
    Lj = lib().vwo_upsampled_length(len(base), level)
    out = np.empty(Lj)
    lib().vwo_upsample_scale(_p(base), len(base), level, _p(out))
    return out


def symmetric_index(idx: int, n: int) -> int:
    return lib().vwo_symmetric_index(idx, n)


def conv(kind: str, x, f) -> np.ndarray:
    x, f = _arr(x), _arr(f)
    out = np.empty(len(x))
    fn = {"circular": lib().vwo_circular_conv, "direct": lib().vwo_circular_conv_direct, "zero": lib().vwo_zero_conv,
          "symmetric": lib().vwo_symmetric_conv, "fft": lib().vwo_fft_conv}[kind]
    fn(_p(x), len(x), _p(f), len(f), _p(out))
    return out


def decompose(x, lo, hi, boundary: int, levels: int, core: bool = True):
    """MultiLevelMODWTTransform.decompose (core=True) or BatchMODWT.multiLevelAoS semantics (core=False).
    Returns (details [J][N], approx [N])."""
    x, lo, hi = _arr(x), _arr(lo), _arr(hi)
    n = len(x)
    det = np.empty((levels, n))
    app = np.empty(n)
    bad = c_longlong(-1)
    st = lib().vwo_ml_decompose(_p(x), n, _p(lo), _p(hi), len(lo), boundary, levels, 1 if core else 0, _p(det), _p(app),
                                ctypes.byref(bad))
    if st != 0:
        raise OracleError(st, bad.value)
    return det, app


def reconstruct(det, app, lo, hi, boundary: int, wavelet_id: int = 0, detail_mask: int = 0xFFFFFFFF,
                approx_zero: bool = False) -> np.ndarray:
    det, app, lo, hi = _arr(det), _arr(app), _arr(lo), _arr(hi)
    J, n = det.shape
    y = np.empty(n)
    st = lib().vwo_ml_reconstruct(_p(det), _p(app), n, _p(lo), _p(hi), len(lo), wavelet_id, boundary, J,
                                  detail_mask & 0xFFFFFFFF, 1 if approx_zero else 0, _p(y))
    if st != 0:
        raise OracleError(st)
    return y


def sym_decide(wavelet_id: int, L: int, level: int):
    a, b, c, d = c_int(), c_int(), c_int(), c_int()
    lib().vwo_sym_decide(wavelet_id, L, level, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c), ctypes.byref(d))
    return a.value, b.value, c.value, d.value


def modwt_forward(x, lo, hi, boundary: int):
    x, lo, hi = _arr(x), _arr(lo), _arr(hi)
    a, d = np.empty(len(x)), np.empty(len(x))
    bad = c_longlong(-1)
    st = lib().vwo_modwt_forward(_p(x), len(x), _p(lo), _p(hi), len(lo), boundary, _p(a), _p(d), ctypes.byref(bad))
    if st != 0:
        raise OracleError(st, bad.value)
    return a, d


def modwt_inverse(a, d, lo, hi, boundary: int, batch_optimized: bool = False) -> np.ndarray:
    a, d, lo, hi = _arr(a), _arr(d), _arr(lo), _arr(hi)
    y = np.empty(len(a))
    lib().vwo_modwt_inverse(_p(a), _p(d), len(a), _p(lo), _p(hi), len(lo), boundary, 1 if batch_optimized else 0, _p(y))
    return y


def swt_forward(x, lo, hi, boundary: int, levels: int):
    x, lo, hi = _arr(x), _arr(lo), _arr(hi)
    det = np.empty((levels, len(x)))
    app = np.empty(len(x))
    lib().vwo_swt_forward(_p(x), len(x), _p(lo), _p(hi), len(lo), boundary, levels, _p(det), _p(app))
    return det, app


def swt_reconstruct_periodic(det, app, lo, hi) -> np.ndarray:
    det, app, lo, hi = _arr(det), _arr(app), _arr(lo), _arr(hi)
    y = np.empty(det.shape[1])
    lib().vwo_swt_reconstruct_periodic(_p(det), _p(app), det.shape[1], _p(lo), _p(hi), len(lo), det.shape[0], _p(y))
    return y


def noise_sigma(c) -> float:
    c = _arr(c)
    return lib().vwo_noise_sigma(_p(c), len(c))


def universal_threshold(sigma: float, n: int) -> float:
    return lib().vwo_universal_threshold(sigma, n)


def threshold(c, t: float, soft: bool) -> np.ndarray:
    c = _arr(c).copy()
    lib().vwo_threshold(_p(c), len(c), t, 1 if soft else 0)
    return c


def swt_denoise(x, lo, hi, boundary: int, levels: int, thr: float = -1.0, soft: bool = True, wavelet_id: int = 0):
    x, lo, hi = _arr(x), _arr(lo), _arr(hi)
    y = np.empty(len(x))
    t = c_double()
    st = lib().vwo_swt_denoise(_p(x), len(x), _p(lo), _p(hi), len(lo), wavelet_id, boundary, levels, thr,
                               1 if soft else 0, _p(y), ctypes.byref(t))
    if st != 0:
        raise OracleError(st)
    return y, t.value


def batch_single(x, lo, hi, is_haar: bool):
    x, lo, hi = _arr(x), _arr(lo), _arr(hi)
    a, d = np.empty(len(x)), np.empty(len(x))
    lib().vwo_batch_single(_p(x), len(x), _p(lo), _p(hi), len(lo), 1 if is_haar else 0, _p(a), _p(d))
    return a, d


def conv_with_history(hist, x, flo, fhi):
    hist, x, flo, fhi = _arr(hist), _arr(x), _arr(flo), _arr(fhi)
    a, d = np.empty(len(x)), np.empty(len(x))
    lib().vwo_conv_with_history(_p(hist), len(hist), _p(x), len(x), _p(flo), _p(fhi), len(flo), _p(a), _p(d))
    return a, d


class StreamRestatement:
    """BatchStreamingMODWT (ext/extensions/modwt/BatchStreamingMODWT.java) for ZERO_PADDING / SYMMETRIC,
    one signal: per-level left history of L_j - 1 samples, initialised from the first block (zeros,
    or the half-sample mirror of the block, fillSymmetricHistoryFromSoA :326-335), convolved with the
    level input (generalBatchMODWTSoAWithScaledFiltersAndHistory = vwo_conv_with_history), updated
    from the level input (updateHistoryFromSoA :337-352); flushMultiLevel (:231-275) runs a synthetic
    tail (zeros, or the last history samples reflected, buildTailFromHistorySoA :362-376) through every
    level's history without updating it."""

    def __init__(self, lo, hi, boundary: int, levels: int):
        self.lo, self.hi = _arr(lo), _arr(hi)
        self.boundary, self.levels = boundary, levels
        self.flo = [upsample_scale(self.lo, j) for j in range(1, levels + 1)]
        self.fhi = [upsample_scale(self.hi, j) for j in range(1, levels + 1)]
        self.hist = [None] * levels

    def process(self, block):
        cur = _arr(block)
        n = len(cur)
        det = np.empty((self.levels, n))
        for j in range(self.levels):
            hl = len(self.flo[j]) - 1
            if self.hist[j] is None:
                if self.boundary == ZERO_PADDING:
                    self.hist[j] = np.zeros(hl)
                else:
                    self.hist[j] = np.array([cur[symmetric_index(p - hl, n)] for p in range(hl)])
            a, d = conv_with_history(self.hist[j], cur, self.flo[j], self.fhi[j])
            det[j] = d
            if hl > 0:  # updateHistoryFromSoA
                self.hist[j] = cur[n - hl:].copy() if n >= hl else np.concatenate([self.hist[j][n:], cur])
            cur = a
        return det, cur

    def flush(self, tail_len: int):
        h0 = self.hist[0]
        cur = np.zeros(tail_len) if self.boundary == ZERO_PADDING else \
            np.array([h0[len(h0) - 1 - t] for t in range(tail_len)])
        det = np.empty((self.levels, tail_len))
        for j in range(self.levels):
            a, d = conv_with_history(self.hist[j], cur, self.flo[j], self.fhi[j])
            det[j] = d
            cur = a
        return det, cur


def batch_fwd_inv(x: np.ndarray, lo, hi, boundary: int, levels: int, wavelet_id: int = 0):
    """Core decompose + reconstruct per row, OpenMP over rows.  Returns (y, threads)."""
    x, lo, hi = _arr(x), _arr(lo), _arr(hi)
    B, n = x.shape
    y = np.empty_like(x)
    th = lib().vwo_batch_fwd_inv(_p(x), B, n, _p(lo), _p(hi), len(lo), wavelet_id, boundary, levels, _p(y))
    return y, th


def batch_denoise(x: np.ndarray, lo, hi, boundary: int, levels: int, thr: float = -1.0, soft: bool = True,
                  wavelet_id: int = 0):
    x, lo, hi = _arr(x), _arr(lo), _arr(hi)
    B, n = x.shape
    y = np.empty_like(x)
    th = lib().vwo_batch_denoise(_p(x), B, n, _p(lo), _p(hi), len(lo), wavelet_id, boundary, levels, thr,
                                 1 if soft else 0, _p(y))
    return y, th


def fill_uniform(count: int, seed: int = 42, offset: int = 0) -> np.ndarray:
    out = np.empty(count)
    lib().vwo_fill_uniform(_p(out), count, seed, offset)
    return out


class JavaRandom:
    """java.util.Random restatement (48-bit LCG 0x5DEECE66D); nextDouble is bit-reproducible."""

    MULT = 0x5DEECE66D
    MASK = (1 << 48) - 1

    def __init__(self, seed: int):
        self.seed = (seed ^ self.MULT) & self.MASK

    def next(self, bits: int) -> int:
        self.seed = (self.seed * self.MULT + 0xB) & self.MASK
        r = self.seed >> (48 - bits)
        if r >= 1 << 31:
            r -= 1 << 32  # (int) cast of Java's next(32)
        return r

    def nextDouble(self) -> float:
        hi = self.next(26) & ((1 << 26) - 1)
        lo = self.next(27) & ((1 << 27) - 1)
        return ((hi << 27) + lo) * (1.0 / (1 << 53))


def java_random_signal(n: int, seed: int) -> np.ndarray:
    """`new Random(seed).nextDouble() * 2 - 1` per sample, the reference tests' common input."""
    r = JavaRandom(seed)
    return np.array([r.nextDouble() * 2 - 1 for _ in range(n)])


# ---- WaveletDenoiser (core/denoising/WaveletDenoiser.java) -----------------------------------------
UNIVERSAL, SURE, MINIMAX, BAYES, FIXED = 0, 1, 2, 3, 4


def calc_threshold(c, sigma: float, method: int) -> float:
    """calculateThreshold :394-436 (SURE is the reference's O(n^2) search)."""
    c = _arr(c)
    out = c_double()
    st = lib().vwo_calc_threshold(_p(c), len(c), sigma, method, ctypes.byref(out))
    if st != 0:
        raise OracleError(st)
    return out.value


def sure_risk(c, t: float, sigma: float) -> float:
    c = _arr(c)
    return lib().vwo_sure_risk(_p(c), len(c), t, sigma)


def wavelet_denoise(x, lo, hi, boundary: int, levels: int, method: int, fixed: float = 0.0, soft: bool = True,
                    wavelet_id: int = 0):
    """WaveletDenoiser.denoise (levels == 0) / denoiseFixed (levels == 0, method FIXED) / denoiseMultiLevel.
    Returns (y, thresholds[max(levels, 1)])."""
    x, lo, hi = _arr(x), _arr(lo), _arr(hi)
    y = np.empty(len(x))
    thr = np.empty(max(levels, 1))
    bad = c_longlong(-1)
    st = lib().vwo_wavelet_denoise(_p(x), len(x), _p(lo), _p(hi), len(lo), wavelet_id, boundary, levels, method, fixed,
                                   1 if soft else 0, _p(y), _p(thr), ctypes.byref(bad))
    if st != 0:
        raise OracleError(st, bad.value)
    return y, thr


# ---- MODWTStreamingDenoiser (core/modwt/streaming/MODWTStreamingDenoiser.java) ---------------------
def java_median(v) -> float:
    """MathUtils.median (core/util/MathUtils.java:94-111): exact order statistic(s), even n = mean of the
    middle pair."""
    s = np.sort(np.asarray(v, dtype=np.float64))
    n = len(s)
    return float(s[n // 2]) if n % 2 == 1 else float((s[n // 2 - 1] + s[n // 2]) / 2.0)


def java_mad_guarded(v) -> float:
    """calculateMAD (:212-241) + MathUtils.medianAbsoluteDeviation (:121-137)."""
    v = np.asarray(v, dtype=np.float64)
    fin = np.isfinite(v)
    if not fin.any() or not (v[fin] != 0.0).any():
        return 0.0
    m = java_median(v)
    return java_median(np.abs(v - m))


def java_std_guarded(v) -> float:
    """calculateSTD (:249-270) + MathUtils.standardDeviation (:233-257), sequential sums."""
    v = [float(t) for t in v]
    if sum(1 for t in v if math.isfinite(t)) < 2:
        return 0.0
    acc = 0.0
    for t in v:
        acc += t
    mean = acc / len(v)
    ssd = 0.0
    for t in v:
        d = t - mean
        ssd += d * d
    return math.sqrt(ssd / (len(v) - 1))


class StreamingDenoiserRestatement:
    """MODWTStreamingDenoiser.denoise (:94-126) for one stream: noise window update (:133-206),
    calculateThreshold (:277-326), WaveletDenoiser.denoise / denoiseFixed."""

    def __init__(self, lo, hi, boundary: int, wavelet_id: int, method: int, soft: bool, mult: float,
                 estimation: str, window: int):
        self.lo, self.hi, self.boundary, self.wid = _arr(lo), _arr(hi), boundary, wavelet_id
        self.method, self.soft, self.mult, self.est, self.w = method, soft, mult, estimation, window
        self.window = np.zeros(window)
        self.idx = 0
        self.level = 0.0

    def _positions(self, n):
        w = self.w
        if n <= w:
            return list(range(n))
        strata = min(w, 10)
        per, extra, size = w // strata, w % strata, n // strata
        out = []
        for s in range(strata):
            start = s * size
            end = n if s == strata - 1 else (s + 1) * size
            take = per + (1 if s < extra else 0)
            if take > 0:
                length = end - start
                step = max(1, length // take)
                i = 0
                while i < take and len(out) < w:
                    j = start + (i * step) % length
                    if j < n:
                        out.append(j)
                    i += 1
        rem = w - len(out)
        if rem > 0:
            i = max(0, n - rem)
            while i < n and len(out) < w:
                out.append(i)
                i += 1
        return out

    def denoise(self, x):
        x = _arr(x)
        if self.est != "FIXED":
            _, d = modwt_forward(x, self.lo, self.hi, self.boundary)
            for j in self._positions(len(d)):
                self.window[self.idx] = abs(d[j])
                self.idx = (self.idx + 1) % self.w
            if self.est == "MAD":
                self.level = java_mad_guarded(self.window) / 0.6745
            else:
                self.level = java_std_guarded(self.window)
        if abs(self.mult - 1.0) < 1e-10:
            y, _ = wavelet_denoise(x, self.lo, self.hi, self.boundary, 0, self.method, 0.0, self.soft, self.wid)
            return y
        sigma = self.level
        if sigma <= 0.0 or self.est == "FIXED":
            _, d = modwt_forward(x, self.lo, self.hi, self.boundary)
            sigma = java_mad_guarded(np.abs(d)) / 0.6745
        n = len(x)
        if self.method == UNIVERSAL:
            t = sigma * math.sqrt(2.0 * math.log(n))
        elif self.method == SURE:
            t = sigma * math.sqrt(2.0 * math.log(n)) * 0.8
        elif self.method == MINIMAX:
            ln = math.log(n)
            t = 0.0 if n <= 32 else sigma * (0.3936 + 0.1829 * ln) if n <= 64 else sigma * (0.4745 + 0.1148 * ln)
        else:
            t = sigma
        y, _ = wavelet_denoise(x, self.lo, self.hi, self.boundary, 0, FIXED, t * self.mult, self.soft, self.wid)
        return y

"""Batch facade: Python mirror of ``ext/extensions/modwt`` (BatchMODWT, BatchStreamingMODWT).

The reference converts AoS ``double[B][N]`` to SoA and runs Java Vector-API loops; here a [B, N]
array (numpy or torch CUDA) goes to the device as one launch, one workgroup per signal.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_int64, c_void_p
from dataclasses import dataclass

import numpy as np

from . import _native as nat
from .engine import Engine, _check, _is_device_tensor
from .errors import InvalidArgumentException
from .modwt import BoundaryMode, _check_boundary, _engine_for
from .wavelets import Haar, Wavelet

try:
    import torch
except Exception:  # pragma: no cover
    torch = None


def _validate_aos(signals, what: str = "signals"):
    """BatchMODWT.validateAoS :201-212."""
    if signals is None or len(signals) == 0:
        raise InvalidArgumentException(f"{what} must be non-null and non-empty")
    if isinstance(signals, (list, tuple)):
        n = len(signals[0])
        if n == 0:
            raise InvalidArgumentException("signal length must be > 0")
        for s in signals[1:]:
            if s is None or len(s) != n:
                raise InvalidArgumentException("all signals must be non-null and same length")
        if _is_device_tensor(signals[0]):
            return torch.stack(list(signals))
        return np.stack([np.asarray(s, dtype=np.float64) for s in signals])
    if signals.ndim != 2 or signals.shape[1] == 0:
        raise InvalidArgumentException("signals must be a non-empty [batch][length] array")
    return signals


def _check_batch_reach(wavelet: Wavelet, n: int, levels: int) -> None:
    """BatchSIMDMODWT.generalBatchMODWTSoAWithScaledFilters (:384-424) indexes (t - l + N) % N: with an
    upsampled filter longer than N + 1 that index goes negative and Java throws
    ArrayIndexOutOfBoundsException at the first such level (IndexError here, before any work)."""
    L = len(wavelet.lowPassDecomposition())
    for j in range(1, levels + 1):
        Lj = (L - 1) * (1 << (j - 1)) + 1
        if Lj > n + 1:
            raise IndexError(f"Index {n - Lj + 1} out of bounds for length {n} (level {j} filter length {Lj})")


@dataclass
class SingleLevelResult:
    approx: object   # [B][N]
    detail: object   # [B][N]


@dataclass
class MultiLevelResult:
    detailPerLevel: object  # [levels][B][N]
    finalApprox: object     # [B][N]


class BatchMODWT:
    """ext/extensions/modwt/BatchMODWT.java:34-213 -- PERIODIC batch MODWT, AoS in / AoS out."""

    SingleLevelResult = SingleLevelResult
    MultiLevelResult = MultiLevelResult

    @staticmethod
    def singleLevelAoS(wavelet: Wavelet, signals, fma: bool = False) -> SingleLevelResult:
        """singleLevelAoS :62-79 (BatchSIMDMODWT.batchMODWTSoA: Haar uses 0.5/-0.5 taps, :86-140)."""
        x = _validate_aos(signals)
        flags = (nat.FLAG_FMA if fma else 0) | (nat.FLAG_BATCH_HAAR if isinstance(wavelet, Haar) else 0)
        a, d = _engine_for(x).forward1(x, wavelet.lowPassDecomposition(), wavelet.highPassDecomposition(),
                                       nat.PERIODIC, flags)
        return SingleLevelResult(a, d)

    @staticmethod
    def multiLevelAoS(wavelet: Wavelet, signals, levels: int, fma: bool = False) -> MultiLevelResult:
        """multiLevelAoS :90-111 -- no level cap, no finite check (BatchSIMDMODWT :343-424)."""
        if levels < 1:
            raise InvalidArgumentException("levels must be >= 1")
        x = _validate_aos(signals)
        _check_batch_reach(wavelet, x.shape[1], levels)
        det, app = _engine_for(x).forward(x, wavelet.lowPassDecomposition(), wavelet.highPassDecomposition(),
                                          wavelet.wavelet_id, nat.PERIODIC, levels,
                                          nat.FLAG_REF_NONFINITE | (nat.FLAG_FMA if fma else 0))
        return MultiLevelResult(det, app)

    @staticmethod
    def inverseSingleLevelAoS(wavelet: Wavelet, approx, detail, fma: bool = False):
        """inverseSingleLevelAoS :122-139 -- core MODWTTransform.inverse per signal (pairwise sums)."""
        a = _validate_aos(approx, "approx")
        d = _validate_aos(detail, "detail")
        if a.shape != d.shape:
            raise InvalidArgumentException("approx/detail shapes must match")
        return _engine_for(a).inverse1(a, d, wavelet.lowPassReconstruction(), wavelet.highPassReconstruction(),
                                       nat.PERIODIC, nat.FLAG_FMA if fma else 0)

    @staticmethod
    def inverseMultiLevelAoS(wavelet: Wavelet, detailPerLevel, finalApprox, fma: bool = False):
        """inverseMultiLevelAoS :151-178 -- core MultiLevelMODWTTransform.reconstruct (PERIODIC) per signal."""
        if detailPerLevel is None or len(detailPerLevel) == 0:
            raise InvalidArgumentException("levels must be > 0")
        app = _validate_aos(finalApprox, "finalApprox")
        if isinstance(detailPerLevel, (list, tuple)):
            det = (torch.stack([_validate_aos(l) for l in detailPerLevel]) if _is_device_tensor(app)
                   else np.stack([_validate_aos(l) for l in detailPerLevel]))
        else:
            det = detailPerLevel
        if tuple(det.shape[1:]) != tuple(app.shape):
            raise InvalidArgumentException("detailPerLevel[L] must be non-null and length=batch for all L")
        J = det.shape[0]
        return _engine_for(app).inverse(det, app, wavelet.lowPassReconstruction(), wavelet.highPassReconstruction(),
                                        wavelet.wavelet_id, nat.PERIODIC, J,
                                        nat.FLAG_CORE_LEVELS | nat.FLAG_REF_NONFINITE | (nat.FLAG_FMA if fma else 0))


class BatchSIMDMODWT:
    """ext/extensions/modwt/BatchSIMDMODWT.java -- the facade's Structure-of-Arrays entry points.

    SoA layout: one flat array, element t of signal b at index t*batchSize + b.  On the device the
    layout change is a tiled transpose (vw_transpose_*, HBM-bound); the transforms run on the AoS
    kernels, whose per-signal arithmetic is the reference's per-lane arithmetic (mul then add, taps
    ascending).  Returns arrays instead of filling caller arrays.
    """

    @staticmethod
    def convertToSoA(signals):
        """convertToSoA :282-292: [B][N] -> flat [N*B]."""
        x = _validate_aos(signals)
        B, N = x.shape
        return _engine_for(x).transpose(x, B, N)

    @staticmethod
    def convertFromSoA(soaData, batchSize: int, signalLength: int):
        """convertFromSoA :299-308: flat [N*B] -> [B][N]."""
        eng = _engine_for(soaData)
        return eng.transpose(soaData, signalLength, batchSize).reshape(batchSize, signalLength)

    @staticmethod
    def batchMODWTSoA(soaSignals, wavelet: Wavelet, batchSize: int, signalLength: int, fma: bool = False):
        """batchMODWTSoA :64-84 (Haar: 0.5/-0.5 taps :86-140).  Returns (soaApprox, soaDetail)."""
        r = BatchMODWT.singleLevelAoS(wavelet, BatchSIMDMODWT.convertFromSoA(soaSignals, batchSize, signalLength),
                                      fma=fma)
        eng = _engine_for(r.approx)
        return (eng.transpose(r.approx, batchSize, signalLength), eng.transpose(r.detail, batchSize, signalLength))

    @staticmethod
    def batchMultiLevelMODWTSoA(soaSignals, wavelet: Wavelet, batchSize: int, signalLength: int, levels: int,
                                fma: bool = False):
        """batchMultiLevelMODWTSoA :343-381.  Returns (soaDetailPerLevel [levels][N*B], soaApproxOut [N*B])."""
        r = BatchMODWT.multiLevelAoS(wavelet, BatchSIMDMODWT.convertFromSoA(soaSignals, batchSize, signalLength),
                                     levels, fma=fma)
        eng = _engine_for(r.finalApprox)
        det = [eng.transpose(r.detailPerLevel[j], batchSize, signalLength) for j in range(levels)]
        stack = torch.stack if _is_device_tensor(r.finalApprox) else np.stack
        return stack(det), eng.transpose(r.finalApprox, batchSize, signalLength)


class BatchStreamingMODWT:
    """ext/extensions/modwt/BatchStreamingMODWT.java:19-400.

    PERIODIC: independent blocks.  ZERO_PADDING / SYMMETRIC: per-level left history kept on the
    device (vw_stream), initialised from the first block, carried across blocks, flushable.
    """

    class Builder:
        def __init__(self):
            self._wavelet = None
            self._boundary = BoundaryMode.PERIODIC
            self._levels = 1

        def wavelet(self, w: Wavelet):
            self._wavelet = w
            return self

        def boundary(self, b: BoundaryMode):
            self._boundary = b
            return self

        def levels(self, n: int):
            self._levels = n
            return self

        def build(self) -> "BatchStreamingMODWT":
            return BatchStreamingMODWT(self._wavelet, self._boundary, self._levels)

    @staticmethod
    def builder() -> "BatchStreamingMODWT.Builder":
        return BatchStreamingMODWT.Builder()

    def __init__(self, wavelet: Wavelet, boundaryMode: BoundaryMode = BoundaryMode.PERIODIC, levels: int = 1,
                 device: int | None = None):
        if wavelet is None:
            raise TypeError("wavelet cannot be null")
        if levels < 1:
            raise InvalidArgumentException("levels must be >= 1")
        _check_boundary(boundaryMode)
        self.wavelet = wavelet
        self.boundaryMode = BoundaryMode(boundaryMode)
        self.levels = levels
        self._engine = Engine.get(device)
        h = c_void_p()
        lo, hi = wavelet.lowPassDecomposition(), wavelet.highPassDecomposition()
        _check(self._engine.lib.vw_stream_create(self._engine.ctx, nat.taps_array(lo), nat.taps_array(hi), len(lo),
                                                 int(self.boundaryMode), levels, byref(h)))
        self._h = h

    def close(self) -> None:
        if self._h:
            _check(self._engine.lib.vw_stream_destroy(self._h))
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _ensure_levels(self, expected: int) -> None:
        if self.levels != expected:
            from .errors import InvalidStateException
            raise InvalidStateException(f"This instance is configured for levels={self.levels}, expected={expected}")

    def _process(self, block):
        x = _validate_aos(block, "block")
        xa, dev, xp, _ = self._engine._prep(x, np.float64)
        B, n = xa.shape
        det = self._engine._empty(xa, dev, (self.levels, B, n))
        app = self._engine._empty(xa, dev, (B, n))
        # the reference's NaN spread through the zero taps (BatchMODWT blocks for PERIODIC; for ZERO /
        # SYMMETRIC the history-convolution loop, BatchSIMDMODWT.java:447-507, multiplies every tap too)
        fl = (0 if dev else nat.FLAG_HOST_MEMORY) | nat.FLAG_REF_NONFINITE
        _check(self._engine.lib.vw_stream_process_f64(self._h, xp, B, n, fl,
                                                      self._engine._ptr(det, dev), self._engine._ptr(app, dev)))
        self._B = B  # batch of the last block (sizes the host outputs of a flush)
        return det, app, dev

    def processSingleLevel(self, block) -> SingleLevelResult:
        """processSingleLevel :55-102 (PERIODIC -> BatchMODWT.singleLevelAoS)."""
        self._ensure_levels(1)
        if self.boundaryMode == BoundaryMode.PERIODIC:
            return BatchMODWT.singleLevelAoS(self.wavelet, block)
        det, app, _ = self._process(block)
        return SingleLevelResult(app, det[0])

    def processMultiLevel(self, block) -> MultiLevelResult:
        """processMultiLevel :110-164."""
        if self.boundaryMode == BoundaryMode.PERIODIC:
            return BatchMODWT.multiLevelAoS(self.wavelet, block, self.levels)
        det, app, _ = self._process(block)
        return MultiLevelResult(det, app)

    def _flush(self, tailLength: int, host: bool = True):
        B = self._last_batch()
        det = np.empty((self.levels, B, tailLength))
        app = np.empty((B, tailLength))
        _check(self._engine.lib.vw_stream_flush_f64(self._h, tailLength, nat.FLAG_HOST_MEMORY | nat.FLAG_REF_NONFINITE,
                                                    det.ctypes.data_as(c_void_p), app.ctypes.data_as(c_void_p)))
        return det, app

    def _last_batch(self) -> int:
        B = getattr(self, "_B", 0)
        if B <= 0:
            from .errors import InvalidStateException
            raise InvalidStateException("No prior blocks processed; cannot flush")
        return B

    def flushSingleLevel(self, tailLength: int) -> SingleLevelResult:
        """flushSingleLevel :181-222."""
        self._ensure_levels(1)
        if self.boundaryMode == BoundaryMode.PERIODIC:
            raise NotImplementedError("Flush is only applicable to ZERO_PADDING/SYMMETRIC")
        if tailLength <= 0:
            return SingleLevelResult(np.zeros((0, 0)), np.zeros((0, 0)))
        det, app = self._flush(tailLength)
        return SingleLevelResult(app, det[0])

    def flushMultiLevel(self, tailLength: int) -> MultiLevelResult:
        """flushMultiLevel :231-275."""
        if self.boundaryMode == BoundaryMode.PERIODIC:
            raise NotImplementedError("Flush is only applicable to ZERO_PADDING/SYMMETRIC")
        if tailLength <= 0:
            return MultiLevelResult(np.zeros((self.levels, 0, 0)), np.zeros((0, 0)))
        det, app = self._flush(tailLength)
        return MultiLevelResult(det, app)

    def getMinFlushTailLength(self) -> int:
        return min(self.getHistoryLengthForLevel(j) for j in range(1, self.levels + 1))

    def getHistoryLengthForLevel(self, level: int) -> int:
        if level < 1 or level > self.levels:
            raise InvalidArgumentException(f"level must be in [1,{self.levels}]")
        return int(self._engine.lib.vw_stream_history_length(self._h, level))

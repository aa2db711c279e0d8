"""Streaming MODWT: Python mirror of ``core/modwt/streaming`` (MODWTStreamingTransform, its Impl and
MultiLevelMODWTStreamingTransform) on the HIP engine.

The reference pushes samples one at a time through a circular buffer and transforms each window as it
fills.  Here ``process(data)`` finds every window the new samples complete and transforms them in ONE
batched device call (the windows are independent signals), then publishes the results in stream
order -- the same windows, the same numbers, one launch instead of one JVM transform per window.

Flow API: ``subscribe(s)`` takes a ``java.util.concurrent.Flow.Subscriber``-like object (``onNext``,
optional ``onComplete`` / ``onError`` / ``onSubscribe``) or a plain callable (``onNext``).
"""
from __future__ import annotations

import enum
import time

import numpy as np

from . import _native as nat
from .errors import InvalidArgumentException, InvalidSignalException, InvalidStateException
from .modwt import BoundaryMode, MODWTResult, MultiLevelMODWTTransform, _check_boundary, _engine_for
from .wavelets import Wavelet


class StreamingStatistics:
    """MODWTStreamingTransform.StreamingStatistics (:154-190): counters of the stream."""

    def __init__(self):
        self.reset()

    def reset(self) -> None:
        self._samples = 0
        self._blocks = 0
        self._ns = 0

    def _record(self, samples: int, blocks: int, ns: int) -> None:
        self._samples += samples
        self._blocks += blocks
        self._ns += ns

    def getSamplesProcessed(self) -> int:
        return self._samples

    def getBlocksProcessed(self) -> int:
        return self._blocks

    def getAverageProcessingTime(self) -> float:
        """Nanoseconds per block (a batched call's time is shared by its blocks)."""
        return self._ns / self._blocks if self._blocks else 0.0


class _Publisher:
    """The Flow.Publisher half of SubmissionPublisher, synchronously delivered."""

    def __init__(self):
        self._subs = []

    def subscribe(self, subscriber) -> None:
        if subscriber is None:
            raise TypeError("subscriber cannot be null")
        self._subs.append(subscriber)
        if hasattr(subscriber, "onSubscribe"):
            subscriber.onSubscribe(self)

    def hasSubscribers(self) -> bool:
        return bool(self._subs)

    def _submit(self, item) -> None:
        for s in self._subs:
            (s.onNext if hasattr(s, "onNext") else s)(item)

    def _complete(self) -> None:
        for s in self._subs:
            if hasattr(s, "onComplete"):
                s.onComplete()


class MODWTStreamingTransform:
    """core/modwt/streaming/MODWTStreamingTransform.java factories (:61-97)."""

    DEFAULT_BUFFER_SIZE = 256

    @staticmethod
    def create(wavelet: Wavelet, boundaryMode: BoundaryMode, bufferSize: int = DEFAULT_BUFFER_SIZE):
        return MODWTStreamingTransformImpl(wavelet, boundaryMode, bufferSize)

    @staticmethod
    def createMultiLevel(wavelet: Wavelet, boundaryMode: BoundaryMode, bufferSize: int, levels: int):
        return MultiLevelMODWTStreamingTransform(wavelet, boundaryMode, bufferSize, levels)


class _StreamBase(_Publisher):
    def __init__(self, wavelet, boundaryMode, bufferSize: int):
        super().__init__()
        if wavelet is None:
            raise InvalidArgumentException("Wavelet cannot be null")
        if boundaryMode is None:
            raise InvalidArgumentException("Boundary mode cannot be null")
        if bufferSize <= 0:
            raise InvalidArgumentException(f"Buffer size must be positive, got: {bufferSize}")
        _check_boundary(BoundaryMode(boundaryMode))
        self.wavelet = wavelet
        self.boundaryMode = BoundaryMode(boundaryMode)
        self.bufferSize = int(bufferSize)
        self._pending = np.empty(0)
        self._closed = False
        self.statistics = StreamingStatistics()

    def _check_open(self) -> None:
        if self._closed:
            raise InvalidStateException("Transform is closed")

    def process(self, data) -> None:
        self._check_open()
        if data is None or len(data) == 0:
            raise InvalidSignalException("Data cannot be null or empty")
        self._pending = np.concatenate([self._pending, np.asarray(data, dtype=np.float64).ravel()])
        n = len(data)
        t0 = time.perf_counter_ns()
        blocks = self._drain()
        self.statistics._record(n, blocks, time.perf_counter_ns() - t0)

    def processSample(self, sample: float) -> None:
        self.process(np.array([sample], dtype=np.float64))

    def getBufferLevel(self) -> int:
        return int(len(self._pending))

    def getStatistics(self) -> StreamingStatistics:
        return self.statistics

    def isClosed(self) -> bool:
        return self._closed

    def reset(self) -> None:
        self._check_open()
        self._pending = np.empty(0)
        self.statistics.reset()

    def flush(self) -> None:
        self._check_open()
        self._flush()

    def close(self) -> None:
        if not self._closed:
            self._flush()
            self._closed = True
            self._complete()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _flush(self) -> None:
        """Remaining samples, zero-padded to one buffer (MODWTStreamingTransformImpl.flush :228-252)."""
        if len(self._pending) == 0:
            return
        block = np.zeros((1, self.bufferSize))
        block[0, :len(self._pending)] = self._pending
        self._pending = np.empty(0)
        self._publish(block)
        self.statistics._record(0, 1, 0)


class MODWTStreamingTransformImpl(_StreamBase):
    """core/modwt/streaming/MODWTStreamingTransformImpl.java -- sliding windows of bufferSize samples
    that overlap by L-1 (:75-136), each transformed by MODWTTransform.forward (:188-198)."""

    def __init__(self, wavelet: Wavelet, boundaryMode: BoundaryMode, bufferSize: int):
        super().__init__(wavelet, boundaryMode, bufferSize)
        L = len(wavelet.lowPassDecomposition())
        self.filterLength = L
        self.overlapSize = L - 1
        if (bufferSize + self.overlapSize) * 8 > 100 * 1024 * 1024:
            raise InvalidArgumentException("Buffer size too large, would require more than 100MB")
        if bufferSize < L:
            raise InvalidArgumentException(
                f"Buffer size must be at least as large as filter length: bufferSize={bufferSize}, filterLength={L}")
        self.hop = bufferSize - self.overlapSize  # samples consumed per window (:202-218)

    def _drain(self) -> int:
        n = len(self._pending)
        if n < self.bufferSize:
            return 0
        k = 1 + (n - self.bufferSize) // self.hop
        idx = np.arange(k)[:, None] * self.hop + np.arange(self.bufferSize)[None, :]
        self._publish(self._pending[idx])
        self._pending = self._pending[k * self.hop:]
        return k

    def _publish(self, windows: np.ndarray) -> None:
        w = self.wavelet
        a, d = _engine_for(windows).forward1(windows, w.lowPassDecomposition(), w.highPassDecomposition(),
                                              int(self.boundaryMode), nat.FLAG_VALIDATE)
        for b in range(windows.shape[0]):
            self._submit(MODWTResult(a[b], d[b]))


class MODWTResultWrapper:
    """MultiLevelMODWTStreamingTransform.MODWTResultWrapper (:256-290): a level's details with the final
    approximation, or an empty approximation below the last level."""

    def __init__(self, approx, details):
        self._a = approx
        self._d = details

    def approximationCoeffs(self):
        return self._a.copy()

    def detailCoeffs(self):
        return self._d.copy()

    def getSignalLength(self) -> int:
        return int(len(self._d))

    def isValid(self) -> bool:
        return bool(np.isfinite(self._a).all() and np.isfinite(self._d).all())


class MultiLevelMODWTStreamingTransform(_StreamBase):
    """core/modwt/streaming/MultiLevelMODWTStreamingTransform.java -- non-overlapping blocks of bufferSize
    samples, each decomposed to `levels` (MultiLevelMODWTTransform.decompose, :133-166); per block one
    MODWTResult per level: that level's details, and the approximation at the last level only
    (getApproximationForLevel :238-240)."""

    def __init__(self, wavelet: Wavelet, boundaryMode: BoundaryMode, bufferSize: int, levels: int):
        super().__init__(wavelet, boundaryMode, bufferSize)
        if levels < 1:
            raise InvalidArgumentException(f"Levels must be at least 1, got: {levels}")
        self.levels = int(levels)
        self._tx = MultiLevelMODWTTransform(wavelet, self.boundaryMode)

    def _drain(self) -> int:
        k = len(self._pending) // self.bufferSize
        if k == 0:
            return 0
        self._publish(self._pending[:k * self.bufferSize].reshape(k, self.bufferSize))
        self._pending = self._pending[k * self.bufferSize:]
        return k

    def _publish(self, blocks: np.ndarray) -> None:
        res = self._tx.decompose(blocks, self.levels)
        det, app = res.details_array, res.approximation_array
        empty = np.empty(0)
        for b in range(blocks.shape[0]):
            for level in range(1, self.levels + 1):
                self._submit(MODWTResultWrapper(app[b] if level == self.levels else empty, det[level - 1, b]))


class MODWTStreamingDenoiser:
    """core/modwt/streaming/MODWTStreamingDenoiser.java -- block-by-block denoising with a running noise
    estimate (a Flow.Publisher of the denoised blocks).

    denoise(samples) (:94-126): unless noiseEstimation is FIXED, the block's single-level MODWT details
    (MODWTTransform.forward) update a ring window of |d| (all of them, or the reference's stratified
    sample when the block has more details than the window, :133-206) and the noise level becomes
    MAD(window)/0.6745 or STD(window) (MathUtils.medianAbsoluteDeviation / standardDeviation).  With a
    threshold multiplier of 1 the block is denoised by WaveletDenoiser.denoise (its own sigma); otherwise
    by denoiseFixed with calculateThreshold(samples) * multiplier (:277-326).

    On the device: the forward, the ring update (vw_window_gather_abs_f64; the window stays in HBM
    between blocks), the exact medians (vw_median_f64, two passes for the MAD), the sequential standard
    deviation (vw_stddev_f64) and the denoise pipeline (vw_wavelet_denoise_f64).  The host keeps the
    integer bookkeeping (ring index, stratified positions) and the scalar threshold formulas.
    """

    class NoiseEstimation(enum.Enum):
        MAD = "MAD"
        STD = "STD"
        FIXED = "FIXED"

    class Builder:
        def __init__(self):
            from .denoise import ThresholdMethod, ThresholdType
            from .wavelets import Daubechies
            self._wavelet = Daubechies.DB4
            self._boundary = BoundaryMode.PERIODIC
            self._bufferSize = 256
            self._type = ThresholdType.SOFT
            self._method = ThresholdMethod.UNIVERSAL
            self._mult = 1.0
            self._noise = MODWTStreamingDenoiser.NoiseEstimation.MAD
            self._window = 1024

        def _need(self, v, what):
            if v is None:
                raise InvalidArgumentException(f"{what} cannot be null")
            return v

        def wavelet(self, w):
            self._wavelet = self._need(w, "Wavelet")
            return self

        def boundaryMode(self, b):
            self._boundary = BoundaryMode(self._need(b, "Boundary mode"))
            return self

        def bufferSize(self, n: int):
            if n <= 0:
                raise InvalidArgumentException("Buffer size must be positive")
            self._bufferSize = int(n)
            return self

        def thresholdType(self, t):
            self._type = self._need(t, "Threshold type")
            return self

        def thresholdMethod(self, m):
            self._method = self._need(m, "Threshold method")
            return self

        def thresholdMultiplier(self, x: float):
            if x <= 0:
                raise InvalidArgumentException("Threshold multiplier must be positive")
            self._mult = float(x)
            return self

        def noiseEstimation(self, e):
            self._noise = self._need(e, "Noise estimation")
            return self

        def noiseWindowSize(self, n: int):
            if n <= 0:
                raise InvalidArgumentException("Noise window size must be positive")
            self._window = int(n)
            return self

        def build(self) -> "MODWTStreamingDenoiser":
            return MODWTStreamingDenoiser(self)

    @staticmethod
    def builder() -> "MODWTStreamingDenoiser.Builder":
        return MODWTStreamingDenoiser.Builder()

    def __init__(self, b: "MODWTStreamingDenoiser.Builder"):
        import torch
        from .denoise import WaveletDenoiser
        from .engine import Engine
        from .modwt import MODWTTransform
        self._torch = torch
        self.transform = MODWTTransform(b._wavelet, b._boundary)
        self.denoiser = WaveletDenoiser(b._wavelet, b._boundary)
        self.bufferSize = b._bufferSize
        self.thresholdType = b._type
        self.thresholdMethod = b._method
        self.thresholdMultiplier = b._mult
        self.noiseEstimation = b._noise
        self.noiseWindowSize = b._window
        self._eng = Engine.get()
        self._dev = torch.device("cuda", self._eng.device)
        self._window = (torch.zeros(self.noiseWindowSize, dtype=torch.float64, device=self._dev)
                        if self.noiseEstimation != self.NoiseEstimation.FIXED else None)
        self._widx = 0
        self._level = 0.0
        self._samples = 0
        self._closed = False
        self._subscribers = []

    # -- device statistics ---------------------------------------------------------------------------
    def _ptr(self, t):
        from ctypes import c_void_p
        return c_void_p(t.data_ptr())

    def _mad(self, vals) -> float:
        """calculateMAD (:212-241): 0 when nothing finite or every finite value is 0, else
        MathUtils.medianAbsoluteDeviation = median(|v - median(v)|) (two exact device medians)."""
        from .engine import _check
        torch = self._torch
        fin = torch.isfinite(vals)
        if not bool(fin.any()) or not bool((vals[fin] != 0).any()):
            return 0.0
        n = vals.numel()
        med = torch.empty(1, dtype=torch.float64, device=self._dev)
        mad = torch.empty(1, dtype=torch.float64, device=self._dev)
        self._eng.bind_torch_stream()
        _check(self._eng.lib.vw_median_f64(self._eng.ctx, self._ptr(vals), 1, n, None, 0, self._ptr(med)))
        _check(self._eng.lib.vw_median_f64(self._eng.ctx, self._ptr(vals), 1, n, self._ptr(med), 0, self._ptr(mad)))
        return float(mad.item())

    def _std(self, vals) -> float:
        """calculateSTD (:249-270): 0 with fewer than 2 finite values, else MathUtils.standardDeviation."""
        from .engine import _check
        if int(self._torch.isfinite(vals).sum()) < 2:
            return 0.0
        out = self._torch.empty(1, dtype=self._torch.float64, device=self._dev)
        self._eng.bind_torch_stream()
        _check(self._eng.lib.vw_stddev_f64(self._eng.ctx, self._ptr(vals), vals.numel(), 0, self._ptr(out)))
        return float(out.item())

    def _gather_abs(self, src, idx, dst, start: int) -> None:
        from ctypes import c_void_p
        from .engine import _check
        a = np.ascontiguousarray(np.asarray(idx, dtype=np.int32))
        self._eng.bind_torch_stream()
        _check(self._eng.lib.vw_window_gather_abs_f64(self._eng.ctx, self._ptr(src), a.ctypes.data_as(c_void_p),
                                                      len(a), self._ptr(dst), dst.numel(), start))

    @staticmethod
    def stratified_positions(n: int, w: int):
        """updateNoiseEstimation's detail positions (:140-200), in write order."""
        if n <= w:
            return list(range(n))
        strata = min(w, 10)
        per, extra = w // strata, w % strata
        size = n // strata
        out = []
        for s in range(strata):
            s0 = s * size
            s1 = n if s == strata - 1 else (s + 1) * size
            take = per + (1 if s < extra else 0)
            if take > 0:
                length = s1 - s0
                step = max(1, length // take)
                for i in range(take):
                    if len(out) >= w:
                        break
                    idx = s0 + (i * step) % length
                    if idx < n:
                        out.append(idx)
        remaining = w - len(out)
        if remaining > 0:
            for i in range(max(0, n - remaining), n):
                if len(out) >= w:
                    break
                out.append(i)
        return out

    def _update(self, x) -> None:
        det = self.transform.forward(x).detailCoeffs()
        pos = self.stratified_positions(det.numel(), self.noiseWindowSize)
        self._gather_abs(det, pos, self._window, self._widx)
        self._widx = (self._widx + len(pos)) % self.noiseWindowSize
        if self.noiseEstimation == self.NoiseEstimation.MAD:
            self._level = self._mad(self._window) / 0.6745
        elif self.noiseEstimation == self.NoiseEstimation.STD:
            self._level = self._std(self._window)

    def _threshold(self, x) -> float:
        """calculateThreshold (:277-326)."""
        import math
        from .denoise import ThresholdMethod
        sigma = self._level
        if sigma <= 0.0 or self.noiseEstimation == self.NoiseEstimation.FIXED:
            det = self.transform.forward(x).detailCoeffs()
            absd = self._torch.empty_like(det)
            self._gather_abs(det, range(det.numel()), absd, 0)
            sigma = self._mad(absd) / 0.6745
        n = x.numel()
        m = ThresholdMethod(self.thresholdMethod)
        if m == ThresholdMethod.UNIVERSAL:
            return sigma * math.sqrt(2.0 * math.log(n))
        if m == ThresholdMethod.SURE:
            return sigma * math.sqrt(2.0 * math.log(n)) * 0.8
        if m == ThresholdMethod.MINIMAX:
            log_n = math.log(n)
            if n <= 32:
                return 0.0
            if n <= 64:
                return sigma * (0.3936 + 0.1829 * log_n)
            return sigma * (0.4745 + 0.1148 * log_n)
        if m == ThresholdMethod.FIXED:
            return sigma
        raise InvalidArgumentException(f"Unknown threshold method: {m}")

    # -- public API ----------------------------------------------------------------------------------
    def denoise(self, samples):
        """:94-126.  A host array in -> a host array out; a CUDA tensor stays on the device."""
        if self._closed:
            raise InvalidStateException("Denoiser is closed")
        if samples is None or len(samples) == 0:
            raise InvalidArgumentException("Samples cannot be null or empty")
        torch = self._torch
        host = not (isinstance(samples, torch.Tensor) and samples.is_cuda)
        x = (torch.as_tensor(np.asarray(samples, dtype=np.float64)).to(self._dev) if host
             else samples.to(torch.float64).contiguous())
        if self.noiseEstimation != self.NoiseEstimation.FIXED:
            self._update(x)
        if abs(self.thresholdMultiplier - 1.0) < 1e-10:
            y = self.denoiser.denoise(x, self.thresholdMethod, self.thresholdType)
        else:
            y = self.denoiser.denoiseFixed(x, self._threshold(x) * self.thresholdMultiplier, self.thresholdType)
        self._samples += x.numel()
        out = y.cpu().numpy() if host else y
        for s in list(self._subscribers):
            s(out.copy() if host else out.clone())
        return out

    def getEstimatedNoiseLevel(self) -> float:
        return self._level

    def getSamplesProcessed(self) -> int:
        return self._samples

    def subscribe(self, subscriber) -> None:
        """Flow.Publisher.subscribe: `subscriber(block)` is called with every denoised block."""
        self._subscribers.append(subscriber)

    def close(self) -> None:
        self._closed = True
        self._subscribers.clear()

    def isClosed(self) -> bool:
        return self._closed

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


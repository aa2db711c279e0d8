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

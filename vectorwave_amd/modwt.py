"""MODWT transforms: Python mirror of VectorWave's ``core/modwt`` API, backed by the HIP engine.

Same class and method names, argument meaning and error behaviour as
  MODWTTransform            core/modwt/MODWTTransform.java
  MultiLevelMODWTTransform  core/modwt/MultiLevelMODWTTransform.java
  MODWTResult / MultiLevelMODWTResult / MutableMultiLevelMODWTResult  (core/modwt/*.java)
Inputs may be numpy arrays (host; results come back as numpy) or torch CUDA tensors (device; results
stay in HBM).  A 2-D input [B, N] is a batch of B equal-length signals processed by one launch.
"""
from __future__ import annotations

import enum
from typing import List, Optional, Sequence

import numpy as np

from . import _native as nat
from .engine import Engine, _is_device_tensor, max_levels as _max_levels
from .errors import ErrorCode, InvalidArgumentException, InvalidSignalException
from .wavelets import Wavelet

try:
    import torch
except Exception:  # pragma: no cover
    torch = None


class BoundaryMode(enum.IntEnum):
    """core/api/BoundaryMode.java:20-50 (C-ABI numbering)."""
    PERIODIC = nat.PERIODIC
    SYMMETRIC = nat.SYMMETRIC
    ZERO_PADDING = nat.ZERO_PADDING
    CONSTANT = 3


def _check_boundary(mode: BoundaryMode) -> None:
    if mode not in (BoundaryMode.PERIODIC, BoundaryMode.SYMMETRIC, BoundaryMode.ZERO_PADDING):
        raise InvalidArgumentException("MODWT only supports PERIODIC, ZERO_PADDING, and SYMMETRIC boundary modes",
                                       ErrorCode.CFG_UNSUPPORTED_BOUNDARY_MODE)


def _copy(a):
    return a.clone() if _is_device_tensor(a) else np.array(a, copy=True)


def _energy(a) -> float:
    """computeEnergy (MultiLevelMODWTResultImpl.java:211-216): ``energy += c * c`` in index order -- each
    square rounded, then added to the running sum, left to right.  ``np.add.accumulate`` is that
    sequential loop (a reduction like ``np.sum`` / ``np.dot`` would sum pairwise), so the value is the
    reference's bit for bit.  A device tensor is read back first: energies are host-side scalars."""
    if _is_device_tensor(a):
        a = a.detach().double().cpu().numpy()
    a = np.asarray(a, dtype=np.float64).ravel()
    if a.size == 0:
        return 0.0
    return float(np.add.accumulate(a * a)[-1])


def _total_energy(res) -> float:
    """getTotalEnergy (MultiLevelMODWTResultImpl.java:109-117): total = approximation energy, then
    total += the detail energy of level 1, 2, ..., J."""
    total = res.getApproximationEnergy()
    for j in range(1, res.getLevels() + 1):
        total += res.getDetailEnergyAtLevel(j)
    return total


def _length(x) -> int:
    return int(x.shape[-1])


# ----------------------------------------------------------------------------------------------
class MODWTResult:
    """core/modwt/MODWTResult.java:36-100 -- getters return defensive copies."""

    def __init__(self, approximation, detail):
        if approximation.shape != detail.shape:
            raise ValueError("Approximation and detail coefficients must have the same length")
        self._a = approximation
        self._d = detail

    @staticmethod
    def create(approximation, detail) -> "MODWTResult":
        return MODWTResult(approximation, detail)

    def approximationCoeffs(self):
        return _copy(self._a)

    def detailCoeffs(self):
        return _copy(self._d)

    def getSignalLength(self) -> int:
        return _length(self._a)

    def isValid(self) -> bool:
        if _is_device_tensor(self._a):
            return bool(torch.isfinite(self._a).all().item() and torch.isfinite(self._d).all().item())
        return bool(np.isfinite(self._a).all() and np.isfinite(self._d).all())


class MultiLevelMODWTResult:
    """core/modwt/MultiLevelMODWTResult.java:25-85.  details stored [J, (B,) N], level 1 first."""

    def __init__(self, details, approximation):
        self._det = details
        self._app = approximation

    def getLevels(self) -> int:
        return int(self._det.shape[0])

    def getSignalLength(self) -> int:
        return _length(self._app)

    def getDetailCoeffsAtLevel(self, level: int):
        if level < 1 or level > self.getLevels():
            raise InvalidArgumentException(f"Invalid level {level}", ErrorCode.CFG_INVALID_DECOMPOSITION_LEVEL)
        return _copy(self._det[level - 1])

    def getApproximationCoeffs(self):
        return _copy(self._app)

    def getDetailEnergyAtLevel(self, level: int) -> float:
        return _energy(self._det[level - 1])

    def getApproximationEnergy(self) -> float:
        return _energy(self._app)

    def getTotalEnergy(self) -> float:
        return _total_energy(self)

    def getRelativeEnergyDistribution(self) -> List[float]:
        # immutable impl order: [approx, d1..dJ]  (core/modwt/MultiLevelMODWTResultImpl.java:121-138)
        tot = self.getTotalEnergy()
        J = self.getLevels()
        if tot == 0:
            return [0.0] * (J + 1)
        return [self.getApproximationEnergy() / tot] + [self.getDetailEnergyAtLevel(j) / tot for j in range(1, J + 1)]

    def isValid(self) -> bool:
        if _is_device_tensor(self._app):
            return bool(torch.isfinite(self._app).all().item() and torch.isfinite(self._det).all().item())
        return bool(np.isfinite(self._app).all() and np.isfinite(self._det).all())

    def copy(self) -> "MultiLevelMODWTResult":
        return type(self)(_copy(self._det), _copy(self._app))

    # raw (no-copy) access for the engine
    @property
    def details_array(self):
        return self._det

    @property
    def approximation_array(self):
        return self._app


class MutableMultiLevelMODWTResult(MultiLevelMODWTResult):
    """core/modwt/MutableMultiLevelMODWTResult.java:19-123 -- in-place coefficient access."""

    def getMutableDetailCoeffs(self, level: int):
        if level < 1 or level > self.getLevels():
            raise InvalidArgumentException(f"Invalid level {level}", ErrorCode.CFG_INVALID_DECOMPOSITION_LEVEL)
        return self._det[level - 1]

    def getMutableApproximationCoeffs(self):
        return self._app

    def setDetailCoeffs(self, level: int, coeffs) -> None:
        self._det[level - 1][...] = coeffs

    def setApproximationCoeffs(self, coeffs) -> None:
        self._app[...] = coeffs

    def applyThreshold(self, level: int, threshold: float, soft: bool) -> None:
        """MutableMultiLevelMODWTResult.applyThreshold :83-92 (level 0 = approximation), on the device."""
        arr = self._app if level == 0 else self.getMutableDetailCoeffs(level)
        rows = arr if arr.ndim == 2 else arr.reshape(1, -1)
        B = rows.shape[0]
        if _is_device_tensor(arr):
            thr = torch.full((B,), float(threshold), dtype=torch.float64, device=arr.device)
        else:
            thr = np.full((B,), float(threshold))
        Engine.get(arr.device.index if _is_device_tensor(arr) else None).threshold_inplace(rows, thr, soft)

    def clearCaches(self) -> None:
        pass

    def getRelativeEnergyDistribution(self) -> List[float]:
        # mutable impl order: [d1..dJ, approx]  (core/modwt/MutableMultiLevelMODWTResultImpl.java:191-208)
        tot = self.getTotalEnergy()
        J = self.getLevels()
        if tot == 0:
            return [0.0] * (J + 1)
        return [self.getDetailEnergyAtLevel(j) / tot for j in range(1, J + 1)] + [self.getApproximationEnergy() / tot]

    def toImmutable(self) -> MultiLevelMODWTResult:
        return MultiLevelMODWTResult(_copy(self._det), _copy(self._app))


def _engine_for(x) -> Engine:
    return Engine.get(x.device.index if _is_device_tensor(x) else None)


def _validate_signal(x) -> None:
    if x is None:
        raise TypeError("signal cannot be null")
    if _length(x) == 0:
        raise InvalidSignalException("Signal cannot be empty", ErrorCode.VAL_EMPTY)


# ----------------------------------------------------------------------------------------------
class MODWTTransform:
    """core/modwt/MODWTTransform.java -- single-level MODWT (any N >= 1, pairwise inverse sums)."""

    def __init__(self, wavelet: Wavelet, boundaryMode: BoundaryMode, fma: bool = False):
        if wavelet is None or boundaryMode is None:
            raise TypeError("wavelet / boundaryMode cannot be null")
        _check_boundary(boundaryMode)
        self.wavelet = wavelet
        self.boundaryMode = BoundaryMode(boundaryMode)
        self._fma = nat.FLAG_FMA if fma else 0

    def getWavelet(self) -> Wavelet:
        return self.wavelet

    def getBoundaryMode(self) -> BoundaryMode:
        return self.boundaryMode

    def forward(self, signal) -> MODWTResult:
        """MODWTTransform.forward :131-189 (validation :369-414)."""
        _validate_signal(signal)
        w = self.wavelet
        a, d = _engine_for(signal).forward1(signal, w.lowPassDecomposition(), w.highPassDecomposition(),
                                            int(self.boundaryMode), nat.FLAG_VALIDATE | self._fma)
        return MODWTResult(a, d)

    def inverse(self, modwtResult: MODWTResult, batch_optimized: bool = False):
        """MODWTTransform.inverse :203-299 (batch_optimized: inverseBatchOptimized :619-689)."""
        if modwtResult is None:
            raise TypeError("modwtResult cannot be null")
        if not modwtResult.isValid():
            raise InvalidSignalException("MODWTResult contains invalid coefficients", ErrorCode.VAL_NON_FINITE_VALUES)
        w = self.wavelet
        flags = self._fma | (nat.FLAG_BATCH_SYM_INVERSE if batch_optimized else 0)
        return _engine_for(modwtResult._a).inverse1(modwtResult._a, modwtResult._d, w.lowPassReconstruction(),
                                                   w.highPassReconstruction(), int(self.boundaryMode), flags)

    def forwardBatch(self, signals) -> List[MODWTResult]:
        """MODWTTransform.forwardBatch :486-514: same-length batches go to the device in one launch."""
        if signals is None:
            raise TypeError("signals array cannot be null")
        if len(signals) == 0:
            return []
        lengths = {_length(s) for s in signals}
        if len(lengths) == 1 and not isinstance(signals, list):
            a, d = self._forward_rows(signals)
            return [MODWTResult(a[i], d[i]) for i in range(a.shape[0])]
        if len(lengths) == 1:
            stack = torch.stack(list(signals)) if _is_device_tensor(signals[0]) else np.stack([np.asarray(s) for s in signals])
            a, d = self._forward_rows(stack)
            return [MODWTResult(a[i], d[i]) for i in range(a.shape[0])]
        return [self.forward(s) for s in signals]

    def _forward_rows(self, x):
        w = self.wavelet
        return _engine_for(x).forward1(x, w.lowPassDecomposition(), w.highPassDecomposition(), int(self.boundaryMode),
                                       nat.FLAG_VALIDATE | self._fma)

    def inverseBatch(self, results: Sequence[MODWTResult]):
        """MODWTTransform.inverseBatch :531-559 (same length, B >= 4, N >= 64 -> inverseBatchOptimized)."""
        if results is None:
            raise TypeError("results array cannot be null")
        if len(results) == 0:
            return []
        n0 = results[0].getSignalLength()
        same = all(r.getSignalLength() == n0 for r in results)
        if same and len(results) >= 4 and n0 >= 64:
            dev = _is_device_tensor(results[0]._a)
            A = torch.stack([r._a for r in results]) if dev else np.stack([r._a for r in results])
            D = torch.stack([r._d for r in results]) if dev else np.stack([r._d for r in results])
            w = self.wavelet
            y = _engine_for(A).inverse1(A, D, w.lowPassReconstruction(), w.highPassReconstruction(),
                                         int(self.boundaryMode), self._fma | nat.FLAG_BATCH_SYM_INVERSE)
            return [y[i] for i in range(y.shape[0])]
        return [self.inverse(r) for r in results]


# ----------------------------------------------------------------------------------------------
class MultiLevelMODWTTransform:
    """core/modwt/MultiLevelMODWTTransform.java -- pyramid cascade, level cap 9, FFT-switch region."""

    MAX_DECOMPOSITION_LEVELS = 10

    def __init__(self, wavelet: Wavelet, boundaryMode: BoundaryMode, fma: bool = False):
        if wavelet is None or boundaryMode is None:
            raise TypeError("wavelet / boundaryMode cannot be null")
        _check_boundary(boundaryMode)
        self.wavelet = wavelet
        self.boundaryMode = BoundaryMode(boundaryMode)
        self._fma = nat.FLAG_FMA if fma else 0

    def getWavelet(self) -> Wavelet:
        return self.wavelet

    def getBoundaryMode(self) -> BoundaryMode:
        return self.boundaryMode

    def getMaximumLevels(self, signalLength: int) -> int:
        return _max_levels(signalLength, self.wavelet.filter_length)

    @staticmethod
    def getMaxDecompositionLevels() -> int:
        return MultiLevelMODWTTransform.MAX_DECOMPOSITION_LEVELS

    def _decompose_arrays(self, signal, levels: Optional[int]):
        _validate_signal(signal) if signal is not None else None
        if levels is None:
            levels = self.getMaximumLevels(_length(signal))
        w = self.wavelet
        flags = nat.FLAG_CORE_LEVELS | nat.FLAG_VALIDATE | nat.FLAG_FFT_SWITCH | self._fma
        return _engine_for(signal).forward(signal, w.lowPassDecomposition(), w.highPassDecomposition(), w.wavelet_id,
                                           int(self.boundaryMode), levels, flags)

    def decompose(self, signal, levels: Optional[int] = None) -> MultiLevelMODWTResult:
        """decompose :195-255."""
        det, app = self._decompose_arrays(signal, levels)
        return MultiLevelMODWTResult(det, app)

    def decomposeMutable(self, signal, levels: Optional[int] = None) -> MutableMultiLevelMODWTResult:
        """decomposeMutable :267-330."""
        det, app = self._decompose_arrays(signal, levels)
        return MutableMultiLevelMODWTResult(det, app)

    def _reconstruct(self, result: MultiLevelMODWTResult, mask: int, approx_zero: bool, guard: bool = True):
        if result is None:
            raise TypeError("result cannot be null")
        w = self.wavelet
        J = result.getLevels()
        det = result.details_array if mask else None
        app = None if approx_zero else result.approximation_array
        return _engine_for(result.approximation_array).inverse(
            det, app, w.lowPassReconstruction(), w.highPassReconstruction(), w.wavelet_id, int(self.boundaryMode), J,
            self._fma | nat.FLAG_REF_NONFINITE | (nat.FLAG_CORE_LEVELS if guard else 0), detail_mask=mask,
            approx_zero=approx_zero,
            shape=tuple(result.approximation_array.shape))

    def reconstruct(self, result: MultiLevelMODWTResult):
        """reconstruct :339-349 (cascade J..1; K4 periodic / K5 zero / K6 symmetric)."""
        return self._reconstruct(result, (1 << result.getLevels()) - 1, False)

    def reconstructFromLevel(self, result: MultiLevelMODWTResult, startLevel: int):
        """reconstructFromLevel :361-386: levels finer than startLevel get zero details."""
        if result is None:
            raise TypeError("result cannot be null")
        J = result.getLevels()
        if startLevel < 1 or startLevel > J:
            raise InvalidArgumentException(f"Invalid start level: {startLevel}. Must be between 1 and {J}")
        mask = 0
        for lev in range(startLevel, J + 1):
            mask |= 1 << (lev - 1)
        return self._reconstruct(result, mask, False)

    def reconstructLevels(self, result: MultiLevelMODWTResult, minLevel: int, maxLevel: int):
        """reconstructLevels :398-446: only details in [minLevel, maxLevel]; approx only if J <= maxLevel."""
        if result is None:
            raise TypeError("result cannot be null")
        J = result.getLevels()
        if minLevel < 1 or maxLevel > J or minLevel > maxLevel:
            raise InvalidArgumentException("Invalid level range for partial reconstruction",
                                           ErrorCode.CFG_INVALID_DECOMPOSITION_LEVEL)
        mask = 0
        for lev in range(minLevel, maxLevel + 1):
            mask |= 1 << (lev - 1)
        return self._reconstruct(result, mask, not (J <= maxLevel))

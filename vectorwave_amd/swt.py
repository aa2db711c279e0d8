"""SWT facade: Python mirror of ``core/swt/VectorWaveSwtAdapter.java`` on the HIP engine."""
from __future__ import annotations

import math
from typing import Optional

import numpy as np

from . import _native as nat
from .engine import Engine, _is_device_tensor
from .errors import ErrorCode, InvalidSignalException
from .modwt import (BoundaryMode, MultiLevelMODWTTransform, MutableMultiLevelMODWTResult, _check_boundary,
                    _engine_for, _length)
from .wavelets import Wavelet

try:
    import torch
except Exception:  # pragma: no cover
    torch = None


class VectorWaveSwtAdapter:
    """SWT (== MODWT) with mutable coefficients, thresholding and denoising.

    forward   :198-394   (parallel branch N >= threshold and J > 2 skips validation and the level
                          cap, exactly like forwardParallel :210-267; its arithmetic is K1's)
    inverse   :435-487   (PERIODIC -> reconstructPeriodic; others -> MultiLevelMODWTTransform)
    denoise   :532-562   (fused on the device: forward -> exact median |d1| -> threshold -> inverse)
    """

    DEFAULT_PARALLEL_THRESHOLD = 4096

    def __init__(self, wavelet: Wavelet, boundaryMode: BoundaryMode = BoundaryMode.PERIODIC,
                 enableParallel: bool = True, parallelThreshold: int = DEFAULT_PARALLEL_THRESHOLD, fma: bool = False):
        if wavelet is None or boundaryMode is None:
            raise TypeError("Wavelet / Boundary mode cannot be null")
        self.wavelet = wavelet
        self.boundaryMode = BoundaryMode(boundaryMode)
        self.enableParallel = enableParallel
        self.parallelThreshold = parallelThreshold
        self._fma = nat.FLAG_FMA if fma else 0
        self.modwtTransform = MultiLevelMODWTTransform(wavelet, boundaryMode, fma=fma)

    # AutoCloseable
    def close(self) -> None:
        pass

    def cleanup(self) -> None:
        pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def getWavelet(self) -> Wavelet:
        return self.wavelet

    def getBoundaryMode(self) -> BoundaryMode:
        return self.boundaryMode

    def _forward_flags(self, n: int, levels: int) -> int:
        if self.enableParallel and n >= self.parallelThreshold and levels > 2:
            # forwardParallel: no validation, no level check, every upsampled tap multiplied (NaN spread)
            return self._fma | nat.FLAG_REF_NONFINITE
        return nat.FLAG_CORE_LEVELS | nat.FLAG_VALIDATE | self._fma  # decomposeSWT :337-364

    def forward(self, signal, levels: Optional[int] = None) -> MutableMultiLevelMODWTResult:
        if levels is None:
            levels = self.modwtTransform.getMaximumLevels(_length(signal))
        if _length(signal) == 0:
            raise InvalidSignalException("Signal cannot be empty for SWT", ErrorCode.VAL_EMPTY)
        w = self.wavelet
        det, app = _engine_for(signal).forward(signal, w.lowPassDecomposition(), w.highPassDecomposition(),
                                               w.wavelet_id, int(self.boundaryMode), levels,
                                               self._forward_flags(_length(signal), levels))
        return MutableMultiLevelMODWTResult(det, app)

    def inverse(self, result: MutableMultiLevelMODWTResult):
        if result is None:
            raise TypeError("Result cannot be null")
        J = result.getLevels()
        # PERIODIC: reconstructPeriodic (same SEQ sums, (t+l) % n wraps, no L_j <= N guard)
        return self.modwtTransform._reconstruct(result, (1 << J) - 1, False,
                                                guard=self.boundaryMode != BoundaryMode.PERIODIC)

    def applyThreshold(self, result: MutableMultiLevelMODWTResult, level: int, threshold: float, soft: bool) -> None:
        if result is None:
            raise TypeError("Result cannot be null")
        result.applyThreshold(level, threshold, soft)

    def estimateNoiseSigma(self, coeffs):
        """estimateNoiseSigma :627-645 (exact median on the device); one value per row."""
        return _engine_for(coeffs).noise_sigma(coeffs)

    def applyUniversalThreshold(self, result: MutableMultiLevelMODWTResult, soft: bool) -> None:
        """applyUniversalThreshold :505-520: sigma from d1, T = sigma*sqrt(2 ln N), all detail levels."""
        if result is None:
            raise TypeError("Result cannot be null")
        d1 = result.getMutableDetailCoeffs(1)
        rows = d1 if d1.ndim == 2 else d1.reshape(1, -1)
        eng = _engine_for(d1)
        sigma = eng.noise_sigma(rows)
        c = math.sqrt(2 * math.log(result.getSignalLength()))
        thr = sigma * c
        for level in range(1, result.getLevels() + 1):
            arr = result.getMutableDetailCoeffs(level)
            eng.threshold_inplace(arr if arr.ndim == 2 else arr.reshape(1, -1), thr, soft)

    def denoise(self, signal, levels: int, threshold: float = -1.0, soft: bool = True, return_thresholds: bool = False):
        """denoise :532-562 -- one fused device pipeline."""
        if _length(signal) == 0:
            raise InvalidSignalException("Signal cannot be empty for SWT", ErrorCode.VAL_EMPTY)
        w = self.wavelet
        flags = self._forward_flags(_length(signal), levels)
        return _engine_for(signal).denoise(signal, w.lowPassDecomposition(), w.highPassDecomposition(), w.wavelet_id,
                                           int(self.boundaryMode), levels, threshold, soft, flags,
                                           want_thresholds=return_thresholds)

    def extractLevel(self, signal, levels: int, targetLevel: int):
        """extractLevel :576-598: zero every level but targetLevel (0 = approximation), reconstruct."""
        res = self.forward(signal, levels)
        mask = 0 if targetLevel == 0 else (1 << (targetLevel - 1))
        if targetLevel < 0 or targetLevel > levels:
            mask = 0
        return self.modwtTransform._reconstruct(res, mask, targetLevel != 0,
                                                guard=self.boundaryMode != BoundaryMode.PERIODIC)

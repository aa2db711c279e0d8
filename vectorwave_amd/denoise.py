"""Wavelet denoising: Python mirror of ``core/denoising/WaveletDenoiser.java`` on the HIP engine.

Every call is one device pipeline (vw_wavelet_denoise_f64): forward transform -> exact median of |d_1|
(sigma = MAD / 0.6745) -> one threshold per (level, signal) by the selected method -> inverse with the
per-level threshold fused into the detail staging.  Accepts one signal ``[N]`` or a batch ``[B, N]``
(numpy: host-memory path; torch CUDA tensors stay resident in HBM); a batch row is denoised exactly as
the reference denoises that row on its own.
"""
from __future__ import annotations

import enum

from . import _native as nat
from .errors import ErrorCode, InvalidArgumentException
from .modwt import BoundaryMode, _check_boundary, _engine_for, _validate_signal
from .wavelets import Daubechies, Wavelet


class ThresholdMethod(enum.IntEnum):
    """WaveletDenoiser.ThresholdMethod (:588-615); values = the C ABI's VW_THR_*."""
    UNIVERSAL = 0
    SURE = 1
    MINIMAX = 2
    BAYES = 3
    FIXED = 4


class ThresholdType(enum.IntEnum):
    """WaveletDenoiser.ThresholdType (:620-634)."""
    SOFT = 1
    HARD = 0


class WaveletDenoiser:
    """core/denoising/WaveletDenoiser.java.

    denoise(signal, method[, type])              :111-143  single-level MODWTTransform, sigma from its details
    denoiseMultiLevel(signal, levels, method, t) :155-170  MultiLevelMODWTTransform; level j thresholded with
                                                           sigma / sqrt(2^j) on its own coefficients (:204-231)
    denoiseFixed(signal, threshold, type)        :354-364  single level, given threshold
    Thresholds (calculateThreshold :394-436): UNIVERSAL sigma*sqrt(2 ln n); SURE (the reference's exhaustive
    risk search, reproduced bit for bit; N <= 16384 on the device); MINIMAX; BAYES (sequential sums).
    """

    ThresholdMethod = ThresholdMethod
    ThresholdType = ThresholdType
    MAX_SAFE_LEVEL_FOR_SCALING = 31

    def __init__(self, wavelet: Wavelet, boundaryMode: BoundaryMode, fma: bool = False):
        if wavelet is None:
            raise InvalidArgumentException("wavelet cannot be null", ErrorCode.VAL_NULL_ARGUMENT)
        if boundaryMode is None:
            raise InvalidArgumentException("boundaryMode cannot be null", ErrorCode.VAL_NULL_ARGUMENT)
        _check_boundary(BoundaryMode(boundaryMode))
        self.wavelet = wavelet
        self.boundaryMode = BoundaryMode(boundaryMode)
        self._fma = nat.FLAG_FMA if fma else 0

    @staticmethod
    def forFinancialData() -> "WaveletDenoiser":
        """:98-100 -- DB4, PERIODIC."""
        return WaveletDenoiser(Daubechies.DB4, BoundaryMode.PERIODIC)

    def _run(self, signal, levels: int, method: ThresholdMethod, fixed: float, type_: ThresholdType,
             return_thresholds: bool, extra_flags: int):
        _validate_signal(signal)
        if method is None or type_ is None:
            raise TypeError("method / type cannot be null")
        w = self.wavelet
        flags = nat.FLAG_VALIDATE | self._fma | extra_flags
        return _engine_for(signal).wavelet_denoise(signal, w.lowPassDecomposition(), w.highPassDecomposition(),
                                                   w.wavelet_id, int(self.boundaryMode), levels,
                                                   int(ThresholdMethod(method)), fixed,
                                                   ThresholdType(type_) == ThresholdType.SOFT, flags,
                                                   want_thresholds=return_thresholds)

    def denoise(self, signal, method: ThresholdMethod, type: ThresholdType = ThresholdType.SOFT,
                return_thresholds: bool = False):
        """:111-143.  method FIXED raises (calculateThreshold :415-424); use denoiseFixed."""
        if method == ThresholdMethod.FIXED:
            raise InvalidArgumentException("Fixed threshold method requires explicit threshold value",
                                           ErrorCode.CFG_UNSUPPORTED_OPERATION)
        return self._run(signal, 0, method, 0.0, type, return_thresholds, 0)

    def denoiseMultiLevel(self, signal, levels: int, method: ThresholdMethod, type: ThresholdType,
                          return_thresholds: bool = False):
        """:155-170 (+ DenoisedMultiLevelResult :180-231)."""
        if method == ThresholdMethod.FIXED:
            raise InvalidArgumentException("Fixed threshold method requires explicit threshold value",
                                           ErrorCode.CFG_UNSUPPORTED_OPERATION)
        if levels is None or levels < 1:
            raise InvalidArgumentException(f"Invalid number of decomposition levels: {levels}",
                                           ErrorCode.CFG_INVALID_DECOMPOSITION_LEVEL)
        return self._run(signal, int(levels), method, 0.0, type, return_thresholds,
                         nat.FLAG_CORE_LEVELS | nat.FLAG_FFT_SWITCH)

    def denoiseFixed(self, signal, threshold: float, type: ThresholdType, return_thresholds: bool = False):
        """:354-364."""
        return self._run(signal, 0, ThresholdMethod.FIXED, float(threshold), type, return_thresholds, 0)

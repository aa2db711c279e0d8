"""vectorwave_amd -- MI355X (gfx950) MODWT / SWT engine with VectorWave's API.

The compute path is libvectorwave_amd.so (hand-written HIP kernels behind a C ABI,
include/vectorwave_amd.h).  This package is the host-side mirror of the reference's Java API:

  MODWTTransform, MultiLevelMODWTTransform, MODWTResult, MultiLevelMODWTResult,
  MutableMultiLevelMODWTResult, BoundaryMode                  (core/modwt, core/api)
  VectorWaveSwtAdapter                                        (core/swt)
  WaveletDenoiser                                             (core/denoising)
  MODWTStreamingTransform, MultiLevelMODWTStreamingTransform  (core/modwt/streaming)
  BatchMODWT, BatchStreamingMODWT                             (ext/extensions/modwt)
  Haar, Daubechies, Symlet, Coiflet                           (core/api wavelets)
"""
from .wavelets import Coiflet, Daubechies, Haar, Symlet, Wavelet, available_wavelets, get_wavelet
from .errors import (ErrorCode, InvalidArgumentException, InvalidSignalException, InvalidStateException,
                     WaveletTransformException)
from .modwt import (BoundaryMode, MODWTResult, MODWTTransform, MultiLevelMODWTResult, MultiLevelMODWTTransform,
                    MutableMultiLevelMODWTResult)
from .swt import VectorWaveSwtAdapter
from .denoise import ThresholdMethod, ThresholdType, WaveletDenoiser
from .streaming import (MODWTStreamingDenoiser, MODWTStreamingTransform, MODWTStreamingTransformImpl,
                        MultiLevelMODWTStreamingTransform)
from .batch import BatchMODWT, BatchSIMDMODWT, BatchStreamingMODWT
from .engine import Engine, max_levels, version
from .multidevice import DeviceGroup

__all__ = [
    "Coiflet", "Daubechies", "Haar", "Symlet", "Wavelet", "available_wavelets", "get_wavelet",
    "ErrorCode", "InvalidArgumentException", "InvalidSignalException", "InvalidStateException",
    "WaveletTransformException", "BoundaryMode", "MODWTResult", "MODWTTransform", "MultiLevelMODWTResult",
    "MultiLevelMODWTTransform", "MutableMultiLevelMODWTResult", "VectorWaveSwtAdapter", "BatchMODWT",
    "WaveletDenoiser", "ThresholdMethod", "ThresholdType", "BatchSIMDMODWT", "MODWTStreamingTransform",
    "MODWTStreamingTransformImpl", "MultiLevelMODWTStreamingTransform",
    "BatchStreamingMODWT", "Engine", "max_levels", "version", "DeviceGroup",
]

"""ctypes binding of the C ABI in include/vectorwave_amd.h (libvectorwave_amd.so, built in-tree).

This is the same surface a JNI / FFM shim binds.  The library is required: there is
no CPU fallback in the product path -- if the shared object is missing or was built without the
gfx950 kernels, importing the engine raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int64, c_uint, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VW_LIB_PATH", os.path.join(_HERE, "libvectorwave_amd.so"))

# flags (include/vectorwave_amd.h)
FLAG_CORE_LEVELS = 1 << 0
FLAG_VALIDATE = 1 << 1
FLAG_FFT_SWITCH = 1 << 2
FLAG_FMA = 1 << 3
FLAG_HOST_MEMORY = 1 << 4
FLAG_SYNC = 1 << 5
FLAG_BATCH_SYM_INVERSE = 1 << 6
FLAG_BATCH_HAAR = 1 << 7
FLAG_REF_NONFINITE = 1 << 8

PERIODIC, SYMMETRIC, ZERO_PADDING = 0, 1, 2

# Every symbol include/vectorwave_amd.h declares, with its ctypes signature.
_dp = POINTER(c_double)
_fp = POINTER(c_float)
SIGNATURES = {
    "vw_ctx_create": (c_int, [c_int, POINTER(c_void_p)]),
    "vw_ctx_destroy": (c_int, [c_void_p]),
    "vw_ctx_use_null_stream": (c_int, [c_void_p]),
    "vw_ctx_set_stream": (c_int, [c_void_p, c_void_p]),
    "vw_ctx_get_stream": (c_void_p, [c_void_p]),
    "vw_ctx_set_option": (c_int, [c_void_p, c_char_p, c_int]),
    "vw_ctx_synchronize": (c_int, [c_void_p]),
    "vw_ctx_device": (c_int, [c_void_p]),
    "vw_last_error": (c_char_p, []),
    "vw_last_error_index": (c_int64, []),
    "vw_version": (c_char_p, []),
    "vw_set_signal_base": (None, [c_int64]),
    "vw_max_levels": (c_int, [c_int64, c_int]),
    "vw_upsampled_length": (c_int64, [c_int, c_int]),
    "vw_modwt_forward_f64": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64, _dp, _dp, c_int, c_int, c_int,
                                     c_int, c_uint, c_void_p, c_void_p]),
    "vw_modwt_forward_f32": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64, _dp, _dp, c_int, c_int, c_int,
                                     c_int, c_uint, c_void_p, c_void_p]),
    "vw_modwt_inverse_f64": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, _dp, _dp, c_int, c_int, c_int,
                                     c_int, c_uint, c_int, c_uint, c_void_p]),
    "vw_modwt_inverse_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, _dp, _dp, c_int, c_int, c_int,
                                     c_int, c_uint, c_int, c_uint, c_void_p]),
    # ctxs: a (c_void_p * n) array of vw_ctx handles
    "vw_modwt_forward_multi_f64": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_int64, c_int64, _dp, _dp, c_int,
                                           c_int, c_int, c_int, c_uint, c_void_p, c_void_p]),
    "vw_modwt_inverse_multi_f64": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int64, c_int64, _dp, _dp, c_int,
                                           c_int, c_int, c_int, c_uint, c_int, c_uint, c_void_p]),
    # device-resident: per-context arrays of device pointers (c_void_p * n) and rows (c_int64 * n)
    "vw_modwt_forward_multi_dev_f64": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int64, c_int64, _dp, _dp,
                                               c_int, c_int, c_int, c_int, c_uint, c_void_p, c_void_p]),
    "vw_modwt_inverse_multi_dev_f64": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int64, _dp, _dp,
                                               c_int, c_int, c_int, c_int, c_uint, c_int, c_uint, c_void_p]),
    "vw_modwt1_forward_f64": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64, _dp, _dp, c_int, c_int, c_uint,
                                      c_void_p, c_void_p]),
    "vw_modwt1_inverse_f64": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int64, _dp, _dp, c_int, c_int, c_uint,
                                      c_void_p]),
    "vw_swt_denoise_f64": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64, _dp, _dp, c_int, c_int, c_int,
                                   c_int, c_double, c_int, c_uint, c_void_p, c_void_p]),
    "vw_wavelet_denoise_f64": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_int64, _dp, _dp, c_int, c_int, c_int,
                                       c_int, c_int, c_double, c_int, c_uint, c_void_p, c_void_p]),
    "vw_transpose_f64": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_uint, c_void_p]),
    "vw_transpose_f32": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_uint, c_void_p]),
    "vw_noise_sigma_f64": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_uint, c_void_p]),
    "vw_threshold_f64": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_int, c_uint]),
    "vw_stream_create": (c_int, [c_void_p, _dp, _dp, c_int, c_int, c_int, POINTER(c_void_p)]),
    "vw_stream_destroy": (c_int, [c_void_p]),
    "vw_stream_process_f64": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_uint, c_void_p, c_void_p]),
    "vw_stream_flush_f64": (c_int, [c_void_p, c_int64, c_uint, c_void_p, c_void_p]),
    "vw_stream_history_length": (c_int64, [c_void_p, c_int]),
    "vw_stream_batch": (c_int64, [c_void_p]),
    "vw_fill_uniform_f64": (c_int, [c_void_p, c_void_p, c_int64, c_uint64, c_int64]),
    "vw_fill_uniform_f32": (c_int, [c_void_p, c_void_p, c_int64, c_uint64, c_int64]),
    "vw_device_alloc": (c_int, [c_void_p, c_int64, POINTER(c_void_p)]),
    "vw_device_free": (c_int, [c_void_p, c_void_p]),
    "vw_memcpy": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int]),
    "vw_ctx_enable_timing": (c_int, [c_void_p, c_int]),
    "vw_ctx_kernel_time": (c_int, [c_void_p, c_char_p, POINTER(c_double), POINTER(c_int64)]),
    "vw_ctx_reset_timing": (c_int, [c_void_p]),
    "vw_ctx_kernel_spans": (c_int, [c_void_p, c_char_p, c_void_p, c_int64, POINTER(c_double), POINTER(c_double),
                                    POINTER(c_int64)]),
    "vw_median_f64": (c_int, [c_void_p, c_void_p, c_int64, c_int64, c_void_p, c_uint, c_void_p]),
    "vw_stddev_f64": (c_int, [c_void_p, c_void_p, c_int64, c_uint, c_void_p]),
    "vw_window_gather_abs_f64": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_int64]),
    "vw_capture_begin": (c_int, [c_void_p]),
    "vw_capture_end": (c_int, [c_void_p, POINTER(c_void_p)]),
    "vw_graph_launch": (c_int, [c_void_p, c_int64]),
    "vw_graph_destroy": (c_int, [c_void_p]),
    # pipelined round trips: per-set arrays of device pointers (c_void_p * sets)
    "vw_pipeline_create": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                   c_int64, _dp, _dp, c_int, c_int, c_int, c_int, c_uint, POINTER(c_void_p)]),
    "vw_pipeline_run": (c_int, [c_void_p, c_int64]),
    "vw_pipeline_join": (c_int, [c_void_p]),
    "vw_pipeline_last_set": (c_int64, [c_void_p]),
    "vw_pipeline_destroy": (c_int, [c_void_p]),
}

_lib = None


def load() -> ctypes.CDLL:
    """Load libvectorwave_amd.so once; raise (never fall back) when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"vectorwave_amd native library not found at {LIB_PATH}; build it with "
            f"`python -c 'import __graft_entry__ as g; g.build()'` (make -C vectorwave_amd/csrc)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error() -> str:
    msg = load().vw_last_error()
    return msg.decode() if msg else ""


def last_error_index() -> int:
    return int(load().vw_last_error_index())


def taps_array(values) -> ctypes.Array:
    arr = (c_double * len(values))(*[float(v) for v in values])
    return arr

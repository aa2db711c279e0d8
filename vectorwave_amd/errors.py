"""Exception taxonomy: mirror of VectorWave's ``core/exception`` package.

Reference: core/exception/ErrorCode.java:24-118 (codes), InvalidSignalException,
InvalidArgumentException, InvalidStateException.  The C ABI returns status codes
(include/vectorwave_amd.h); :func:`raise_for_status` maps them back to these exceptions, the same
way a JNI shim would rethrow them.
"""
from __future__ import annotations

import enum


class ErrorCode(enum.Enum):
    """Subset of core/exception/ErrorCode.java that the MODWT/SWT path raises."""

    VAL_NON_FINITE_VALUES = ("VAL_003", "Non-finite values (NaN or Infinity) in input")
    VAL_TOO_LARGE = ("VAL_005", "Value too large")
    VAL_EMPTY = ("VAL_006", "Empty input")
    CFG_UNSUPPORTED_BOUNDARY_MODE = ("CFG_003", "Unsupported boundary mode")
    CFG_INVALID_DECOMPOSITION_LEVEL = ("CFG_004", "Invalid decomposition level")
    CFG_UNSUPPORTED_OPERATION = ("CFG_001", "Unsupported operation")
    VAL_NULL_ARGUMENT = ("VAL_001", "Null argument")
    STATE_INVALID = ("STATE_001", "Invalid state")

    @property
    def code(self) -> str:
        return self.value[0]


class WaveletTransformException(RuntimeError):
    def __init__(self, message: str, error_code: ErrorCode | None = None):
        super().__init__(message)
        self.error_code = error_code


class InvalidSignalException(WaveletTransformException):
    def __init__(self, message: str, error_code: ErrorCode | None = None, index: int = -1):
        super().__init__(message, error_code)
        self.index = index


class InvalidArgumentException(WaveletTransformException, ValueError):
    pass


class InvalidStateException(WaveletTransformException):
    pass


class DeviceError(RuntimeError):
    """HIP runtime failure inside the engine (VW_ERR_DEVICE)."""


# status codes of include/vectorwave_amd.h
VW_OK = 0
VW_ERR_NULL = 1
VW_ERR_EMPTY = 2
VW_ERR_NONFINITE = 3
VW_ERR_LEVEL = 4
VW_ERR_TOO_LARGE = 5
VW_ERR_BOUNDARY = 6
VW_ERR_ARG = 7
VW_ERR_DEVICE = 8
VW_ERR_UNSUPPORTED = 9
VW_ERR_STATE = 10


def raise_for_status(status: int, message: str, index: int = -1) -> None:
    """Rethrow a C-ABI status as the reference's exception type (the JNI shim's job)."""
    if status == VW_OK:
        return
    if status == VW_ERR_NULL:
        raise TypeError(message or "null argument")  # NullPointerException
    if status == VW_ERR_EMPTY:
        raise InvalidSignalException(message, ErrorCode.VAL_EMPTY)
    if status == VW_ERR_NONFINITE:
        raise InvalidSignalException(message, ErrorCode.VAL_NON_FINITE_VALUES, index)
    if status == VW_ERR_LEVEL:
        raise InvalidArgumentException(message, ErrorCode.CFG_INVALID_DECOMPOSITION_LEVEL)
    if status == VW_ERR_TOO_LARGE:
        raise InvalidArgumentException(message, ErrorCode.VAL_TOO_LARGE)
    if status == VW_ERR_BOUNDARY:
        raise InvalidArgumentException(message, ErrorCode.CFG_UNSUPPORTED_BOUNDARY_MODE)
    if status == VW_ERR_ARG:
        raise InvalidArgumentException(message)
    if status == VW_ERR_UNSUPPORTED:
        raise NotImplementedError(message)  # UnsupportedOperationException
    if status == VW_ERR_STATE:
        raise InvalidStateException(message, ErrorCode.STATE_INVALID)
    raise DeviceError(f"status {status}: {message}")

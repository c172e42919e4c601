"""Enumerations and exceptions (values identical to the C API, spfft/types.h, spfft/errors.h)."""
from __future__ import annotations

import enum


class ExchangeType(enum.IntEnum):
    DEFAULT = 0
    BUFFERED = 1
    BUFFERED_FLOAT = 2
    COMPACT_BUFFERED = 3
    COMPACT_BUFFERED_FLOAT = 4
    UNBUFFERED = 5


class ProcessingUnit(enum.IntEnum):
    HOST = 1
    GPU = 2


class IndexFormat(enum.IntEnum):
    TRIPLETS = 0


class TransformType(enum.IntEnum):
    C2C = 0
    R2C = 1


class Scaling(enum.IntEnum):
    NONE = 0
    FULL = 1


class ErrorCode(enum.IntEnum):
    SUCCESS = 0
    UNKNOWN = 1
    INVALID_HANDLE = 2
    OVERFLOW = 3
    ALLOCATION = 4
    INVALID_PARAMETER = 5
    DUPLICATE_INDICES = 6
    INVALID_INDICES = 7
    MPI_SUPPORT = 8
    MPI = 9
    MPI_PARAMETER_MISMATCH = 10
    HOST_EXECUTION = 11
    FFTW = 12
    GPU = 13
    GPU_PRECEDING = 14
    GPU_SUPPORT = 15
    GPU_ALLOCATION = 16
    GPU_LAUNCH = 17
    GPU_NO_DEVICE = 18
    GPU_INVALID_VALUE = 19
    GPU_INVALID_DEVICE_PTR = 20
    GPU_COPY = 21
    GPU_FFT = 22
    INTERNAL = 23


class SpfftError(RuntimeError):
    """Base class; ``code`` is the C API error code."""

    code = ErrorCode.UNKNOWN

    def __init__(self, message: str = "", code: int | None = None):
        if code is not None:
            self.code = ErrorCode(code)
        super().__init__(message or self.code.name)


def _make(name, code, base=SpfftError):
    return type(name, (base,), {"code": code})


InvalidHandleError = _make("InvalidHandleError", ErrorCode.INVALID_HANDLE)
OverflowError_ = _make("OverflowError", ErrorCode.OVERFLOW)
HostAllocationError = _make("HostAllocationError", ErrorCode.ALLOCATION)
InvalidParameterError = _make("InvalidParameterError", ErrorCode.INVALID_PARAMETER)
DuplicateIndicesError = _make("DuplicateIndicesError", ErrorCode.DUPLICATE_INDICES)
InvalidIndicesError = _make("InvalidIndicesError", ErrorCode.INVALID_INDICES)
MPISupportError = _make("MPISupportError", ErrorCode.MPI_SUPPORT)
MPIError = _make("MPIError", ErrorCode.MPI)
MPIParameterMismatchError = _make("MPIParameterMismatchError", ErrorCode.MPI_PARAMETER_MISMATCH)
HostExecutionError = _make("HostExecutionError", ErrorCode.HOST_EXECUTION)
FFTWError = _make("FFTWError", ErrorCode.FFTW)
InternalError = _make("InternalError", ErrorCode.INTERNAL)
GPUError = _make("GPUError", ErrorCode.GPU)
GPUPrecedingError = _make("GPUPrecedingError", ErrorCode.GPU_PRECEDING, GPUError)
GPUSupportError = _make("GPUSupportError", ErrorCode.GPU_SUPPORT, GPUError)
GPUAllocationError = _make("GPUAllocationError", ErrorCode.GPU_ALLOCATION, GPUError)
GPULaunchError = _make("GPULaunchError", ErrorCode.GPU_LAUNCH, GPUError)
GPUNoDeviceError = _make("GPUNoDeviceError", ErrorCode.GPU_NO_DEVICE, GPUError)
GPUInvalidValueError = _make("GPUInvalidValueError", ErrorCode.GPU_INVALID_VALUE, GPUError)
GPUInvalidDevicePointerError = _make("GPUInvalidDevicePointerError",
                                     ErrorCode.GPU_INVALID_DEVICE_PTR, GPUError)
GPUCopyError = _make("GPUCopyError", ErrorCode.GPU_COPY, GPUError)
GPUFFTError = _make("GPUFFTError", ErrorCode.GPU_FFT, GPUError)

_BY_CODE = {cls.code: cls for cls in (
    InvalidHandleError, OverflowError_, HostAllocationError, InvalidParameterError,
    DuplicateIndicesError, InvalidIndicesError, MPISupportError, MPIError,
    MPIParameterMismatchError, HostExecutionError, FFTWError, InternalError, GPUError,
    GPUPrecedingError, GPUSupportError, GPUAllocationError, GPULaunchError, GPUNoDeviceError,
    GPUInvalidValueError, GPUInvalidDevicePointerError, GPUCopyError, GPUFFTError)}


def raise_for(code: int, message: str = "") -> None:
    """Raises the exception class of a non-zero C API error code."""
    if code == 0:
        return
    cls = _BY_CODE.get(code, SpfftError)
    raise cls(message, code)

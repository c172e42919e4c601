"""SpFFT-AMD: sparse 3D FFT for AMD Instinct MI355X (gfx950).

A brand-new MI355X-native implementation of the SpFFT capabilities
(Grid/Transform API, C/C++/Fortran bindings, C2C and R2C, centred indices,
slab/pencil distribution over RCCL). The compute path is hand-written HIP for
CDNA4; this package is the Python front end over the native library.

Layout:
  spfft_amd.grid      Grid / Transform (+Float), multi_transform_*
  spfft_amd.ops       native library loader, DLPack views, kernel-level helpers
  spfft_amd.parallel  communicators (torch.distributed, in-process groups) and
                      distributed helpers
  spfft_amd.utils     index generators (spherical cutoff, reference test data),
                      dense oracles, timing
  spfft_amd.models    benchmark workload configurations (BASELINE.json configs)
"""
from .types import (ErrorCode, ExchangeType, IndexFormat, ProcessingUnit, Scaling,  # noqa: F401
                    SpfftError, TransformType)
from .types import *  # noqa: F401,F403  (exception classes)
from .grid import (Grid, GridFloat, Transform, TransformFloat,  # noqa: F401
                   multi_transform_backward, multi_transform_forward)
from .utils.timing import timing_enable, timing_json, timing_report, timing_reset  # noqa: F401

__version__ = "1.0.0"


def device_count() -> int:
    from .ops._lib import lib
    return int(lib().spfft_amd_device_count())


def build_info() -> str:
    from .ops._lib import lib
    return lib().spfft_amd_build_info().decode()


def rccl_communicators() -> int:
    """RCCL communicators this process has created (grids with the same members on
    the same devices share one)."""
    import ctypes
    from .ops._lib import lib
    n = ctypes.c_int()
    rc = lib().spfft_amd_rccl_communicators(ctypes.byref(n))
    if rc != 0:
        raise RuntimeError(f"spfft_amd_rccl_communicators failed ({rc})")
    return n.value


def library_streams() -> int:
    """HIP streams the library currently owns (private transform streams, created on a
    transform's first call unless it was given a stream first, and RCCL channel
    streams)."""
    import ctypes
    from .ops._lib import lib
    n = ctypes.c_int()
    rc = lib().spfft_amd_library_streams(ctypes.byref(n))
    if rc != 0:
        raise RuntimeError(f"spfft_amd_library_streams failed ({rc})")
    return n.value

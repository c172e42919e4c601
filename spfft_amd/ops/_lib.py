"""Loader and ctypes prototypes of the native library ``libspfft_amd.so``.

The library is built in-tree (``spfft_amd/_native``) by ``spfft_amd.build``.
PyTorch (when importable) is imported first so that the HIP runtime and RCCL
that torch ships are the ones the library binds to (same SONAMEs): one HIP
runtime per process.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE_DIR = os.path.join(os.path.dirname(_HERE), "_native")
LIB_NAME = "libspfft_amd.so"
# the testing library: the same kernels and host code plus fault injection and
# test probes (CMake SPFFT_TESTING_LIBRARY); loaded when SPFFT_AMD_LIBRARY names it
TESTING_LIB_PATH = os.path.join(NATIVE_DIR, "libspfft_amd_testing.so")

_lock = threading.Lock()
_lib = None

c_int_p = ctypes.POINTER(ctypes.c_int)
c_ll_p = ctypes.POINTER(ctypes.c_longlong)
c_void_pp = ctypes.POINTER(ctypes.c_void_p)
c_size_t_p = ctypes.POINTER(ctypes.c_size_t)

ALLGATHER_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_size_t)
ALLTOALLV_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, c_size_t_p,
                                c_size_t_p, ctypes.c_void_p, c_size_t_p, c_size_t_p)
BARRIER_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)
DESTROY_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


class CommCallbacks(ctypes.Structure):
    _fields_ = [
        ("context", ctypes.c_void_p),
        ("rank", ctypes.c_int),
        ("size", ctypes.c_int),
        ("allgather", ALLGATHER_CB),
        ("alltoallv", ALLTOALLV_CB),
        ("barrier", BARRIER_CB),
        ("destroy", DESTROY_CB),
    ]


def library_path() -> str:
    env = os.environ.get("SPFFT_AMD_LIBRARY")
    if env:
        return env
    return os.path.join(NATIVE_DIR, LIB_NAME)


def _prototypes(lib):
    E = ctypes.c_int  # SpfftError
    I = ctypes.c_int
    V = ctypes.c_void_p
    D = ctypes.c_void_p  # data pointers passed as raw addresses
    sig = {}
    for pre in ("spfft_", "spfft_float_"):
        sig[pre + "grid_create"] = [c_void_pp, I, I, I, I, I, I]
        sig[pre + "grid_destroy"] = [V]
        for g in ("max_dim_x", "max_dim_y", "max_dim_z", "max_num_local_z_columns",
                  "max_local_z_length", "processing_unit", "device_id", "num_threads"):
            sig[pre + "grid_" + g] = [V, c_int_p]
        sig[pre + "transform_create"] = [c_void_pp, V, I, I, I, I, I, I, I, I, V]
        sig[pre + "transform_destroy"] = [V]
        sig[pre + "transform_clone"] = [V, c_void_pp]
        sig[pre + "transform_forward"] = [V, I, D, I]
        sig[pre + "transform_backward"] = [V, D, I]
        sig[pre + "transform_get_space_domain"] = [V, I, c_void_pp]
        for g in ("dim_x", "dim_y", "dim_z", "local_z_length", "local_slice_size", "local_z_offset",
                  "num_local_elements", "device_id", "num_threads", "type", "processing_unit"):
            sig[pre + "transform_" + g] = [V, c_int_p]
        sig[pre + "transform_global_size"] = [V, c_ll_p]
        sig[pre + "transform_num_global_elements"] = [V, c_ll_p]
        sig[pre + "multi_transform_forward"] = [I, c_void_pp, c_int_p, c_void_pp, c_int_p]
        sig[pre + "multi_transform_backward"] = [I, c_void_pp, c_void_pp, c_int_p]
    sig["spfft_amd_comm_create_callbacks"] = [c_void_pp, ctypes.POINTER(CommCallbacks)]
    sig["spfft_amd_comm_create_local_group"] = [I, c_void_pp]
    sig["spfft_amd_comm_destroy"] = [V]
    sig["spfft_amd_comm_rank"] = [V, c_int_p]
    sig["spfft_amd_comm_size"] = [V, c_int_p]
    sig["spfft_amd_grid_create_distributed"] = [c_void_pp, I, I, I, I, I, I, I, V, I]
    sig["spfft_amd_float_grid_create_distributed"] = [c_void_pp, I, I, I, I, I, I, I, V, I]
    sig["spfft_amd_grid_exchange_type"] = [V, c_int_p]
    sig["spfft_amd_float_grid_exchange_type"] = [V, c_int_p]
    sig["spfft_amd_grid_data_plane"] = [V, ctypes.POINTER(ctypes.c_char_p)]
    sig["spfft_amd_float_grid_data_plane"] = [V, ctypes.POINTER(ctypes.c_char_p)]
    sig["spfft_amd_grid_data_plane_info"] = [V, ctypes.POINTER(ctypes.c_char_p)]
    sig["spfft_amd_float_grid_data_plane_info"] = [V, ctypes.POINTER(ctypes.c_char_p)]
    sig["spfft_amd_rccl_communicators"] = [c_int_p]
    sig["spfft_amd_library_streams"] = [c_int_p]
    sig["spfft_amd_grid_device_bytes"] = [V, ctypes.POINTER(ctypes.c_ulonglong)]
    sig["spfft_amd_float_grid_device_bytes"] = [V, ctypes.POINTER(ctypes.c_ulonglong)]
    sig["spfft_amd_transform_set_stream"] = [V, V, I]
    sig["spfft_amd_float_transform_set_stream"] = [V, V, I]
    sig["spfft_amd_transform_synchronize"] = [V]
    sig["spfft_amd_transform_reset_stream"] = [V]
    sig["spfft_amd_float_transform_reset_stream"] = [V]
    sig["spfft_amd_float_transform_synchronize"] = [V]
    sig["spfft_amd_transform_local_z_offset_rank"] = [V, I, c_int_p, c_int_p]
    sig["spfft_amd_transform_exchange_plan"] = [V, c_int_p, c_int_p, c_int_p, c_int_p]
    sig["spfft_amd_float_transform_exchange_plan"] = [V, c_int_p, c_int_p, c_int_p, c_int_p]
    sig["spfft_amd_transform_space_domain_dlpack"] = [V, I, c_void_pp]
    sig["spfft_amd_float_transform_space_domain_dlpack"] = [V, I, c_void_pp]
    sig["spfft_amd_transform_forward_xy"] = [V, I]
    sig["spfft_amd_transform_forward_exchange"] = [V, I]
    sig["spfft_amd_transform_forward_z"] = [V, D, I]
    sig["spfft_amd_transform_backward_z"] = [V, D]
    sig["spfft_amd_transform_backward_exchange"] = [V, I]
    sig["spfft_amd_transform_backward_xy"] = [V, I]
    sig["spfft_amd_float_transform_forward_xy"] = [V, I]
    sig["spfft_amd_float_transform_forward_exchange"] = [V, I]
    sig["spfft_amd_float_transform_forward_z"] = [V, D, I]
    sig["spfft_amd_float_transform_backward_z"] = [V, D]
    sig["spfft_amd_float_transform_backward_exchange"] = [V, I]
    sig["spfft_amd_float_transform_backward_xy"] = [V, I]
    sig["spfft_amd_timing_enable"] = [I]
    sig["spfft_amd_timing_reset"] = []
    sig["spfft_amd_timing_json"] = [ctypes.c_char_p, ctypes.c_size_t, c_size_t_p]
    sig["spfft_amd_timing_print"] = [ctypes.c_char_p, ctypes.c_size_t, c_size_t_p]
    # test probes: present in the testing library only
    test_sig = {"spfft_amd_test_comm_shm_check": [V, I, ctypes.POINTER(ctypes.c_double),
                                                  ctypes.POINTER(ctypes.c_double)]}
    for name, args in test_sig.items():
        if hasattr(lib, name):
            sig[name] = args
    for name, args in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = E
    lib.spfft_amd_last_error_message.argtypes = []
    lib.spfft_amd_last_error_message.restype = ctypes.c_char_p
    lib.spfft_amd_device_count.argtypes = []
    lib.spfft_amd_device_count.restype = ctypes.c_int
    lib.spfft_amd_build_info.argtypes = []
    lib.spfft_amd_build_info.restype = ctypes.c_char_p


def is_testing_library() -> bool:
    """True if the loaded library is the testing build (fault injection, probes)."""
    return hasattr(lib(), "spfft_amd_test_fault_injection")


def lib():
    """Returns the loaded native library (loads it on first use)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            try:  # share torch's HIP runtime / RCCL
                import torch  # noqa: F401
            except Exception:  # pragma: no cover - torch is optional
                pass
            path = library_path()
            if not os.path.exists(path):
                raise ImportError(
                    f"SpFFT-AMD native library not found at {path}; run `python -m spfft_amd.build`")
            handle = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
            _prototypes(handle)
            _lib = handle
    return _lib

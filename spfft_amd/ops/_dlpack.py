"""Zero-copy torch views of library-owned memory through DLPack.

The DLManagedTensor is created by the native library
(spfft_amd_transform_space_domain_dlpack); its deleter is native code that
releases the library's reference to the transform, so no Python callback runs
when torch frees the view (safe at interpreter shutdown).
"""
from __future__ import annotations

import ctypes

_PyCapsule_New = ctypes.pythonapi.PyCapsule_New
_PyCapsule_New.restype = ctypes.py_object
_PyCapsule_New.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]


def capsule_to_torch(managed_ptr: int):
    import torch.utils.dlpack

    capsule = _PyCapsule_New(managed_ptr, b"dltensor", None)
    return torch.utils.dlpack.from_dlpack(capsule)

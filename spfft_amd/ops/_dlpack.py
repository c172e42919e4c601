"""Zero-copy torch views of library-owned device memory through DLPack.

The space-domain slab of a GPU transform lives in the Grid's HBM arena; this
wraps it as a torch tensor without a copy. The owner object is kept alive for
as long as any tensor view exists.
"""
from __future__ import annotations

import ctypes

kDLCPU = 1
kDLROCM = 10
kDLFloat = 2
kDLComplex = 5


class DLDevice(ctypes.Structure):
    _fields_ = [("device_type", ctypes.c_int), ("device_id", ctypes.c_int)]


class DLDataType(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint8), ("bits", ctypes.c_uint8), ("lanes", ctypes.c_uint16)]


class DLTensor(ctypes.Structure):
    _fields_ = [
        ("data", ctypes.c_void_p),
        ("device", DLDevice),
        ("ndim", ctypes.c_int),
        ("dtype", DLDataType),
        ("shape", ctypes.POINTER(ctypes.c_int64)),
        ("strides", ctypes.POINTER(ctypes.c_int64)),
        ("byte_offset", ctypes.c_uint64),
    ]


class DLManagedTensor(ctypes.Structure):
    pass


_DELETER = ctypes.CFUNCTYPE(None, ctypes.POINTER(DLManagedTensor))
DLManagedTensor._fields_ = [("dl_tensor", DLTensor), ("manager_ctx", ctypes.c_void_p),
                            ("deleter", _DELETER)]

_alive: dict[int, tuple] = {}


@_DELETER
def _deleter(ptr):
    _alive.pop(ctypes.addressof(ptr.contents), None)


_PyCapsule_New = ctypes.pythonapi.PyCapsule_New
_PyCapsule_New.restype = ctypes.py_object
_PyCapsule_New.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]


def to_torch(ptr: int, shape, dtype_code: int, bits: int, device_type: int, device_id: int,
             owner):
    """Returns a torch tensor aliasing `ptr` (contiguous, row-major `shape`)."""
    import torch.utils.dlpack

    ndim = len(shape)
    shape_arr = (ctypes.c_int64 * max(1, ndim))(*shape)
    mt = DLManagedTensor()
    mt.dl_tensor.data = ptr
    mt.dl_tensor.device = DLDevice(device_type, device_id)
    mt.dl_tensor.ndim = ndim
    mt.dl_tensor.dtype = DLDataType(dtype_code, bits, 1)
    mt.dl_tensor.shape = shape_arr
    mt.dl_tensor.strides = None
    mt.dl_tensor.byte_offset = 0
    mt.manager_ctx = None
    mt.deleter = _deleter
    _alive[ctypes.addressof(mt)] = (mt, shape_arr, owner)
    capsule = _PyCapsule_New(ctypes.addressof(mt), b"dltensor", None)
    return torch.utils.dlpack.from_dlpack(capsule)

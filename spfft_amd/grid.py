"""Pythonic front end of the native library: Grid / Transform (and single-precision twins).

Mirrors the C++ API of SpFFT (reference: include/spfft/grid.hpp, transform.hpp,
multi_transform.hpp). Arrays may be numpy arrays (host memory) or torch tensors
(host or device memory). The space domain of a GPU transform is returned as a
zero-copy torch view of the Grid's HBM slab.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import numpy as np

from .ops._lib import lib
from .types import ExchangeType, IndexFormat, ProcessingUnit, Scaling, TransformType, raise_for

try:  # torch is optional for host-only use
    import torch
except Exception:  # pragma: no cover
    torch = None


_SHUTDOWN = [False]


def _at_exit():
    # objects still alive at interpreter exit are not destroyed through the native
    # library: the HIP runtime may already be tearing down.
    _SHUTDOWN[0] = True


import atexit  # noqa: E402

atexit.register(_at_exit)


def _check(code: int) -> None:
    if code != 0:
        msg = lib().spfft_amd_last_error_message()
        raise_for(code, msg.decode() if msg else "")


def _is_torch(a) -> bool:
    return torch is not None and isinstance(a, torch.Tensor)


class _Precision:
    def __init__(self, single: bool):
        self.single = single
        self.prefix = "spfft_float_" if single else "spfft_"
        self.amd = "spfft_amd_float_" if single else "spfft_amd_"
        self.real = np.float32 if single else np.float64
        self.complex = np.complex64 if single else np.complex128

    def fn(self, name):
        return getattr(lib(), self.prefix + name)

    def amd_fn(self, name):
        return getattr(lib(), self.amd + name)

    @property
    def torch_complex(self):
        return torch.complex64 if self.single else torch.complex128

    @property
    def torch_real(self):
        return torch.float32 if self.single else torch.float64


def _data_ptr(a, prec: _Precision, writable: bool, what: str):
    """Returns (address, keepalive) of a complex array argument."""
    if a is None:
        return None, None
    if _is_torch(a):
        if a.dtype in (torch.complex64, torch.complex128):
            if a.dtype != prec.torch_complex:
                raise TypeError(f"{what}: expected {prec.torch_complex}, got {a.dtype}")
        elif a.dtype != prec.torch_real:
            raise TypeError(f"{what}: expected {prec.torch_complex}, got {a.dtype}")
        if not a.is_contiguous():
            if writable:
                raise ValueError(f"{what} must be contiguous")
            a = a.contiguous()
        return a.data_ptr(), a
    arr = np.asarray(a)
    if arr.dtype not in (prec.complex, prec.real) or not arr.flags.c_contiguous:
        if writable:
            raise TypeError(f"{what}: expected a C-contiguous {np.dtype(prec.complex)} array")
        arr = np.ascontiguousarray(arr, dtype=prec.complex)
    return arr.ctypes.data, arr


class _GridBase:
    _single = False

    def __init__(self, max_dim_x: int, max_dim_y: int, max_dim_z: int,
                 max_num_local_z_columns: int, processing_unit=ProcessingUnit.HOST,
                 max_num_threads: int = -1, *, max_local_z_length: Optional[int] = None,
                 comm=None, exchange_type=ExchangeType.DEFAULT, _handle=None):
        self._prec = _Precision(self._single)
        self._comm = comm
        if _handle is not None:
            self._h = _handle
            return
        h = ctypes.c_void_p()
        if comm is None:
            _check(self._prec.fn("grid_create")(ctypes.byref(h), max_dim_x, max_dim_y, max_dim_z,
                                                max_num_local_z_columns, int(processing_unit),
                                                max_num_threads))
        else:
            if max_local_z_length is None:
                raise ValueError("distributed grids need max_local_z_length")
            create = (lib().spfft_amd_float_grid_create_distributed if self._single
                      else lib().spfft_amd_grid_create_distributed)
            _check(create(ctypes.byref(h), max_dim_x, max_dim_y, max_dim_z,
                          max_num_local_z_columns, max_local_z_length, int(processing_unit),
                          max_num_threads, comm.handle, int(exchange_type)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and not _SHUTDOWN[0]:
            try:
                self._prec.fn("grid_destroy")(h)
            except Exception:
                pass
            self._h = None

    def _get(self, name):
        v = ctypes.c_int()
        _check(self._prec.fn("grid_" + name)(self._h, ctypes.byref(v)))
        return v.value

    max_dim_x = property(lambda self: self._get("max_dim_x"))
    max_dim_y = property(lambda self: self._get("max_dim_y"))
    max_dim_z = property(lambda self: self._get("max_dim_z"))
    max_num_local_z_columns = property(lambda self: self._get("max_num_local_z_columns"))
    max_local_z_length = property(lambda self: self._get("max_local_z_length"))
    processing_unit = property(lambda self: ProcessingUnit(self._get("processing_unit")))
    device_id = property(lambda self: self._get("device_id"))
    num_threads = property(lambda self: self._get("num_threads"))

    @property
    def exchange_type(self) -> ExchangeType:
        v = ctypes.c_int()
        _check(self._prec.amd_fn("grid_exchange_type")(self._h, ctypes.byref(v)))
        return ExchangeType(v.value)

    @property
    def data_plane(self) -> str:
        """GPU data plane of a distributed grid: "rccl", "ipc", "peer", "loopback",
        "rccl-self" or "none". Collective on first use (it creates the data plane)."""
        v = ctypes.c_char_p()
        _check(self._prec.amd_fn("grid_data_plane")(self._h, ctypes.byref(v)))
        return v.value.decode()

    @property
    def data_plane_info(self) -> dict:
        """The data plane's setup facts: "kind", and where they apply "self_test" /
        "self_test_ms" (route self-test), "devices" (PCI bus ids of every GPU the plane
        touches, relay GPUs included), "link_GBps_measured", "channel_priority" ("high",
        or "normal" when ranks share a GPU). Collective on first use."""
        import json
        v = ctypes.c_char_p()
        _check(self._prec.amd_fn("grid_data_plane_info")(self._h, ctypes.byref(v)))
        return json.loads(v.value.decode())

    @property
    def device_bytes(self) -> int:
        """Device memory the grid allocated (exchange buffers, y/x intermediate, space)."""
        v = ctypes.c_ulonglong()
        _check(self._prec.amd_fn("grid_device_bytes")(self._h, ctypes.byref(v)))
        return v.value

    @property
    def communicator(self):
        return self._comm

    def create_transform(self, processing_unit, transform_type, dim_x: int, dim_y: int,
                         dim_z: int, local_z_length: int, indices,
                         index_format=IndexFormat.TRIPLETS):
        """Plans a transform. `indices` is an (n, 3) or flat int array of (x, y, z) triplets."""
        idx = np.ascontiguousarray(np.asarray(indices, dtype=np.int32).reshape(-1))
        if idx.size % 3:
            raise ValueError("indices must hold triplets")
        n = idx.size // 3
        h = ctypes.c_void_p()
        _check(self._prec.fn("transform_create")(
            ctypes.byref(h), self._h, int(processing_unit), int(transform_type), dim_x, dim_y,
            dim_z, local_z_length, n, int(index_format),
            idx.ctypes.data if n else None))
        cls = TransformFloat if self._single else Transform
        t = cls(h, self)
        in_process = getattr(self._comm, "in_process", False)
        if ProcessingUnit(processing_unit) == ProcessingUnit.GPU and torch is not None \
                and not in_process:
            # torch semantics: run on the current torch stream (ordered with torch work
            # on it, no cross-stream event per call); calls stay synchronous.
            # Ranks of an in-process group keep private streams: they share torch's
            # current stream, and one rank's exchange must not queue behind another's.
            t.set_stream(torch.cuda.current_stream(), synchronous=True)
        return t


class Grid(_GridBase):
    """Double-precision grid (spfft::Grid)."""

    _single = False


class GridFloat(_GridBase):
    """Single-precision grid (spfft::GridFloat)."""

    _single = True


class _TransformBase:
    _single = False

    def __init__(self, handle, grid):
        self._h = handle
        self._grid = grid  # keeps the grid (buffers) alive
        self._prec = _Precision(self._single)
        self._stream = None
        self._cache = {}
        self._views = {}
        self._step_keep = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and not _SHUTDOWN[0]:
            try:
                self._prec.fn("transform_destroy")(h)
            except Exception:
                pass
            self._h = None

    @property
    def handle(self):
        return self._h

    def _get(self, name, ll=False):
        # every getter of a transform is immutable after creation: cache it
        c = self._cache.get(name)
        if c is not None:
            return c
        v = ctypes.c_longlong() if ll else ctypes.c_int()
        _check(self._prec.fn("transform_" + name)(self._h, ctypes.byref(v)))
        self._cache[name] = v.value
        return v.value

    type = property(lambda self: TransformType(self._get("type")))
    dim_x = property(lambda self: self._get("dim_x"))
    dim_y = property(lambda self: self._get("dim_y"))
    dim_z = property(lambda self: self._get("dim_z"))
    local_z_length = property(lambda self: self._get("local_z_length"))
    local_z_offset = property(lambda self: self._get("local_z_offset"))
    local_slice_size = property(lambda self: self._get("local_slice_size"))
    global_size = property(lambda self: self._get("global_size", True))
    num_local_elements = property(lambda self: self._get("num_local_elements"))
    num_global_elements = property(lambda self: self._get("num_global_elements", True))
    processing_unit = property(lambda self: ProcessingUnit(self._get("processing_unit")))
    device_id = property(lambda self: self._get("device_id"))
    num_threads = property(lambda self: self._get("num_threads"))

    @property
    def grid(self):
        return self._grid

    def clone(self):
        h = ctypes.c_void_p()
        _check(self._prec.fn("transform_clone")(self._h, ctypes.byref(h)))
        t = type(self)(h, None)
        if self._stream is not None:
            t.set_stream(self._stream)
        return t

    # ---------------------------------------------------------------- data
    def space_domain_shape(self):
        return (self.local_z_length, self.dim_y, self.dim_x)

    def space_domain_ptr(self, location=ProcessingUnit.HOST) -> int:
        p = ctypes.c_void_p()
        _check(self._prec.fn("transform_get_space_domain")(self._h, int(location), ctypes.byref(p)))
        return p.value or 0

    def space_domain(self, location=ProcessingUnit.HOST):
        """View of the space-domain slab [local_z][y][x] (complex, or real for R2C).

        HOST: numpy array; GPU: torch tensor on the grid's device (zero copy).
        The view is created once per location and reused (the slab never moves)."""
        v = self._views.get(int(location))
        if v is None:
            v = self._make_view(location)
            self._views[int(location)] = v
        return v

    def _make_view(self, location):
        shape = self.space_domain_shape()
        real = self.type == TransformType.R2C
        ptr = self.space_domain_ptr(location)
        count = int(np.prod(shape))
        if ProcessingUnit(location) == ProcessingUnit.HOST:
            dtype = self._prec.real if real else self._prec.complex
            if count == 0 or not ptr:
                return np.zeros(shape, dtype=dtype)
            buf = (ctypes.c_byte * (count * np.dtype(dtype).itemsize)).from_address(ptr)
            buf._owner = self  # the view keeps the transform (and its grid) alive
            arr = np.frombuffer(buf, dtype=dtype).reshape(shape)
            return arr
        from .ops._dlpack import capsule_to_torch
        m = ctypes.c_void_p()
        _check(self._prec.amd_fn("transform_space_domain_dlpack")(self._h, int(location),
                                                                  ctypes.byref(m)))
        return capsule_to_torch(m.value)

    def _default_output(self):
        n = self.num_local_elements
        if self.processing_unit == ProcessingUnit.GPU and torch is not None:
            return torch.empty(n, dtype=self._prec.torch_complex, device=f"cuda:{self.device_id}")
        return np.empty(n, dtype=self._prec.complex)

    def backward(self, values, output_location=None):
        """Frequency -> space. Returns the space-domain view at `output_location`."""
        if output_location is None:
            output_location = self.processing_unit
        ptr, keep = _data_ptr(values, self._prec, False, "values")
        _check(self._prec.fn("transform_backward")(self._h, ptr, int(output_location)))
        del keep
        return self.space_domain(output_location)

    def forward(self, space=None, output=None, input_location=None, scaling=Scaling.NONE):
        """Space -> frequency. `space` (optional) is copied into the space domain first.

        Returns the frequency values (in index-triplet order)."""
        if input_location is None:
            input_location = self.processing_unit
        if space is not None:
            dst = self.space_domain(input_location)
            if _is_torch(dst):
                dst.copy_(space if _is_torch(space) else torch.as_tensor(np.asarray(space)))
            else:
                src = space.cpu().numpy() if _is_torch(space) else np.asarray(space)
                np.copyto(dst, src.reshape(dst.shape), casting="same_kind")
        if output is None:
            output = self._default_output()
        ptr, keep = _data_ptr(output, self._prec, True, "output")
        _check(self._prec.fn("transform_forward")(self._h, int(input_location), ptr, int(scaling)))
        del keep
        return output

    # --------------------------------------------------- streams / step API
    def set_stream(self, stream=None, synchronous: bool = True):
        """Execute on a HIP stream (int handle or torch.cuda.Stream; 0 = legacy default
        stream). None returns to the library's private stream."""
        if stream is None:
            self._stream = None
            _check(self._prec.amd_fn("transform_reset_stream")(self._h))
            return
        if not isinstance(stream, int):
            stream = stream.cuda_stream
        self._stream = stream
        _check(self._prec.amd_fn("transform_set_stream")(self._h, stream or None,
                                                        1 if synchronous else 0))

    def synchronize(self):
        _check(self._prec.amd_fn("transform_synchronize")(self._h))

    # Step-wise execution (spfft/amd.h): backward = backward_z, backward_exchange,
    # backward_xy; forward = forward_xy, forward_exchange, forward_z. Every rank calls
    # the same steps in the same order (the exchanges are collective); work that does
    # not depend on the exchange can be placed between the steps.
    def backward_z(self, values):
        ptr, keep = _data_ptr(values, self._prec, False, "values")
        _check(self._prec.amd_fn("transform_backward_z")(self._h, ptr))
        self._step_keep = keep  # until the next step: the z stage may still read it

    def backward_exchange(self, non_blocking: bool = False):
        _check(self._prec.amd_fn("transform_backward_exchange")(self._h, 1 if non_blocking else 0))

    def backward_xy(self, output_location=None):
        if output_location is None:
            output_location = self.processing_unit
        _check(self._prec.amd_fn("transform_backward_xy")(self._h, int(output_location)))
        self._step_keep = None
        return self.space_domain(output_location)

    def forward_xy(self, input_location=None):
        if input_location is None:
            input_location = self.processing_unit
        _check(self._prec.amd_fn("transform_forward_xy")(self._h, int(input_location)))

    def forward_exchange(self, non_blocking: bool = False):
        _check(self._prec.amd_fn("transform_forward_exchange")(self._h, 1 if non_blocking else 0))

    def forward_z(self, output=None, scaling=Scaling.NONE):
        if output is None:
            output = self._default_output()
        ptr, keep = _data_ptr(output, self._prec, True, "output")
        _check(self._prec.amd_fn("transform_forward_z")(self._h, ptr, int(scaling)))
        self._step_keep = keep
        return output

    def exchange_plan(self):
        """(plane chunks K, stick blocks I, peer writes, relay GPUs) of the GPU exchange."""
        k, i, pw, rl = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(self._prec.amd_fn("transform_exchange_plan")(self._h, ctypes.byref(k), ctypes.byref(i),
                                                            ctypes.byref(pw), ctypes.byref(rl)))
        return k.value, i.value, bool(pw.value), rl.value

    def rank_z_range(self, rank: int):
        off, ln = ctypes.c_int(), ctypes.c_int()
        _check(lib().spfft_amd_transform_local_z_offset_rank(self._h, rank, ctypes.byref(off),
                                                             ctypes.byref(ln)))
        return off.value, ln.value


class Transform(_TransformBase):
    _single = False


class TransformFloat(_TransformBase):
    _single = True


def _multi(transforms: Sequence[_TransformBase]):
    n = len(transforms)
    single = transforms[0]._single if n else False
    prec = _Precision(single)
    arr = (ctypes.c_void_p * max(1, n))(*[t.handle.value for t in transforms])
    return n, prec, arr


def multi_transform_backward(transforms, inputs, output_locations=None):
    """Backward transforms of several independent transforms (distinct grids), overlapped."""
    n, prec, arr = _multi(transforms)
    if output_locations is None:
        output_locations = [t.processing_unit for t in transforms]
    keeps, ptrs = [], (ctypes.c_void_p * max(1, n))()
    for i, v in enumerate(inputs):
        p, k = _data_ptr(v, prec, False, "values")
        ptrs[i] = p
        keeps.append(k)
    locs = (ctypes.c_int * max(1, n))(*[int(x) for x in output_locations])
    _check(prec.fn("multi_transform_backward")(n, arr, ptrs, locs))
    return [t.space_domain(loc) for t, loc in zip(transforms, output_locations)]


def multi_transform_forward(transforms, outputs=None, input_locations=None, scalings=None):
    n, prec, arr = _multi(transforms)
    if input_locations is None:
        input_locations = [t.processing_unit for t in transforms]
    if scalings is None:
        scalings = [Scaling.NONE] * n
    if outputs is None:
        outputs = [t._default_output() for t in transforms]
    keeps, ptrs = [], (ctypes.c_void_p * max(1, n))()
    for i, v in enumerate(outputs):
        p, k = _data_ptr(v, prec, True, "output")
        ptrs[i] = p
        keeps.append(k)
    locs = (ctypes.c_int * max(1, n))(*[int(x) for x in input_locations])
    scs = (ctypes.c_int * max(1, n))(*[int(x) for x in scalings])
    _check(prec.fn("multi_transform_forward")(n, arr, locs, ptrs, scs))
    return outputs

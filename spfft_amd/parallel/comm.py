"""Communicator handles for distributed grids without MPI."""
from __future__ import annotations

import ctypes
import threading
from typing import Callable, List

from ..ops import _lib
from ..ops._lib import lib


def _check(code):
    from ..grid import _check as chk
    chk(code)


class Communicator:
    """Owns a native SpfftAmdComm handle."""

    in_process = False  # ranks are threads of this process (LocalGroup)

    def __init__(self, handle):
        self.handle = handle

    @property
    def rank(self) -> int:
        v = ctypes.c_int()
        _check(lib().spfft_amd_comm_rank(self.handle, ctypes.byref(v)))
        return v.value

    @property
    def size(self) -> int:
        v = ctypes.c_int()
        _check(lib().spfft_amd_comm_size(self.handle, ctypes.byref(v)))
        return v.value

    def shm_check(self, iters: int = 200):
        """Collective. Node-local shared-memory collectives (the relay data plane's host
        synchronisation) against this communicator's own: microseconds per checked
        allgather + barrier round, ``(shm_us, comm_us)``; ``shm_us`` is None when the
        ranks cannot share a segment."""
        L = lib()
        if not hasattr(L, "spfft_amd_test_comm_shm_check"):
            raise RuntimeError("shm_check is a probe of the testing library: set SPFFT_AMD_LIBRARY to "
                               "spfft_amd/_native/libspfft_amd_testing.so")
        shm, com = ctypes.c_double(), ctypes.c_double()
        _check(L.spfft_amd_test_comm_shm_check(self.handle, int(iters), ctypes.byref(shm), ctypes.byref(com)))
        return (shm.value if shm.value >= 0 else None), com.value

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                lib().spfft_amd_comm_destroy(h)
            except Exception:
                pass
            self.handle = None


class LocalGroup:
    """`size` communicators of one in-process group; drive each from its own thread."""

    def __init__(self, size: int):
        arr = (ctypes.c_void_p * size)()
        _check(lib().spfft_amd_comm_create_local_group(size, arr))
        self.comms = [Communicator(ctypes.c_void_p(arr[r])) for r in range(size)]
        for c in self.comms:
            c.in_process = True

    def __getitem__(self, r):
        return self.comms[r]

    def __len__(self):
        return len(self.comms)


def run_ranks(size: int, fn: Callable[[int, Communicator], object]) -> List[object]:
    """Runs fn(rank, comm) on `size` threads sharing a LocalGroup; re-raises the first error."""
    group = LocalGroup(size)
    results: List[object] = [None] * size
    errors: List[BaseException] = []

    def body(r):
        try:
            results[r] = fn(r, group[r])
        except BaseException as e:  # noqa: BLE001
            errors.append(e)

    threads = [threading.Thread(target=body, args=(r,)) for r in range(size)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
    return results


class TorchDistComm(Communicator):
    """Control plane over torch.distributed.

    Uses a gloo group for host-side collectives (the default group when it is
    gloo, otherwise a new gloo group over the same ranks). The GPU data plane
    (RCCL) is created by the library and bootstrapped through allgather().
    """

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist

        self._dist = dist
        self._torch = torch
        if group is None:
            if dist.get_backend() == "gloo":
                group = dist.group.WORLD
            else:
                group = dist.new_group(backend="gloo")
        self._group = group
        self._rank = dist.get_rank(group)
        self._size = dist.get_world_size(group)

        def allgather(ctx, send, recv, nbytes):
            try:
                t = torch.empty(nbytes, dtype=torch.uint8)
                if nbytes:
                    ctypes.memmove(t.data_ptr(), send, nbytes)
                outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self._size)]
                dist.all_gather(outs, t, group=self._group)
                for r, o in enumerate(outs):
                    if nbytes:
                        ctypes.memmove(recv + r * nbytes, o.data_ptr(), nbytes)
                return 0
            except Exception:  # noqa: BLE001
                return 1

        def alltoallv(ctx, send, scounts, sdispls, recv, rcounts, rdispls):
            try:
                P = self._size
                sc = [scounts[i] for i in range(P)]
                sd = [sdispls[i] for i in range(P)]
                rc = [rcounts[i] for i in range(P)]
                rd = [rdispls[i] for i in range(P)]
                inp = torch.empty(sum(sc), dtype=torch.uint8)
                off = 0
                for i in range(P):
                    if sc[i]:
                        ctypes.memmove(inp.data_ptr() + off, send + sd[i], sc[i])
                    off += sc[i]
                out = torch.empty(sum(rc), dtype=torch.uint8)
                dist.all_to_all_single(out, inp, rc, sc, group=self._group)
                off = 0
                for i in range(P):
                    if rc[i]:
                        ctypes.memmove(recv + rd[i], out.data_ptr() + off, rc[i])
                    off += rc[i]
                return 0
            except Exception:  # noqa: BLE001
                return 1

        def barrier(ctx):
            try:
                dist.barrier(group=self._group)
                return 0
            except Exception:  # noqa: BLE001
                return 1

        # keep the ctypes callback objects alive for the lifetime of the handle
        self._cbs = (_lib.ALLGATHER_CB(allgather), _lib.ALLTOALLV_CB(alltoallv),
                     _lib.BARRIER_CB(barrier), _lib.DESTROY_CB(0))
        cb = _lib.CommCallbacks()
        cb.context = None
        cb.rank = self._rank
        cb.size = self._size
        cb.allgather, cb.alltoallv, cb.barrier, cb.destroy = self._cbs
        h = ctypes.c_void_p()
        _check(lib().spfft_amd_comm_create_callbacks(ctypes.byref(h), ctypes.byref(cb)))
        super().__init__(h)

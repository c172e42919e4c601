"""Multi-process probe of the RCCL data plane: P torch.distributed ranks (gloo
control plane), every rank on cuda:<LOCAL_RANK % ndev>; each runs a distributed
GPU transform whose pencil<->slab exchange goes through the library's RCCL
communicator, and checks it against the dense numpy oracle.

Launch: python -m torch.distributed.run --nproc-per-node P --master-addr 127.0.0.1 \
            --master-port 29531 tools/rccl_probe.py [exchange]
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spfft_amd as sp  # noqa: E402
from spfft_amd.parallel import TorchDistComm, make_distributed  # noqa: E402
from spfft_amd.utils.indices import distribute_sticks, sphere_indices  # noqa: E402
from spfft_amd.utils.oracle import dense_backward, max_rel_error  # noqa: E402


def _np(x):
    return x.cpu().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    host = "--host" in sys.argv
    exch_name = args[0] if args else "COMPACT_BUFFERED"
    exchange = getattr(sp.ExchangeType, exch_name)
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if "--rccl-net" in sys.argv:
        # ranks sharing one GPU through a real multi-rank RCCL communicator (one
        # virtual host per rank, RCCL socket transport on loopback): the
        # RcclDeviceComm path that ships to 8 GPUs, end to end
        os.environ["SPFFT_RCCL_VIRTUAL_HOSTS"] = "1"
    pu = sp.ProcessingUnit.HOST if host else sp.ProcessingUnit.GPU
    dev = "cuda"
    if not host:
        torch.cuda.set_device(local_rank % torch.cuda.device_count())
    dist.init_process_group("gloo")
    rank, P = dist.get_rank(), dist.get_world_size()
    comm = TorchDistComm()
    dims = (40, 36, 30)
    iters = 3
    for a in sys.argv[1:]:
        if a.startswith("--iters="):
            iters = int(a.split("=")[1])
        if a.startswith("--dims="):
            dims = tuple(int(v) for v in a.split("=")[1].split(","))
    gidx = sphere_indices(*dims, 0.5)
    parts = distribute_sticks(gidx, P, dims)
    s = make_distributed(comm, dims, gidx, processing_unit=pu, exchange_type=exchange)
    start = sum(len(p) for p in parts[:rank])
    e1 = e2 = 0.0
    # fresh values every iteration: a stale read of a previous exchange shows up
    for it in range(iters):
        rng = np.random.default_rng(5 + it)
        vals = rng.standard_normal(len(gidx)) + 1j * rng.standard_normal(len(gidx))
        ref = dense_backward(gidx, vals, dims)
        mine = vals[start:start + len(s.indices)]
        v = mine if host else torch.as_tensor(mine, device=dev)
        out = _np(s.transform.backward(v))
        e1 = max(e1, max_rel_error(out, ref[s.z_offset:s.z_offset + s.z_length]))
        f = _np(s.transform.forward(None, scaling=sp.Scaling.FULL))
        e2 = max(e2, max_rel_error(f, mine))
    tol = 1e-5 if "FLOAT" in exch_name else 1e-11
    ok = e1 < tol and e2 < tol
    kind = "" if host else f" [{s.grid.data_plane}]"
    if not host and s.grid.data_plane in ("ipc", "relay"):
        kind += f" self-test: {s.grid.data_plane_info.get('self_test')}"
    if not host:
        kind += f" channel priority: {s.grid.data_plane_info.get('channel_priority')}"
    print(f"rank {rank}/{P} {exch_name}{kind} x{iters}: backward err {e1:.2e} forward err {e2:.2e} "
          f"{'OK' if ok else 'FAIL'}", flush=True)
    del s
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()

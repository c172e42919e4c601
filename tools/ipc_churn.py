#!/usr/bin/env python3
"""Grid churn across processes on the peer-write (IPC) data plane: grids are created
collectively but dropped by each rank at a different time, the way a library Grid
lives in an application (reference contract: destroying a Grid is purely local,
src/memory/gpu_array.hpp:88).

Every round creates a grid (exchange type and stick / plane distribution drawn per
round, ranks with empty sides included) with two transforms on it, runs both on
different streams in turn against the dense oracle, then:
  - rank (round % P) drops its grid at once (and sleeps a little, so the others run
    ahead into the next round's collective creation),
  - the other ranks keep theirs alive until after the next round's grid exists.
The last round runs a fresh UNBUFFERED grid. Any error is agreed on (all_reduce)
and reported by rank 0; the exit status is nonzero on failure.

    python -m torch.distributed.run --standalone --local-addr=127.0.0.1 --nproc-per-node 3 \\
        tools/ipc_churn.py --rounds 12
"""
import argparse
import gc
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

EXCHANGES = ["UNBUFFERED", "COMPACT_BUFFERED", "COMPACT_BUFFERED_FLOAT", "BUFFERED", "BUFFERED_FLOAT"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--seed", type=int, default=3)
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    import spfft_amd as sp
    from spfft_amd.parallel import TorchDistComm
    from spfft_amd.utils.indices import calculate_num_local_xy_planes, create_value_indices
    from spfft_amd.utils.oracle import dense_backward, dense_forward, max_rel_error

    dist.init_process_group("gloo")
    rank, P = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
    rng = np.random.default_rng(a.seed)  # the same draws on every rank
    kept = []  # grids (and transforms) this rank has not dropped yet
    bad = 0
    for r in range(a.rounds):
        last = r == a.rounds - 1
        nx, ny, nz = dims = (int(rng.integers(8, 40)), int(rng.integers(8, 40)), int(rng.integers(8, 48)))
        exchange = "UNBUFFERED" if last else str(rng.choice(EXCHANGES))
        single = exchange.endswith("FLOAT") or bool(rng.random() < 0.3)
        sticks = [float(rng.integers(0, 3)) for _ in range(P)]
        if sum(sticks) == 0:
            sticks[0] = 1.0
        planes_d = [float(rng.integers(0, 3)) for _ in range(P)]
        if sum(planes_d) == 0:
            planes_d[-1] = 1.0
        parts = create_value_indices(rng, sticks, float(rng.uniform(0.4, 1.0)), 1.0, nx, ny, nz, False)
        planes = [calculate_num_local_xy_planes(q, nz, planes_d) for q in range(P)]
        offsets = np.concatenate([[0], np.cumsum(planes)])
        starts = np.concatenate([[0], np.cumsum([len(p) for p in parts])])
        all_idx = np.concatenate(parts)
        field = rng.standard_normal((nz, ny, nx)) + 1j * rng.standard_normal((nz, ny, nx))
        vals = dense_forward(field, all_idx, dims)
        ref = dense_backward(all_idx, vals, dims)
        ms = max(len(np.unique(p[:, 0].astype(np.int64) * ny + p[:, 1])) if len(p) else 0 for p in parts)
        tol = 2e-4 if single else 1e-10
        err, msg, plane = 0.0, "", "?"
        try:
            G = sp.GridFloat if single else sp.Grid
            grid = G(nx, ny, nz, max(1, ms), sp.ProcessingUnit.GPU, 1, max_local_z_length=max(planes),
                     comm=TorchDistComm(), exchange_type=getattr(sp.ExchangeType, exchange))
            ts = [grid.create_transform(sp.ProcessingUnit.GPU, sp.TransformType.C2C, nx, ny, nz,
                                        planes[rank], parts[rank]) for _ in range(2)]
            ts[0].set_stream(torch.cuda.Stream())  # the other stays on torch's current stream
            cnp = np.complex64 if single else np.complex128
            mine = np.ascontiguousarray(vals[starts[rank]:starts[rank + 1]], dtype=cnp)
            v = torch.as_tensor(mine, device="cuda")
            for t in ts:
                out = t.backward(v).cpu().numpy()
                if planes[rank]:
                    err = max(err, max_rel_error(out, ref[offsets[rank]:offsets[rank + 1]]))
                f = t.forward(None, scaling=sp.Scaling.FULL).cpu().numpy()
                if len(f):
                    err = max(err, max_rel_error(f, mine))
            plane = grid.data_plane
        except Exception as e:  # agreed on below
            err, msg = float("inf"), f"{type(e).__name__}: {e}"
            grid, ts = None, []
        # uneven teardown: one rank drops this round's grid now and lags behind,
        # the others keep it (and the previous round's) until the next grid exists
        if rank == r % P:
            grid = ts = None
            for g in kept:
                g.clear()
            kept = []
            gc.collect()
            time.sleep(0.05)
        else:
            for g in kept[:-1]:
                g.clear()
            kept = kept[-1:] + [[grid, ts]]
        e = torch.tensor([err if np.isfinite(err) else 1e300], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        worst = float(e.item())
        ok = worst < tol
        bad += 0 if ok else 1
        if rank == 0:
            print(f"{'ok  ' if ok else 'FAIL'} round {r}: dims={dims} {exchange} plane={plane} "
                  f"sticks={sticks} planes={planes_d} err={worst:.2e} {msg}", flush=True)
        elif msg:
            print(f"rank {rank} round {r}: {msg}", flush=True)
    kept = []
    gc.collect()
    if rank == 0:
        print(f"{a.rounds - bad}/{a.rounds} rounds passed", flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

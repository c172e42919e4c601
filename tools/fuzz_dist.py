#!/usr/bin/env python3
"""Randomised multi-process sweep: the cases of tools/fuzz_gpu.py (every engine path,
type, precision, random stick / plane distributions including empty ranks, every
exchange type, centred indices) on one OS process per rank over torch.distributed,
the launch path of bench.py. On a GPU box the ranks share its device: the data plane
is the IPC peer-write plane, or one multi-rank RCCL communicator with
SPFFT_RCCL_VIRTUAL_HOSTS=1.

    python -m torch.distributed.run --standalone --local-addr=127.0.0.1 --nproc-per-node 3 \\
        tools/fuzz_dist.py --cases 50 [--host]
"""
import argparse
import gc
import importlib.util
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _fuzz_module():
    spec = importlib.util.spec_from_file_location("fuzz_gpu", os.path.join(REPO, "tools", "fuzz_gpu.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=50)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max-elems", type=int, default=1 << 19)
    ap.add_argument("--host", action="store_true")
    ap.add_argument("--only", type=int, default=-1, help="run only this case (the draws of the others still happen)")
    ap.add_argument("--teardown", choices=["lazy", "collective"], default="lazy",
                    help="collective: drop each case's grid on every rank, then barrier, before the next case")
    ap.add_argument("--maxima", choices=["global", "local"], default="global",
                    help="local: every rank passes its own stick count and plane count as the "
                         "grid maxima (zero on empty ranks), so exchange sides differ per rank")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    import spfft_amd as sp
    from spfft_amd.parallel import TorchDistComm
    from spfft_amd.utils.indices import calculate_num_local_xy_planes, create_value_indices
    from spfft_amd.utils.oracle import dense_backward, dense_forward, max_rel_error

    fz = _fuzz_module()
    dist.init_process_group("gloo")
    rank, P = dist.get_rank(), dist.get_world_size()
    if not a.host:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count()))
    PU = sp.ProcessingUnit.HOST if a.host else sp.ProcessingUnit.GPU
    rng = np.random.default_rng(a.seed)  # the same draws on every rank
    bad = 0
    grid = t = None
    for c in range(a.cases):
        if a.teardown == "collective":
            grid = t = None
            gc.collect()
            dist.barrier()
        nx, ny, nz = dims = fz.draw_dims(rng, a.max_elems)
        r2c = bool(rng.random() < 0.4)
        single = bool(rng.random() < 0.4)
        exchange = str(rng.choice(fz.EXCHANGES))
        stick_dist = [float(rng.integers(0, 3)) for _ in range(P)]
        if sum(stick_dist) == 0:
            stick_dist[0] = 1.0
        plane_dist = [float(rng.integers(0, 3)) for _ in range(P)]
        if sum(plane_dist) == 0:
            plane_dist[-1] = 1.0
        parts = create_value_indices(rng, stick_dist, float(rng.uniform(0.3, 1.0)),
                                     float(rng.uniform(0.4, 1.0)), nx, ny, nz, r2c)
        centred = bool(rng.random() < 0.3)
        if centred:
            half, n3 = np.array([nx // 2, ny // 2, nz // 2]), np.array([nx, ny, nz])
            parts = [np.where(p > half, p - n3, p).astype(np.int32) for p in parts]
        planes = [calculate_num_local_xy_planes(r, nz, plane_dist) for r in range(P)]
        offsets = np.concatenate([[0], np.cumsum(planes)])
        all_idx = np.concatenate(parts)
        space = rng.standard_normal((nz, ny, nx))
        field = space if r2c else space + 1j * rng.standard_normal((nz, ny, nx))
        vals = dense_forward(field, all_idx, dims, r2c=r2c)
        ref = dense_backward(all_idx, vals, dims, r2c=r2c)
        starts = np.concatenate([[0], np.cumsum([len(p) for p in parts])])
        sticks = [len(np.unique(p[:, 0].astype(np.int64) * ny + p[:, 1])) if len(p) else 0 for p in parts]
        ms = max(sticks)
        tol = 2e-4 if (single or exchange.endswith("FLOAT")) else 1e-10
        if a.only >= 0 and c != a.only:
            continue
        err = 0.0
        msg = ""
        eb = ef = 0.0
        try:
            G = sp.GridFloat if single else sp.Grid
            if a.maxima == "local":
                gs, gz = sticks[rank], planes[rank]
            else:
                gs, gz = max(1, ms), max(planes)
            grid = G(nx, ny, nz, gs, PU, 1, max_local_z_length=gz, comm=TorchDistComm(),
                     exchange_type=getattr(sp.ExchangeType, exchange))
            t = grid.create_transform(PU, sp.TransformType.R2C if r2c else sp.TransformType.C2C,
                                      nx, ny, nz, planes[rank], parts[rank])
            cnp = np.complex64 if single else np.complex128
            rnp = np.float32 if single else np.float64
            v = np.ascontiguousarray(vals[starts[rank]:starts[rank + 1]], dtype=cnp)
            slab = np.ascontiguousarray(field[offsets[rank]:offsets[rank + 1]], dtype=rnp if r2c else cnp)
            if not a.host:
                v, slab = torch.as_tensor(v, device="cuda"), torch.as_tensor(slab, device="cuda")
            out = t.backward(v)
            out = out if a.host else out.cpu().numpy()
            eb = max_rel_error(out, ref[offsets[rank]:offsets[rank + 1]]) if planes[rank] else 0.0
            f = t.forward(slab)
            f = f if a.host else f.cpu().numpy()
            ef = max_rel_error(f, vals[starts[rank]:starts[rank + 1]]) if len(f) else 0.0
            err = max(eb, ef)
            if a.only >= 0:
                print(f"rank {rank}: values={len(parts[rank])} planes={planes[rank]} backward={eb:.2e} "
                      f"forward={ef:.2e}", flush=True)
            plane = grid.data_plane if not a.host else "host"
        except Exception as e:  # reported, and agreed on below
            err, msg, plane = float("inf"), f"{type(e).__name__}: {e}", "?"
        e = torch.tensor([err if np.isfinite(err) else 1e300], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        worst = float(e.item())
        ok = worst < tol
        bad += 0 if ok else 1
        if rank == 0:
            print(f"{'ok  ' if ok else 'FAIL'} case {c}: dims={dims} {'R2C' if r2c else 'C2C'} "
                  f"{'fp32' if single else 'fp64'} P={P} {exchange} plane={plane} sticks={stick_dist} "
                  f"planes={plane_dist}{' centred' if centred else ''} err={worst:.2e} {msg}", flush=True)
    if rank == 0:
        print(f"{a.cases - bad}/{a.cases} passed", flush=True)
    dist.destroy_process_group()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

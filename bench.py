#!/usr/bin/env python3
"""Headline benchmark: 3D C2C transforms/sec, 256^3 spherical cutoff, 1/2/4/8 MI355X.

One step = one backward (frequency -> space) + one forward (space -> frequency)
transform of the 256^3 grid with the spherical cutoff |k| <= N/2 (≈8.78 M
frequency values, 51,431 z-sticks), fp64 complex, exactly like one repeat of
the reference benchmark (reference: tests/programs/benchmark.cpp:85-88).
Data is synthetic (random values),
inputs and outputs live in GPU memory ("gpu-gpu" mode of the reference).

A step runs 4 independent transforms of that problem (--transforms, the
reference benchmark's -m, tests/programs/benchmark.cpp:142, 84-96): multi_transform_backward +
multi_transform_forward, one HIP stream per transform, so one transform's
all-to-all and kernel tails overlap the others' kernels. transforms/sec =
2 * transforms * steps / elapsed. --transforms 1 times single calls.

Multi-GPU: launched by torch.distributed.run, one rank per GPU; z-sticks and
xy-planes are split evenly over ranks and the pencil <-> slab redistribution
runs as RCCL all-to-all(v) over xGMI inside the library. The problem size is
fixed as N grows (strong scaling); `value` is the whole-job rate.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# transforms/s of the reference's vendor-FFT calls alone on one MI355X, 256^3
# C2C fp64 r = N/2 (tools/ref_pipeline_bench.py), by the
# number of transforms per step (T on T streams)
REF_FFT_ONLY_256_BY_T = {1: 2210.2, 4: 2418.3}  # profiles/r3/comparator/


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--cutoff", type=float, default=0.5)
    ap.add_argument("--exchange", default="compact",
                    choices=["compact", "compactFloat", "buffered", "bufferedFloat", "unbuffered"])
    ap.add_argument("--precision", default="double", choices=["double", "single"])
    ap.add_argument("--type", default="c2c", choices=["c2c", "r2c"])
    ap.add_argument("--transforms", type=int, default=4,
                    help="independent transforms per step, run with multi_transform_backward/"
                         "forward on one stream each (the reference benchmark's -m): one "
                         "transform's all-to-all overlaps the others' FFT kernels")
    ap.add_argument("--streams", default="auto", choices=["auto", "per-transform", "one"],
                    help="with --sync stream and T > 1: one stream per transform (their kernels "
                         "and exchanges overlap), or all transforms on torch's current stream "
                         "(identical single-GPU transforms then run batched, one launch per "
                         "stage for up to 8). auto: one stream on 1 GPU (batched launches "
                         "measured +2%% over 4 streams at 256^3, profiles/r3/t4_streams.txt), "
                         "per-transform streams on N > 1 GPUs (one transform's all-to-all "
                         "overlaps the others' kernels; distributed plans do not batch)")
    ap.add_argument("--timing", action="store_true", help="print the native timing tree")
    ap.add_argument("--check", action="store_true",
                    help="after timing: round-trip error on every rank and, on one rank, the "
                         "backward transform against the dense numpy oracle")
    ap.add_argument("--sync", default="stream", choices=["stream", "call"],
                    help="stream: transforms are stream-ordered on torch's current stream (no host "
                         "wait per call; the timed loop still ends with a device synchronize); "
                         "call: every backward/forward call blocks until done (SpFFT default)")
    return ap.parse_args()


def _check(a, sp, t, values, gidx, dims, ttype, world):
    """Max relative error of the round trip (and of the backward vs numpy on 1 rank)."""
    import numpy as np
    import torch
    from spfft_amd.utils.oracle import dense_backward, max_rel_error
    out = torch.empty_like(values)
    space = t.backward(values)
    torch.cuda.synchronize()
    err = {}
    if world == 1 and max(dims) <= 512:  # the dense numpy oracle (host memory, time)
        ref = dense_backward(gidx, values.cpu().numpy(), dims,
                             r2c=(ttype == sp.TransformType.R2C))
        err["backward_vs_numpy"] = max_rel_error(space.cpu().numpy(), ref)
    t.forward(None, output=out, scaling=sp.Scaling.FULL)
    torch.cuda.synchronize()
    if ttype == sp.TransformType.R2C:
        # random R2C input is not hermitian on the x = 0 plane: compare the second
        # round trip with the first (the round trip is a projection)
        ref_rt = out.clone()
        t.backward(ref_rt)
        t.forward(None, output=out, scaling=sp.Scaling.FULL)
        torch.cuda.synchronize()
        err["roundtrip"] = max_rel_error(out.cpu().numpy(), ref_rt.cpu().numpy())
    else:
        err["roundtrip"] = max_rel_error(out.cpu().numpy(), values.cpu().numpy())
    return err


def main():
    a = parse()
    import numpy as np
    import torch

    import spfft_amd as sp
    from spfft_amd.utils.indices import distribute_sticks, sphere_indices

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE {world}")
    # one rank per GPU; more ranks than GPUs (rehearsal on a small box) share
    # devices round-robin and the library then moves data by IPC peer writes
    ndev = max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank % ndev)
    dev = torch.device("cuda", local_rank % ndev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # torch.distributed is the control plane only (plan setup, barriers,
        # the timing reduction): gloo. The transform's all-to-all runs on the
        # library's own RCCL communicator over xGMI.
        dist.init_process_group("gloo")

    n = a.size
    dims = (n, n, n)
    ttype = sp.TransformType.R2C if a.type == "r2c" else sp.TransformType.C2C
    gidx = sphere_indices(*dims, a.cutoff, r2c=(ttype == sp.TransformType.R2C))
    exch = {"compact": sp.ExchangeType.COMPACT_BUFFERED,
            "compactFloat": sp.ExchangeType.COMPACT_BUFFERED_FLOAT,
            "buffered": sp.ExchangeType.BUFFERED,
            "bufferedFloat": sp.ExchangeType.BUFFERED_FLOAT,
            "unbuffered": sp.ExchangeType.UNBUFFERED}[a.exchange]
    single = a.precision == "single"
    GridCls = sp.GridFloat if single else sp.Grid
    cdtype = torch.complex64 if single else torch.complex128

    def make_transform():
        # every transform owns its grid (multi_transform rejects shared grids)
        if world == 1:
            g = GridCls(n, n, n, n * n, sp.ProcessingUnit.GPU, 1)
            return g, g.create_transform(sp.ProcessingUnit.GPU, ttype, n, n, n, n, gidx), gidx
        from spfft_amd.parallel import TorchDistComm, make_distributed
        setup = make_distributed(TorchDistComm(), dims, gidx, processing_unit=sp.ProcessingUnit.GPU,
                                 transform_type=ttype, exchange_type=exch, single=single)
        return setup.grid, setup.transform, setup.indices

    T = max(1, a.transforms)
    made = [make_transform() for _ in range(T)]
    grids = [m[0] for m in made]
    ts = [m[1] for m in made]
    local = made[0][2]
    grid, t = grids[0], ts[0]

    plane = grid.data_plane if world > 1 else "none"
    if a.streams == "auto":
        a.streams = "one" if world == 1 else "per-transform"
    streams = []
    if a.sync == "stream":
        if T == 1 or a.streams == "one":
            for tr in ts:
                tr.set_stream(torch.cuda.current_stream(), synchronous=False)
        else:
            streams = [torch.cuda.Stream() for _ in range(T)]
            for tr, st in zip(ts, streams):
                tr.set_stream(st, synchronous=False)

    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    vals = [torch.randn(len(local), dtype=cdtype, device=dev, generator=gen) for _ in range(T)]
    outs = [torch.empty_like(v) for v in vals]
    values, out = vals[0], outs[0]

    def step():
        if T == 1:
            t.backward(values)
            t.forward(None, output=out)
        else:
            sp.multi_transform_backward(ts, vals)
            sp.multi_transform_forward(ts, outputs=outs)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(a.warmup):
        step()
    barrier()
    if a.timing:
        sp.timing_reset()
        sp.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    check = None
    if a.check:
        check = _check(a, sp, t, values, gidx, dims, ttype, world)
        if dist is not None:
            # every rank's round trip counts: rank 0 reports the worst one
            e = torch.tensor([check["roundtrip"]], dtype=torch.float64)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            check["roundtrip"] = float(e.item())
            check["ranks_checked"] = world
    # ranks that share a device (rehearsal on a small box) are not a multi-GPU
    # measurement: record how many distinct devices the job really used
    n_devices = min(world, ndev)
    ms_per_step = 1e3 * elapsed / a.steps
    rate = 2.0 * T * a.steps / elapsed
    # the reference's FFT calls alone (rocFFT via torch.fft)
    # on one MI355X, an upper bound on its throughput for the headline config;
    # no measured reference exists for other configs or for N > 1 GPUs
    headline = (n == 256 and a.cutoff == 0.5 and a.type == "c2c" and not single)
    # comparator per protocol: the reference algorithm's rocFFT calls alone on one
    # MI355X, one transform at a time (T = 1) or T transforms on T streams
    # (tools/ref_pipeline_bench.py --transforms T), so the ratio does not mix the
    # multi-transform overlap into the per-transform speed-up
    ref_rate = REF_FFT_ONLY_256_BY_T.get(T) if (headline and world == 1) else None
    vs_baseline = rate / ref_rate if ref_rate else None
    if a.timing:
        for tr in ts:  # completes the GPU stage intervals (gpu/<direction>/<stage>)
            tr.synchronize()
    if rank == 0:
        if a.timing:
            print(sp.timing_report(), file=sys.stderr)
        rec = {
            "metric": "3D C2C transforms/sec, 256^3 spherical cutoff, 1/2/4/8 MI355X",
            "value": rate,
            "unit": "transforms/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": vs_baseline,
            "vs_baseline_basis": (f"value / {ref_rate:.1f}: the reference algorithm's rocFFT calls "
                                  f"alone on one MI355X with the same {T} transform(s) per step "
                                  f"(BASELINE.md B7, tools/ref_pipeline_bench.py --transforms {T})"
                                  if vs_baseline else None),
            "dtype": "fp32" if single else "fp64",
            "data": "synthetic (random complex values on the spherical-cutoff index set)",
            "config": {
                "model": f"sparse 3D FFT {n}^3 {a.type.upper()} spherical cutoff r={a.cutoff}*N",
                "global_batch": 2 * T,
                "transforms_per_step": T,
                "seq_len": n,
                "parallelism": f"slab/pencil x{world} ({a.exchange} all-to-all)",
                "num_frequency_values": int(len(gidx)),
                "exchange": a.exchange,
                "data_plane": plane,
                "distinct_devices": n_devices,
                "shared_device": n_devices < world,
                "sync": a.sync,
                "streams": a.streams if T > 1 else "one",
                "check_error": check,
                "step": ("1 backward + 1 forward transform" if T == 1 else
                         f"multi_transform backward + forward of {T} independent transforms"),
            },
        }
        print(json.dumps(rec), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

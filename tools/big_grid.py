#!/usr/bin/env python3
"""One large transform on one GPU: checks the device-memory model of docs/MEMORY.md
(tools/memory_model.py) against a real allocation, and the round trip of the
transform at that size.

    python tools/big_grid.py --size 1536 [--precision double] [--type c2c] [--reps 3]

Prints one JSON line: the grid's device bytes (hipMemGetInfo before and after the
grid and transform are created), the model's prediction, the frequency-value
bytes, the median time of a backward+forward pair and the round-trip error
max |forward(backward(v)) - v| / max |v| with full scaling, computed on the GPU.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1536)
    ap.add_argument("--precision", default="double", choices=["double", "single"])
    ap.add_argument("--type", default="c2c", choices=["c2c", "r2c"])
    ap.add_argument("--cutoff", type=float, default=0.5)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()

    import threading
    import torch

    # progress line every 30 s (index generation and planning of ~2e9 values are long)
    start = time.perf_counter()
    stop = threading.Event()

    def beat():
        while not stop.wait(30):
            print(f"... {time.perf_counter() - start:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()

    import spfft_amd as sp
    from spfft_amd.utils.indices import sphere_indices
    import memory_model

    n = a.size
    single = a.precision == "single"
    r2c = a.type == "r2c"
    ttype = sp.TransformType.R2C if r2c else sp.TransformType.C2C
    t0 = time.perf_counter()
    gidx = sphere_indices(n, n, n, a.cutoff, r2c=r2c)
    t_idx = time.perf_counter() - t0
    print(f"indices: {len(gidx)} in {t_idx:.1f} s", file=sys.stderr, flush=True)

    torch.cuda.init()
    torch.cuda.synchronize()
    free0, total = torch.cuda.mem_get_info()
    GridCls = sp.GridFloat if single else sp.Grid
    t0 = time.perf_counter()
    # the grid sized for the index set's sticks (the model's pi r^2), not n * n
    import numpy as np
    sticks = int(np.unique(gidx[:, 0].astype(np.int64) * n + gidx[:, 1]).size)
    grid = GridCls(n, n, n, sticks, sp.ProcessingUnit.GPU, 1)
    t = grid.create_transform(sp.ProcessingUnit.GPU, ttype, n, n, n, n, gidx)
    t_plan = time.perf_counter() - t0
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    grid_bytes = free0 - free1
    print(f"grid + transform: {grid_bytes / 1e9:.1f} GB in {t_plan:.1f} s", file=sys.stderr, flush=True)

    cdtype = torch.complex64 if single else torch.complex128
    gen = torch.Generator(device="cuda")
    gen.manual_seed(7)
    vals = torch.randn(len(gidx), dtype=cdtype, device="cuda", generator=gen)
    out = torch.empty_like(vals)
    del gidx
    t.set_stream(torch.cuda.current_stream(), synchronous=False)

    times = []
    for _ in range(a.reps + 1):
        torch.cuda.synchronize()
        s = time.perf_counter()
        t.backward(vals)
        t.forward(None, output=out, scaling=sp.Scaling.FULL)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - s)
        print(f"pair {1e3 * times[-1]:.1f} ms", file=sys.stderr, flush=True)
    base = vals
    if r2c:  # random input is not hermitian on x = 0: compare two round trips
        base = out.clone()
        t.backward(base)
        t.forward(None, output=out, scaling=sp.Scaling.FULL)
    torch.cuda.synchronize()
    err, scale = 0.0, 0.0
    chunk = 1 << 26
    for i in range(0, base.numel(), chunk):
        b, o = base[i:i + chunk], out[i:i + chunk]
        err = max(err, float((o - b).abs().max().item()))
        scale = max(scale, float(b.abs().max().item()))
    free2, _ = torch.cuda.mem_get_info()
    model, _ = memory_model.grid_bytes(n, 1, 8 if single else 16, cutoff=a.cutoff, r2c=r2c)
    pairs = sorted(times[1:])
    rec = {
        "dims": [n, n, n], "type": a.type, "precision": a.precision, "cutoff": a.cutoff,
        "num_values": int(vals.numel()), "num_sticks": sticks,
        "values_bytes": int(vals.numel() * vals.element_size()),
        "grid_device_bytes_measured": int(grid_bytes),
        "grid_device_bytes_model": int(model),
        "device_bytes_in_use_total": int(total - free2),
        "device_total_bytes": int(total),
        "pair_ms_median": 1e3 * pairs[len(pairs) // 2],
        "roundtrip": err / (scale or 1.0),
        "plan_s": t_plan, "indices_s": t_idx,
    }
    stop.set()
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

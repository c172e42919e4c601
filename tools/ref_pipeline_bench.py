#!/usr/bin/env python3
"""Comparator for BASELINE.md row B6: the reference's GPU algorithm on MI355X
with the vendor FFT, written with torch ops (torch.fft is hipFFT/rocFFT on ROCm).

The reference publishes no numbers, and its ROCm build needs FFTW for the host
side, which this image does not have. This script measures what its GPU path
does on the same hardware, stage by stage (reference: src/execution/
execution_gpu.cpp:249-376, one rank, C2C):

  backward: memset sticks + decompress (compression_gpu.hpp:71-78)
            -> in-place batched z-FFT (transform_1d_gpu.hpp:116-126)
            -> memset planes + stick->plane scatter (transpose_gpu.hpp:95-104)
            -> batched 2D xy-FFT (transform_2d_gpu.hpp:115-125)
  forward:  2D xy-FFT -> plane->stick gather -> z-FFT -> compress

Rows printed (one JSON line each, transforms/s = 2 * steps / elapsed):
  * "ref_pipeline": the whole pipeline above (torch scatter/gather kernels
    stand in for the reference's pack kernels K2-K5);
  * "ref_fft_only": only the vendor FFT calls of that pipeline (z-batch +
    2D batch, both directions): a lower bound on the reference's step time
    even if its pack/unpack kernels cost nothing;
  * "dense_fftn": a dense 3D Z2Z ifftn + fftn of the full N^3 grid.

With --transforms T, T independent copies of each row run per step, one HIP
stream each (the comparator of bench.py's multi_transform headline, where T
transforms per step overlap on T streams); transforms/s = 2 * T * steps / elapsed.

Usage: python tools/ref_pipeline_bench.py [--size 256] [--cutoff 0.5] [--steps 20] [--transforms T]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--cutoff", type=float, default=0.5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--precision", default="double", choices=["double", "single"])
    ap.add_argument("--transforms", type=int, default=1)
    a = ap.parse_args()

    import numpy as np
    import torch

    from spfft_amd.utils.indices import sphere_indices

    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    cdt = torch.complex128 if a.precision == "double" else torch.complex64
    n = a.size
    X = Y = Z = n
    idx = sphere_indices(X, Y, Z, a.cutoff)
    # storage indices (centred -> [0, n)), sticks sorted by key x*Y + y
    st = np.where(idx < 0, idx + n, idx).astype(np.int64)
    key = st[:, 0] * Y + st[:, 1]
    ukeys, slot = np.unique(key, return_inverse=True)
    S = len(ukeys)
    val_idx = torch.as_tensor(slot * Z + st[:, 2], device=dev)  # value -> stick-flat position
    sx, sy = ukeys // Y, ukeys % Y
    plane_idx = torch.as_tensor(sy * X + sx, device=dev)  # stick -> position in a [y][x] plane
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    vals = torch.randn(len(idx), dtype=cdt, device=dev, generator=g)
    out = torch.empty_like(vals)

    sticks = torch.empty(S * Z, dtype=cdt, device=dev)
    planes = torch.empty(Z, Y * X, dtype=cdt, device=dev)

    def backward():
        sticks.zero_()
        sticks[val_idx] = vals
        s = torch.fft.ifft(sticks.view(S, Z), dim=1, norm="forward")  # unnormalised, +i sign
        planes.zero_()
        planes[:, plane_idx] = s.t()
        return torch.fft.ifft2(planes.view(Z, Y, X), norm="forward")

    def forward(space):
        p = torch.fft.fft2(space, norm="backward").view(Z, Y * X)
        s = p[:, plane_idx].t().contiguous()
        s = torch.fft.fft(s, dim=1, norm="backward")
        out.copy_(s.view(-1)[val_idx])

    def pipeline():
        forward(backward())

    zin = torch.randn(S, Z, dtype=cdt, device=dev, generator=g)
    pin = torch.randn(Z, Y, X, dtype=cdt, device=dev, generator=g)

    def fft_only():
        torch.fft.ifft(zin, dim=1, norm="forward")
        torch.fft.ifft2(pin, norm="forward")
        torch.fft.fft2(pin)
        torch.fft.fft(zin, dim=1)

    dense = torch.randn(Z, Y, X, dtype=cdt, device=dev, generator=g)

    def dense_fftn():
        torch.fft.fftn(torch.fft.ifftn(dense, norm="forward"))

    # correctness of the pipeline itself: backward vs the dense oracle
    from spfft_amd.utils.oracle import dense_backward, max_rel_error
    if n <= 128:
        ref = dense_backward(idx, vals.cpu().numpy(), (X, Y, Z))
        err = max_rel_error(backward().cpu().numpy(), ref)
    else:
        space = backward()
        forward(space)
        sync()
        err = max_rel_error((out / (X * Y * Z)).cpu().numpy(), vals.cpu().numpy())

    T = max(1, a.transforms)
    streams = [torch.cuda.Stream() for _ in range(T)] if (T > 1 and dev.type == "cuda") else []

    def run(fn):
        if not streams:
            fn()
            return
        cur = torch.cuda.current_stream()
        for st in streams:
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                fn()
        for st in streams:
            cur.wait_stream(st)

    for name, fn in (("ref_pipeline", pipeline), ("ref_fft_only", fft_only),
                     ("dense_fftn", dense_fftn)):
        if T > 1 and name == "ref_pipeline":
            continue  # shares its buffers across calls: one stream only
        for _ in range(a.warmup):
            run(fn)
        sync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            run(fn)
        sync()
        el = time.perf_counter() - t0
        rec = {"row": name, "size": n, "cutoff": a.cutoff, "precision": a.precision,
               "transforms_per_step": T if streams else 1,
               "transforms_per_s": 2.0 * (T if streams else 1) * a.steps / el,
               "ms_per_step": 1e3 * el / a.steps, "sticks": S, "values": len(idx)}
        if name == "ref_pipeline":
            rec["check_error"] = err
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

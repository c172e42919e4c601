"""Transforms/s of one transform with arbitrary dims (long-line path rates):
backward + forward per step, full-sphere cutoff r = N/2 per axis, on cuda:0.

    python tools/long_bench.py --dims 64,64,8192 [--precision single] [--type r2c]
Run under rocprofv3 --kernel-trace --stats to split the time per kernel.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dims", required=True)
    ap.add_argument("--precision", default="double", choices=["double", "single"])
    ap.add_argument("--type", default="c2c", choices=["c2c", "r2c"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--cutoff", type=float, default=0.5)
    a = ap.parse_args()
    import torch
    import spfft_amd as sp
    from spfft_amd.utils.indices import sphere_indices
    dims = tuple(int(v) for v in a.dims.split(","))
    nx, ny, nz = dims
    r2c = a.type == "r2c"
    single = a.precision == "single"
    idx = sphere_indices(nx, ny, nz, a.cutoff, r2c=r2c)
    G = sp.GridFloat if single else sp.Grid
    g = G(nx, ny, nz, nx * ny, sp.ProcessingUnit.GPU, 1)
    t = g.create_transform(sp.ProcessingUnit.GPU, sp.TransformType.R2C if r2c else sp.TransformType.C2C,
                           nx, ny, nz, nz, idx)
    t.set_stream(torch.cuda.current_stream(), synchronous=False)
    cdt = torch.complex64 if single else torch.complex128
    v = torch.randn(len(idx), dtype=cdt, device="cuda")
    out = torch.empty_like(v)
    for _ in range(2):
        t.backward(v)
        t.forward(None, output=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        t.backward(v)
        t.forward(None, output=out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    t.forward(None, output=out, scaling=sp.Scaling.FULL)
    t.backward(v)
    t.forward(None, output=out, scaling=sp.Scaling.FULL)
    torch.cuda.synchronize()
    err = float(((out - v).abs().max() / v.abs().max()).item())
    print(f"dims={dims} {a.type} {a.precision} values={len(idx)}: {1e3 * dt:.3f} ms per pair "
          f"({2 / dt:.1f} transforms/s), round-trip error {err:.2e}", flush=True)


if __name__ == "__main__":
    main()

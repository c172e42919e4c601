"""Host engine (SPFFT_PU_HOST) throughput: backward + forward per step, spherical
cutoff r = N/2, for a list of sizes and thread counts.

    python tools/host_bench.py [--sizes 64,128] [--threads 1,2,4,8] [--type c2c|r2c]
                               [--precision double|single] [--steps 5]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spfft_amd as sp  # noqa: E402
from spfft_amd.utils.indices import sphere_indices  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="64,128")
    ap.add_argument("--threads", default="1,2,4,8")
    ap.add_argument("--type", default="c2c", choices=["c2c", "r2c"])
    ap.add_argument("--precision", default="double", choices=["double", "single"])
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    r2c = a.type == "r2c"
    single = a.precision == "single"
    G = sp.GridFloat if single else sp.Grid
    for n in (int(s) for s in a.sizes.split(",")):
        idx = sphere_indices(n, n, n, 0.5, r2c=r2c)
        rng = np.random.default_rng(0)
        vals = rng.standard_normal(len(idx)) + 1j * rng.standard_normal(len(idx))
        vals = vals.astype(np.complex64 if single else np.complex128)
        for th in (int(s) for s in a.threads.split(",")):
            g = G(n, n, n, n * n, sp.ProcessingUnit.HOST, th)
            t = g.create_transform(sp.ProcessingUnit.HOST,
                                   sp.TransformType.R2C if r2c else sp.TransformType.C2C,
                                   n, n, n, n, idx)
            out = np.empty_like(vals)
            t.backward(vals)
            t.forward(None, output=out)
            t0 = time.perf_counter()
            for _ in range(a.steps):
                t.backward(vals)
                t.forward(None, output=out)
            dt = (time.perf_counter() - t0) / a.steps
            print(f"{n}^3 {a.type} {a.precision} threads={th}: {1e3 * dt:8.1f} ms per step "
                  f"({2 / dt:8.1f} transforms/s)", flush=True)


if __name__ == "__main__":
    main()

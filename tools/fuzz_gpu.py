#!/usr/bin/env python3
"""Randomised GPU correctness sweep against the dense numpy oracle.

Each case draws dimensions from lengths that select every engine path (compile-time
powers of two and mixed-radix lengths, run-time lengths, in-LDS Bluestein primes, and
the four-step for long lines: 2048, 4096, 6144, 8192 and the prime 4099), a transform
type, a precision, 1-3 virtual ranks with random stick / plane distributions and an
exchange type, then checks backward and forward against numpy.

    python tools/fuzz_gpu.py --cases 200 --seed 1 [--max-elems 1048576]

Prints one line per failing case and a summary; exit status 1 on any failure.
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHORT = [1, 2, 3, 4, 5, 7, 8, 11, 12, 13, 16, 17, 20, 31, 32, 48, 60, 64, 97, 100, 127, 128, 131,
         200, 240, 256]
LONG = [512, 1000, 1024, 1536, 2048, 4096, 4099, 6144, 8192]
EXCHANGES = ["COMPACT_BUFFERED", "COMPACT_BUFFERED_FLOAT", "BUFFERED", "BUFFERED_FLOAT", "UNBUFFERED"]


def draw_dims(rng, max_elems):
    while True:
        dims = [int(rng.choice(SHORT)) for _ in range(3)]
        if rng.random() < 0.35:  # one long axis
            dims[int(rng.integers(3))] = int(rng.choice(LONG))
        if int(np.prod(dims)) <= max_elems:
            return tuple(dims)


def run_case(rng, case, max_elems, host=False):
    import torch
    import spfft_amd as sp
    from spfft_amd.parallel import run_ranks
    from spfft_amd.utils.indices import calculate_num_local_xy_planes, create_value_indices
    from spfft_amd.utils.oracle import dense_backward, dense_forward, max_rel_error

    nx, ny, nz = dims = draw_dims(rng, max_elems)
    r2c = bool(rng.random() < 0.4)
    single = bool(rng.random() < 0.4)
    P = int(rng.choice([1, 1, 2, 3]))
    exchange = str(rng.choice(EXCHANGES))
    fill = float(rng.uniform(0.3, 1.0))
    stick_dist = [float(rng.integers(0, 3)) for _ in range(P)]
    if sum(stick_dist) == 0:
        stick_dist[0] = 1.0
    plane_dist = [float(rng.integers(0, 3)) for _ in range(P)]
    if sum(plane_dist) == 0:
        plane_dist[-1] = 1.0
    parts = create_value_indices(rng, stick_dist, fill, float(rng.uniform(0.4, 1.0)), nx, ny, nz, r2c)
    centred = bool(rng.random() < 0.3)
    if centred:  # the same index set in centred form (negative frequencies)
        half = np.array([nx // 2, ny // 2, nz // 2])
        n3 = np.array([nx, ny, nz])
        parts = [np.where(p > half, p - n3, p).astype(np.int32) for p in parts]
    multi = P == 1 and bool(rng.random() < 0.25)
    planes = [calculate_num_local_xy_planes(r, nz, plane_dist) for r in range(P)]
    offsets = np.concatenate([[0], np.cumsum(planes)])
    all_idx = np.concatenate(parts)
    space = rng.standard_normal((nz, ny, nx))
    field = space if r2c else space + 1j * rng.standard_normal((nz, ny, nx))
    vals = dense_forward(field, all_idx, dims, r2c=r2c)
    ref = dense_backward(all_idx, vals, dims, r2c=r2c)
    starts = np.concatenate([[0], np.cumsum([len(p) for p in parts])])
    ttype = sp.TransformType.R2C if r2c else sp.TransformType.C2C
    PU = sp.ProcessingUnit.HOST if host else sp.ProcessingUnit.GPU
    nthreads = 2 if host else 1

    def dev(x, complex_):
        """Input array for the processing unit (numpy on the host, a GPU tensor)."""
        if host:
            return np.ascontiguousarray(x, dtype=(np.complex64 if single else np.complex128) if complex_
                                        else (np.float32 if single else np.float64))
        return torch.as_tensor(x, dtype=(cdt if complex_ else rdt), device="cuda")

    def npy(y):
        return y if host else y.cpu().numpy()
    G = sp.GridFloat if single else sp.Grid
    cdt = torch.complex64 if single else torch.complex128
    rdt = torch.float32 if single else torch.float64
    tol = 2e-4 if (single or exchange.endswith("FLOAT")) else 1e-10
    desc = (f"case {case}: dims={dims} {'R2C' if r2c else 'C2C'} {'fp32' if single else 'fp64'} P={P} "
            f"{exchange if P > 1 else 'local'} sticks={stick_dist} planes={plane_dist}"
            f"{' centred' if centred else ''}{' multi_transform x3' if multi else ''}")

    def body(rank, comm):
        if not host:
            torch.cuda.set_device(0)
        if P == 1:
            grid = G(nx, ny, nz, nx * ny, PU, nthreads)
        else:
            ms = max(len(np.unique(p[:, 0].astype(np.int64) * ny + p[:, 1])) if len(p) else 0 for p in parts)
            grid = G(nx, ny, nz, max(1, ms), PU, nthreads, max_local_z_length=max(planes),
                     comm=comm, exchange_type=getattr(sp.ExchangeType, exchange))
        t = grid.create_transform(PU, ttype, nx, ny, nz, planes[rank], parts[rank])
        v = dev(vals[starts[rank]:starts[rank + 1]], True)
        out = npy(t.backward(v))
        e = max_rel_error(out, ref[offsets[rank]:offsets[rank + 1]]) if planes[rank] else 0.0
        slab = np.ascontiguousarray(field[offsets[rank]:offsets[rank + 1]])
        f = npy(t.forward(dev(slab, not r2c)))
        ef = max_rel_error(f, vals[starts[rank]:starts[rank + 1]]) if len(f) else 0.0
        return max(e, ef)

    def multi_body():
        # three transforms of the same problem on their own grids, one multi_transform call
        ts = []
        for _ in range(3):
            grid = G(nx, ny, nz, nx * ny, PU, nthreads)
            ts.append((grid, grid.create_transform(PU, ttype, nx, ny, nz, nz, parts[0])))
        v = dev(vals, True)
        outs = sp.multi_transform_backward([t for _, t in ts], [v] * 3)
        e = max(max_rel_error(npy(o), ref) for o in outs)
        sl = dev(np.ascontiguousarray(field), not r2c)
        for _, t in ts:  # forward input: each transform's own space domain
            d = t.space_domain(PU)
            if host:
                d[...] = sl.reshape(d.shape)
            else:
                d.copy_(sl.reshape(d.shape))
        fs = sp.multi_transform_forward([t for _, t in ts])
        return max(e, max(max_rel_error(npy(f), vals) for f in fs))

    if multi:
        errs = [multi_body()]
    else:
        errs = [body(0, None)] if P == 1 else run_ranks(P, body)
    return desc, max(errs), tol


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=100)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max-elems", type=int, default=1 << 20)
    ap.add_argument("--pu", choices=["gpu", "host"], default="gpu",
                    help="host: the same sweep on SPFFT_PU_HOST (runs without a GPU)")
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    bad = 0
    t0 = time.time()
    for c in range(a.cases):
        try:
            desc, err, tol = run_case(rng, c, a.max_elems, host=a.pu == "host")
        except Exception as e:  # a refused or failing case is reported, not fatal
            desc, err, tol = f"case {c}: {type(e).__name__}: {e}", float("inf"), 0.0
        ok = err < tol
        bad += 0 if ok else 1
        print(f"{'ok  ' if ok else 'FAIL'} {desc} err={err:.2e} tol={tol:.0e}", flush=True)
    print(f"{a.cases - bad}/{a.cases} passed in {time.time() - t0:.0f} s", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

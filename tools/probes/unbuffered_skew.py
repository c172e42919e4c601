"""Repro of a fuzz failure: UNBUFFERED on virtual ranks with every stick on one rank
and every plane on another. Prints backward / forward errors per rank and setting."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(dims, stick_dist, plane_dist, exchange, seed=6):
    import torch
    import spfft_amd as sp
    from spfft_amd.parallel import run_ranks
    from spfft_amd.utils.indices import calculate_num_local_xy_planes, create_value_indices
    from spfft_amd.utils.oracle import dense_backward, dense_forward, max_rel_error
    rng = np.random.default_rng(seed)
    nx, ny, nz = dims
    P = len(stick_dist)
    parts = create_value_indices(rng, stick_dist, 0.9, 0.8, nx, ny, nz, False)
    planes = [calculate_num_local_xy_planes(r, nz, plane_dist) for r in range(P)]
    offsets = np.concatenate([[0], np.cumsum(planes)])
    all_idx = np.concatenate(parts)
    field = rng.standard_normal((nz, ny, nx)) + 1j * rng.standard_normal((nz, ny, nx))
    vals = dense_forward(field, all_idx, dims)
    ref = dense_backward(all_idx, vals, dims)
    starts = np.concatenate([[0], np.cumsum([len(p) for p in parts])])
    ms = max(len(np.unique(p[:, 0].astype(np.int64) * ny + p[:, 1])) if len(p) else 0 for p in parts)

    def body(rank, comm):
        torch.cuda.set_device(0)
        grid = sp.Grid(nx, ny, nz, max(1, ms), sp.ProcessingUnit.GPU, 1, max_local_z_length=max(planes),
                       comm=comm, exchange_type=getattr(sp.ExchangeType, exchange))
        t = grid.create_transform(sp.ProcessingUnit.GPU, sp.TransformType.C2C, nx, ny, nz, planes[rank],
                                  parts[rank])
        v = torch.as_tensor(vals[starts[rank]:starts[rank + 1]], device="cuda")
        out = t.backward(v).cpu().numpy()
        eb = max_rel_error(out, ref[offsets[rank]:offsets[rank + 1]]) if planes[rank] else 0.0
        slab = torch.as_tensor(np.ascontiguousarray(field[offsets[rank]:offsets[rank + 1]]), device="cuda")
        f = t.forward(slab).cpu().numpy()
        ef = max_rel_error(f, vals[starts[rank]:starts[rank + 1]]) if len(f) else 0.0
        return (len(parts[rank]), planes[rank], eb, ef)

    res = run_ranks(P, body)
    print(f"{exchange:24s} dims={dims} sticks={stick_dist} planes={plane_dist}: " +
          " | ".join(f"r{r}: vals={n} planes={p} bwd={eb:.1e} fwd={ef:.1e}" for r, (n, p, eb, ef) in enumerate(res)),
          flush=True)


if __name__ == "__main__":
    for ex in ("COMPACT_BUFFERED", "UNBUFFERED"):
        run((2, 64, 5), [1.0, 0.0, 0.0], [0.0, 1.0, 0.0], ex)
        run((2, 64, 5), [1.0, 0.0], [0.0, 1.0], ex)
        run((8, 8, 8), [1.0, 0.0], [0.0, 1.0], ex)
        run((8, 8, 8), [1.0, 1.0], [0.0, 1.0], ex)
        run((8, 8, 8), [1.0, 0.0], [1.0, 1.0], ex)
        run((8, 8, 8), [1.0, 1.0, 1.0], [1.0, 0.0, 1.0], ex)

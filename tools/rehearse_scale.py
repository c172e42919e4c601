"""Rehearsal of the driver's multi-GPU headline on ONE GPU: P virtual ranks (an
in-process group, one thread per rank) run the bench.py problem (256^3 C2C fp64,
r = N/2, sticks and planes split evenly) with T transforms per rank through
multi_transform, with the data plane of the real P-GPU run:

  --plane rccl      every exchange block moves through RCCL (RCCL self-loopback
                    per virtual rank: grouped ncclSend/ncclRecv with the real
                    counts and displacements, the shared channel, chunking)
  --plane loopback  device-to-device copies (same layouts)

It prints each rank's plan line (SPFFT_LOG: chunks, data plane, RCCL channel)
and checks the backward transform of rank 0's slab and every rank's round trip.
Timings are not meaningful (all ranks share one GPU).

    python tools/rehearse_scale.py [--ranks 8] [--size 256] [--transforms 4] [--plane rccl]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--transforms", type=int, default=4)
    ap.add_argument("--plane", default="rccl", choices=["rccl", "loopback"])
    ap.add_argument("--exchange", default="COMPACT_BUFFERED")
    a = ap.parse_args()
    if a.plane == "rccl":
        os.environ["SPFFT_GPU_EXCHANGE"] = "rccl"
    os.environ.setdefault("SPFFT_LOG", "1")
    import torch

    import spfft_amd as sp
    from spfft_amd.parallel import make_distributed, run_ranks
    from spfft_amd.utils.indices import distribute_sticks, sphere_indices
    from spfft_amd.utils.oracle import max_rel_error

    n, P, T = a.size, a.ranks, a.transforms
    dims = (n, n, n)
    gidx = sphere_indices(*dims, 0.5)
    parts = distribute_sticks(gidx, P, dims)
    starts = np.concatenate([[0], np.cumsum([len(p) for p in parts])])
    exch = getattr(sp.ExchangeType, a.exchange)
    before = sp.rccl_communicators()

    def body(rank, comm):
        torch.cuda.set_device(0)
        setups = [make_distributed(comm, dims, gidx, processing_unit=sp.ProcessingUnit.GPU,
                                   exchange_type=exch) for _ in range(T)]
        ts = [s.transform for s in setups]
        g = torch.Generator(device="cuda")
        g.manual_seed(100 + rank)
        ins = [torch.randn(int(starts[rank + 1] - starts[rank]), dtype=torch.complex128,
                           device="cuda", generator=g) for _ in range(T)]
        t0 = time.perf_counter()
        for _ in range(3):
            sp.multi_transform_backward(ts, ins)
            outs = sp.multi_transform_forward(ts, scalings=[sp.Scaling.FULL] * T)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        err = max(max_rel_error(o.cpu().numpy(), i.cpu().numpy()) for o, i in zip(outs, ins))
        return err, dt, setups[0].grid.data_plane

    res = run_ranks(P, body)
    err = max(r[0] for r in res)
    planes = sorted({r[2] for r in res})
    print(f"ranks={P} size={n}^3 transforms={T} exchange={a.exchange} plane={planes} "
          f"rccl_communicators_created={sp.rccl_communicators() - before} "
          f"max_roundtrip_err={err:.2e} {'OK' if err < 1e-11 else 'FAIL'}", flush=True)
    sys.exit(0 if err < 1e-11 else 1)


if __name__ == "__main__":
    main()

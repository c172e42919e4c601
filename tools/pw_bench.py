"""Plane-wave workload throughput on one GPU: H_loc psi for many bands
(PlaneWaveModel.apply_local_potential: backward, V(r) multiply, forward per band,
num_transforms bands per multi_transform call). Prints one JSON line.

    python tools/pw_bench.py --ecut 20 --alat 10 --bands 64 --transforms 8
(SPFFT_BATCH=0 in the environment disables batched launches for comparison.)
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ecut", type=float, default=20.0)
    ap.add_argument("--alat", type=float, default=10.0)
    ap.add_argument("--bands", type=int, default=64)
    ap.add_argument("--transforms", type=int, default=8)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import torch

    import spfft_amd as sp
    from spfft_amd.models import PlaneWaveBasis, PlaneWaveModel
    basis = PlaneWaveBasis(alat=a.alat, ecut=a.ecut)
    model = PlaneWaveModel(basis, processing_unit=sp.ProcessingUnit.GPU, num_transforms=a.transforms)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    psi = [torch.randn(basis.num_pw, dtype=torch.complex128, device=dev, generator=g)
           for _ in range(a.bands)]
    nx, ny, nz = basis.fft_dims
    v_r = torch.rand((nz, ny, nx), dtype=torch.float64, device=dev, generator=g)
    model.apply_local_potential(psi, v_r)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        model.apply_local_potential(psi, v_r)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"workload": "plane-wave H_loc psi", "fft_dims": list(basis.fft_dims),
                      "num_pw": basis.num_pw, "bands": a.bands, "transforms": a.transforms,
                      "batch": os.environ.get("SPFFT_BATCH", "1"),
                      "bands_per_s": a.bands * a.reps / dt,
                      "transforms_per_s": 2 * a.bands * a.reps / dt}), flush=True)


if __name__ == "__main__":
    main()

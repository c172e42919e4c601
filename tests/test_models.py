"""Workload configurations and the plane-wave application model (host and GPU)."""
import numpy as np
import pytest

import spfft_amd as sp
from spfft_amd.models import WORKLOADS, PlaneWaveBasis, PlaneWaveModel, slab_sparsity_indices
from spfft_amd.utils.oracle import dense_backward, dense_forward, max_rel_error


def test_workload_index_sets():
    assert len(WORKLOADS["128c2c"].indices()) == 1097914  # same set bench.py reports
    r2c = WORKLOADS["256r2c"]
    idx = r2c.indices()
    assert idx[:, 0].min() >= 0 and idx[:, 0].max() <= 128
    # reference benchmark data set: x < dimXFreq * sparsity, full sticks
    s = slab_sparsity_indices(8, 6, 4, 0.5, False)
    assert len(s) == 4 * 6 * 4 and s[:, 0].max() == 3
    s = slab_sparsity_indices(8, 6, 4, 1.0, True)
    assert len(s) == (4 + 4 * 6) * 4  # x in [0, 4]; x = 0 keeps y < dimY/2 + 1


def test_readme_workload_host():
    cfg = WORKLOADS["readme2x2x2"]
    setup = cfg.build(processing_unit=sp.ProcessingUnit.HOST)
    rng = np.random.default_rng(0)
    v = rng.standard_normal(len(setup.indices)) + 1j * rng.standard_normal(len(setup.indices))
    out = np.array(setup.transform.backward(v))
    assert max_rel_error(out, dense_backward(setup.indices, v, cfg.dims)) < 1e-13


def _pw_check(pu, device=None):
    basis = PlaneWaveBasis(alat=10.0, ecut=3.0)
    assert basis.num_pw > 50
    dims = basis.fft_dims
    model = PlaneWaveModel(basis, processing_unit=pu, num_transforms=2)
    rng = np.random.default_rng(4)
    nb = 3
    psi = [rng.standard_normal(basis.num_pw) + 1j * rng.standard_normal(basis.num_pw)
           for _ in range(nb)]
    nx, ny, nz = dims
    z, y, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    v_r = 0.3 + 0.2 * np.cos(2 * np.pi * x / nx) * np.sin(2 * np.pi * 2 * z / nz)
    if device is not None:
        import torch
        psi_in = [torch.as_tensor(c, device=device) for c in psi]
        v_in = torch.as_tensor(v_r, device=device)
    else:
        psi_in, v_in = psi, v_r
    hpsi = model.apply_local_potential(psi_in, v_in)
    for c, h in zip(psi, hpsi):
        h = h.cpu().numpy() if hasattr(h, "cpu") else np.asarray(h)
        dense = dense_backward(basis.indices, c, dims) * v_r
        ref = dense_forward(dense, basis.indices, dims) / (nx * ny * nz)
        assert max_rel_error(h, ref) < 1e-12
    rho = model.density(psi_in, [2.0] * nb)
    rho = rho.cpu().numpy() if hasattr(rho, "cpu") else np.asarray(rho)
    # Parseval for the unnormalised backward transform
    expect = 2.0 * nx * ny * nz * sum(np.sum(np.abs(c) ** 2) for c in psi)
    assert abs(rho.sum() - expect) / expect < 1e-12
    t = model.kinetic(psi_in)[0]
    t = t.cpu().numpy() if hasattr(t, "cpu") else t
    assert np.allclose(t, 0.5 * basis.g2 * psi[0])


def test_planewave_model_host():
    _pw_check(sp.ProcessingUnit.HOST)


@pytest.mark.gpu
def test_planewave_model_gpu(gpu):
    _pw_check(sp.ProcessingUnit.GPU, device=gpu)

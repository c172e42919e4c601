"""Plane-wave application model: the workload SpFFT exists for.

Electronic-structure codes expand wavefunctions in plane waves
psi(r) = sum_G c_G exp(i G.r) with |G|^2 / 2 <= E_cut: a spherical set of
frequency indices (the sparse input of the transforms). The two hot operations
per band are:

  * local potential application, H_loc psi = FFT^-1 [ V(r) * FFT[psi](r) ]:
    backward transform, pointwise multiply in real space, forward transform;
  * density accumulation, rho(r) = sum_b w_b |psi_b(r)|^2: backward transforms.

Both run fully on the GPU with the space domain kept resident in the Grid's HBM
slab, several bands at once through multi_transform.

Units: a cubic cell of side `alat` (bohr), E_cut in hartree; G = 2 pi / alat * k.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence

import numpy as np

from ..types import ProcessingUnit, Scaling, TransformType


def _good_fft_size(n: int) -> int:
    """Smallest m >= n of the form 2^a 3^b 5^c (fast lengths for the FFT engines)."""
    m = max(1, n)
    while True:
        r = m
        for p in (2, 3, 5):
            while r % p == 0:
                r //= p
        if r == 1:
            return m
        m += 1


@dataclass
class PlaneWaveBasis:
    """Plane waves with |G|^2/2 <= ecut in a cubic cell; FFT grid holds |G| <= 2 Gmax
    (density / potential products) unless `fft_dims` is given."""
    alat: float
    ecut: float
    fft_dims: tuple = None

    def __post_init__(self):
        gmax = np.sqrt(2.0 * self.ecut)
        kmax = int(np.floor(gmax * self.alat / (2 * np.pi)))
        if self.fft_dims is None:
            n = _good_fft_size(4 * kmax + 1)
            self.fft_dims = (n, n, n)
        n0, n1, n2 = self.fft_dims
        if min(self.fft_dims) < 2 * kmax + 1:
            raise ValueError("FFT grid too small for the cutoff")
        ks = np.arange(-kmax, kmax + 1)
        kx, ky, kz = np.meshgrid(ks, ks, ks, indexing="ij")
        g2 = (2 * np.pi / self.alat) ** 2 * (kx ** 2 + ky ** 2 + kz ** 2)
        m = 0.5 * g2 <= self.ecut + 1e-12
        trip = np.stack([kx[m], ky[m], kz[m]], axis=1).astype(np.int32)
        # stick-major order (x, y storage key, then z): the layout the plan prefers
        key = (np.where(trip[:, 0] < 0, trip[:, 0] + n0, trip[:, 0]).astype(np.int64) * n1
               + np.where(trip[:, 1] < 0, trip[:, 1] + n1, trip[:, 1])) * n2 \
            + np.where(trip[:, 2] < 0, trip[:, 2] + n2, trip[:, 2])
        self.indices = trip[np.argsort(key, kind="stable")]
        self.g2 = (2 * np.pi / self.alat) ** 2 * (self.indices.astype(np.float64) ** 2).sum(axis=1)

    @property
    def num_pw(self) -> int:
        return len(self.indices)


class PlaneWaveModel:
    """Band-parallel local-potential and density operations on one device.

    `num_transforms` transforms (one Grid each, identical plans: a transform and
    its clones) process that many bands per multi_transform call. On the GPU
    the library runs such a group batched, one launch per stage for up to 8
    bands (multi_transform.cpp), so small grids are not launch bound."""

    def __init__(self, basis: PlaneWaveBasis, processing_unit=ProcessingUnit.GPU,
                 num_transforms: int = 8, single: bool = False):
        from ..grid import Grid, GridFloat
        self.basis = basis
        self.pu = processing_unit
        n0, n1, n2 = basis.fft_dims
        cls = GridFloat if single else Grid
        g = cls(n0, n1, n2, n0 * n1, processing_unit, -1)
        t0 = g.create_transform(processing_unit, TransformType.C2C, n0, n1, n2, n2, basis.indices)
        self.transforms = [t0] + [t0.clone() for _ in range(max(1, num_transforms) - 1)]
        self.volume_points = n0 * n1 * n2

    def apply_local_potential(self, psi: Sequence, v_r) -> List:
        """H_loc psi_b for every band b: FFT^-1[V(r) FFT[psi_b](r)] (band coefficients in,
        band coefficients out). `v_r` is the real-space potential [z][y][x]."""
        from ..grid import multi_transform_backward, multi_transform_forward
        out = []
        T = len(self.transforms)
        for start in range(0, len(psi), T):
            group = list(psi[start:start + T])
            ts = self.transforms[:len(group)]
            spaces = multi_transform_backward(ts, group)
            for s in spaces:
                if hasattr(s, "mul_"):
                    s.mul_(v_r)
                else:
                    np.multiply(s, v_r, out=s)
            res = multi_transform_forward(ts, scalings=[Scaling.FULL] * len(ts))
            out.extend(r.clone() if hasattr(r, "clone") else np.array(r) for r in res)
        return out

    def density(self, psi: Sequence, weights: Sequence[float]):
        """rho(r) = sum_b w_b |psi_b(r)|^2 on the real-space grid [z][y][x]."""
        from ..grid import multi_transform_backward
        rho = None
        T = len(self.transforms)
        psi, weights = list(psi), list(weights)
        for start in range(0, len(psi), T):
            group = psi[start:start + T]
            spaces = multi_transform_backward(self.transforms[:len(group)], group)
            for s, w in zip(spaces, weights[start:start + T]):
                contrib = (s.real ** 2 + s.imag ** 2) * w
                rho = contrib if rho is None else rho + contrib
        return rho

    def kinetic(self, psi: Sequence) -> List:
        """T psi_b = |G|^2/2 c_G (diagonal in the plane-wave basis)."""
        g2 = self.basis.g2
        out = []
        for c in psi:
            if type(c).__module__.startswith("torch"):
                import torch
                out.append(c * torch.as_tensor(0.5 * g2, device=c.device, dtype=c.real.dtype))
            else:
                out.append(np.asarray(c) * (0.5 * g2))
        return out

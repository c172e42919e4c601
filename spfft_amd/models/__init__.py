"""Workloads built on the transforms.

* configs: the benchmark configurations of BASELINE.json (index sets, rank
  distribution, ready Grid/Transform).
* planewave: the plane-wave electronic-structure model SpFFT serves (spherical
  cutoff basis, local-potential application, density accumulation).
"""
from .configs import WORKLOADS, Workload, slab_sparsity_indices  # noqa: F401
from .planewave import PlaneWaveBasis, PlaneWaveModel  # noqa: F401

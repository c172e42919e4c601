"""Named workloads: the benchmark configurations of BASELINE.json.

Each workload builds its frequency index set (spherical cutoff or the
reference benchmark's slab sparsity), the per-rank distribution and a
ready-to-run Grid/Transform. bench.py and spfft_bench (C++) measure the same
data sets.

    cfg = WORKLOADS["256c2c"]
    setup = cfg.build(processing_unit=ProcessingUnit.GPU)      # single rank
    setup = cfg.build(comm=TorchDistComm(), ...)               # distributed
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Optional

import numpy as np

from ..types import ExchangeType, ProcessingUnit, TransformType
from ..utils.indices import sphere_indices


def slab_sparsity_indices(nx: int, ny: int, nz: int, sparsity: float, r2c: bool) -> np.ndarray:
    """Reference benchmark data set (tests/programs/benchmark.cpp:172-205): full z-sticks for
    x < dimXFreq * sparsity, (x == 0 ? dimYFreq : dimY) y values, in stick-key order."""
    xf = nx // 2 + 1 if r2c else nx
    yf = ny // 2 + 1 if r2c else ny
    out = []
    for x in range(int(np.ceil(xf * sparsity))):
        if x >= xf * sparsity:
            break
        for y in range(yf if x == 0 else ny):
            trip = np.empty((nz, 3), dtype=np.int32)
            trip[:, 0] = x
            trip[:, 1] = y
            trip[:, 2] = np.arange(nz)
            out.append(trip)
    return np.concatenate(out) if out else np.zeros((0, 3), dtype=np.int32)


@dataclass
class Workload:
    name: str
    dims: tuple
    transform_type: TransformType = TransformType.C2C
    cutoff: Optional[float] = 0.5       # spherical cutoff |k/N| <= cutoff; None: slab sparsity
    sparsity: float = 1.0
    single: bool = False
    exchange: ExchangeType = ExchangeType.COMPACT_BUFFERED
    gpus: tuple = (1,)
    note: str = ""
    extra: dict = field(default_factory=dict)

    @property
    def r2c(self) -> bool:
        return self.transform_type == TransformType.R2C

    def indices(self) -> np.ndarray:
        nx, ny, nz = self.dims
        if self.cutoff is not None:
            return sphere_indices(nx, ny, nz, self.cutoff, r2c=self.r2c)
        return slab_sparsity_indices(nx, ny, nz, self.sparsity, self.r2c)

    def build(self, processing_unit=ProcessingUnit.GPU, comm=None, indices=None):
        """Grid + transform for this workload (collective when `comm` spans several ranks)."""
        from ..grid import Grid, GridFloat
        from ..parallel.distributed import DistributedSetup, make_distributed
        idx = self.indices() if indices is None else indices
        nx, ny, nz = self.dims
        if comm is not None and comm.size > 1:
            return make_distributed(comm, self.dims, idx, processing_unit=processing_unit,
                                    transform_type=self.transform_type,
                                    exchange_type=self.exchange, single=self.single)
        cls = GridFloat if self.single else Grid
        grid = cls(nx, ny, nz, nx * ny, processing_unit, -1)
        t = grid.create_transform(processing_unit, self.transform_type, nx, ny, nz, nz, idx)
        return DistributedSetup(grid, t, idx, 0, nz)


WORKLOADS: Dict[str, Workload] = {
    "readme2x2x2": Workload("readme2x2x2", (2, 2, 2), cutoff=None, gpus=(0,),
                            note="README example: 2x2x2 C2C on SPFFT_PU_HOST"),
    "128c2c": Workload("128c2c", (128, 128, 128), note="128^3 C2C spherical cutoff fp64, 1 GPU"),
    "256r2c": Workload("256r2c", (256, 256, 256), TransformType.R2C,
                       note="256^3 R2C hermitian symmetry fp64, 1 GPU"),
    "256c2c": Workload("256c2c", (256, 256, 256), gpus=(1, 2, 4, 8),
                       note="headline: 256^3 C2C fp64, pencil<->slab over RCCL/xGMI"),
    "512r2c_f32": Workload("512r2c_f32", (512, 512, 512), TransformType.R2C, single=True,
                           gpus=(8,), note="512^3 R2C fp32, 8 GPUs, GPU-direct all-to-all"),
}

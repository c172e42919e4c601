"""Helpers to set up distributed transforms (stick / plane distribution)."""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ..types import ExchangeType, ProcessingUnit, TransformType
from ..utils.indices import distribute_sticks, split_even


def even_planes(nz: int, size: int, rank: int):
    """(offset, length) of an even z-slab split (first nz % size ranks one larger)."""
    counts = split_even(nz, size)
    return int(sum(counts[:rank])), int(counts[rank])


@dataclass
class DistributedSetup:
    grid: object
    transform: object
    indices: np.ndarray
    z_offset: int
    z_length: int


def make_distributed(comm, dims, all_indices: np.ndarray, processing_unit=ProcessingUnit.HOST,
                     transform_type=TransformType.C2C, exchange_type=ExchangeType.DEFAULT,
                     single: bool = False, num_threads: int = -1) -> DistributedSetup:
    """Distributes a stick-major global index list evenly and plans the transform on `comm`."""
    from ..grid import Grid, GridFloat

    rank, size = comm.rank, comm.size
    nx, ny, nz = dims
    local = distribute_sticks(all_indices, size, dims)[rank]
    zoff, zlen = even_planes(nz, size, rank)
    key = (np.where(local[:, 0] < 0, local[:, 0] + nx, local[:, 0]).astype(np.int64) * ny
           + np.where(local[:, 1] < 0, local[:, 1] + ny, local[:, 1]))
    nsticks = int(len(np.unique(key)))
    cls = GridFloat if single else Grid
    grid = cls(nx, ny, nz, max(1, nsticks), processing_unit, num_threads, max_local_z_length=zlen,
               comm=comm, exchange_type=exchange_type)
    t = grid.create_transform(processing_unit, transform_type, nx, ny, nz, zlen, local)
    return DistributedSetup(grid, t, local, zoff, zlen)

"""Frequency-index generators.

* Spherical cutoff (the benchmark data set of BASELINE.md): all centred
  frequencies with (kx/Nx)^2 + (ky/Ny)^2 + (kz/Nz)^2 <= cutoff^2.
* Generators with the semantics of the reference's test utilities
  (reference: tests/test_util/generate_indices.hpp:39-136): random stick
  subsets distributed over ranks, centring, plane distributions.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np


def _centered_range(n: int) -> np.ndarray:
    """Centred frequencies in storage order: 0..n/2, then n/2-n+1..-1."""
    pos = np.arange(0, n // 2 + 1)
    neg = np.arange(n // 2 - n + 1, 0)
    return np.concatenate([pos, neg])


def sphere_sticks(nx: int, ny: int, nz: int, cutoff: float = 0.5, r2c: bool = False):
    """(x, y) centred stick coordinates inside the cutoff sphere, ordered by storage key."""
    xs = np.arange(0, nx // 2 + 1) if r2c else _centered_range(nx)
    ys = _centered_range(ny)
    gx, gy = np.meshgrid(xs, ys, indexing="ij")
    rr = (gx / nx) ** 2 + (gy / ny) ** 2
    m = rr <= cutoff ** 2 + 1e-12
    sx, sy = gx[m], gy[m]
    key = np.where(sx < 0, sx + nx, sx) * ny + np.where(sy < 0, sy + ny, sy)
    order = np.argsort(key, kind="stable")
    return sx[order].astype(np.int32), sy[order].astype(np.int32)


def sphere_indices(nx: int, ny: int, nz: int, cutoff: float = 0.5, r2c: bool = False,
                   sticks=None) -> np.ndarray:
    """(n, 3) int32 centred triplets of the spherical cutoff, stick-major, z in storage order."""
    if sticks is None:
        sticks = sphere_sticks(nx, ny, nz, cutoff, r2c)
    sx, sy = sticks
    zs = _centered_range(nz).astype(np.float64)
    rr = (sx / nx) ** 2 + (sy / ny) ** 2
    zlim2 = cutoff ** 2 + 1e-12 - rr  # per stick
    mask = (zs[None, :] / nz) ** 2 <= zlim2[:, None]
    counts = mask.sum(axis=1)
    out = np.empty((int(counts.sum()), 3), dtype=np.int32)
    out[:, 0] = np.repeat(sx, counts)
    out[:, 1] = np.repeat(sy, counts)
    out[:, 2] = np.broadcast_to(zs[None, :], mask.shape)[mask].astype(np.int32)
    return out


def split_even(n: int, parts: int) -> List[int]:
    """n items split as evenly as possible, the first n % parts parts one larger."""
    return [n // parts + (1 if r < n % parts else 0) for r in range(parts)]


def distribute_sticks(indices: np.ndarray, ranks: int, dims) -> List[np.ndarray]:
    """Splits a stick-major triplet list into `ranks` contiguous groups of whole sticks."""
    nx, ny, _ = dims
    x = np.where(indices[:, 0] < 0, indices[:, 0] + nx, indices[:, 0])
    y = np.where(indices[:, 1] < 0, indices[:, 1] + ny, indices[:, 1])
    key = x.astype(np.int64) * ny + y
    # stick boundaries in list order
    change = np.flatnonzero(np.diff(key)) + 1
    starts = np.concatenate([[0], change])
    ends = np.concatenate([change, [len(key)]])
    counts = split_even(len(starts), ranks)
    out, s = [], 0
    for c in counts:
        if c == 0:
            out.append(indices[:0])
        else:
            out.append(indices[starts[s]:ends[s + c - 1]])
        s += c
    return out


def center_indices(dims, indices_per_rank: Sequence[np.ndarray]) -> List[np.ndarray]:
    """Maps storage indices >= n/2+1 to the negative range (reference center_indices)."""
    out = []
    for idx in indices_per_rank:
        idx = np.array(idx, dtype=np.int32, copy=True).reshape(-1, 3)
        for d in range(3):
            n = dims[d]
            sel = idx[:, d] >= n // 2 + 1
            idx[sel, d] -= n
        out.append(idx)
    return out


def create_value_indices(rng: np.random.Generator, stick_distribution: Sequence[float],
                         total_stick_fraction: float, stick_fill_fraction: float, nx: int,
                         ny: int, nz: int, hermitian: bool) -> List[np.ndarray]:
    """Random sparse index sets per rank (semantics of the reference test generator).

    Sticks (x, y) are kept with probability `total_stick_fraction` and assigned to
    a rank drawn from `stick_distribution`; each z of a stick is kept with
    probability `stick_fill_fraction`. With `hermitian`, only x <= nx/2 is used,
    the x = 0 plane keeps y <= ny/2 and the (0, 0) stick keeps z <= nz/2.
    """
    p = np.asarray(stick_distribution, dtype=np.float64)
    p = p / p.sum()
    nxf = nx // 2 + 1 if hermitian else nx
    nyf = ny // 2 + 1 if hermitian else ny
    nzf = nz // 2 + 1 if hermitian else nz
    per_rank_sticks: List[list] = [[] for _ in p]
    for x in range(nxf):
        for y in range(ny):
            if hermitian and x == 0 and y >= nyf:
                continue
            if rng.random() < total_stick_fraction:
                r = int(rng.choice(len(p), p=p))
                per_rank_sticks[r].append((x, y))
    out = []
    for sticks in per_rank_sticks:
        trip = []
        for (x, y) in sticks:
            for z in range(nz):
                if hermitian and x == 0 and y == 0 and z >= nzf:
                    continue
                if rng.random() < stick_fill_fraction:
                    trip.append((x, y, z))
        out.append(np.array(trip, dtype=np.int32).reshape(-1, 3))
    return out


def calculate_num_local_xy_planes(rank: int, nz: int, plane_distribution: Sequence[float]) -> int:
    """Planes of `rank` for a weighted plane distribution (reference semantics)."""
    w = np.asarray(plane_distribution, dtype=np.float64)
    planes = [int(v / w.sum() * nz) for v in w]
    missing = nz - sum(planes)
    for i, v in enumerate(planes):
        if v > 0 and missing > 0:
            planes[i] += missing
            missing = 0
            break
        if missing < 0:
            take = min(v, -missing)
            planes[i] -= take
            missing += take
            if missing >= 0:
                missing = 0
                break
    if missing > 0:
        planes[0] = missing
    return planes[rank]

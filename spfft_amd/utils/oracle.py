"""Dense numpy oracles for the sparse transforms (test and validation only).

Conventions (SpFFT docs/source/details.rst:6-45): backward uses exp(+2 pi i),
forward exp(-2 pi i), neither normalised; space layout [z][y][x].
"""
from __future__ import annotations

import numpy as np


def storage(idx: np.ndarray, dims) -> np.ndarray:
    idx = np.asarray(idx).reshape(-1, 3).astype(np.int64)
    out = idx.copy()
    for d in range(3):
        out[:, d] = np.where(idx[:, d] < 0, idx[:, d] + dims[d], idx[:, d])
    return out


def _hermitian_fill(line: np.ndarray) -> None:
    """In-place fill where the source is non-zero, two half passes (reference semantics)."""
    n = line.shape[0]
    for k in list(range(1, n // 2 + 1)) + list(range(n // 2 + 1, n)):
        v = line[k]
        nz = v != 0
        if np.ndim(v) == 0:
            if nz:
                line[n - k] = np.conj(v)
        else:
            line[n - k][nz] = np.conj(v[nz])


def dense_backward(indices, values, dims, r2c: bool = False) -> np.ndarray:
    """Space domain [z][y][x] of the sparse spectrum (complex; real for r2c)."""
    nx, ny, nz = dims
    s = storage(indices, dims)
    vals = np.asarray(values).reshape(-1)
    if not r2c:
        F = np.zeros((nx, ny, nz), dtype=np.complex128)
        F[s[:, 0], s[:, 1], s[:, 2]] = vals
        sp = np.fft.ifftn(F) * (nx * ny * nz)
        return np.ascontiguousarray(sp.transpose(2, 1, 0))
    H = np.zeros((nx // 2 + 1, ny, nz), dtype=np.complex128)
    H[s[:, 0], s[:, 1], s[:, 2]] = vals
    # (0,0) stick along z, then the x = 0 plane along y per z (after the z transform)
    _hermitian_fill(H[0, 0, :])
    G = np.fft.ifft(H, axis=2) * nz
    for z in range(nz):
        _hermitian_fill(G[0, :, z])
    G = np.fft.ifft(G, axis=1) * ny
    sp = np.fft.irfft(G, n=nx, axis=0) * nx
    return np.ascontiguousarray(sp.transpose(2, 1, 0))


def dense_forward(space, indices, dims, r2c: bool = False, scale: bool = False) -> np.ndarray:
    """Frequency values at `indices` of the forward transform of space [z][y][x]."""
    nx, ny, nz = dims
    sp = np.asarray(space).reshape(nz, ny, nx).transpose(2, 1, 0)
    F = np.fft.fftn(sp)
    if scale:
        F = F / (nx * ny * nz)
    s = storage(indices, dims)
    return F[s[:, 0], s[:, 1], s[:, 2]]


def max_rel_error(a, b) -> float:
    a = np.asarray(a)
    b = np.asarray(b)
    denom = max(np.max(np.abs(b)) if b.size else 0.0, 1e-300)
    return float(np.max(np.abs(a - b)) / denom) if a.size else 0.0

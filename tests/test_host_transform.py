"""Host (CPU) engine numerics against numpy — the SpFFT local test sweep
(reference: tests/local_tests/test_local_transform.cpp, sizes {1,2,11,12,13,100})."""
import itertools

import numpy as np
import pytest

import spfft_amd as sp
from spfft_amd.utils.indices import center_indices, create_value_indices
from spfft_amd.utils.oracle import dense_backward, dense_forward, max_rel_error

HOST = sp.ProcessingUnit.HOST
SIZES = [1, 2, 11, 12, 13, 100]
# a deterministic cover of the 216 combinations: every size in every axis, both sides
COMBOS = sorted(set([(a, b, c) for a, b, c in itertools.product(SIZES, SIZES, SIZES)
                     if (a * 7 + b * 3 + c) % 9 == 0 or len({a, b, c}) == 1]))


@pytest.mark.parametrize("dims", COMBOS)
@pytest.mark.parametrize("centered", [False, True])
def test_c2c(dims, centered):
    nx, ny, nz = dims
    if nx * ny * nz > 200_000:
        pytest.skip("large dense oracle")
    rng = np.random.default_rng(42)
    idx = create_value_indices(rng, [1.0], 0.7, 0.7, nx, ny, nz, False)[0]
    if centered:
        idx = center_indices(dims, [idx])[0]
    vals = rng.standard_normal(len(idx)) + 1j * rng.standard_normal(len(idx))
    grid = sp.Grid(nx, ny, nz, nx * ny, HOST, 2)
    t = grid.create_transform(HOST, sp.TransformType.C2C, nx, ny, nz, nz, idx)
    ref = dense_backward(idx, vals, dims)
    for _ in range(2):
        out = t.backward(vals)
        assert max_rel_error(out, ref) < 1e-12
    space = rng.standard_normal((nz, ny, nx)) + 1j * rng.standard_normal((nz, ny, nx))
    f = t.forward(space)
    assert max_rel_error(f, dense_forward(space, idx, dims)) < 1e-12
    fs = t.forward(space, scaling=sp.Scaling.FULL)
    assert max_rel_error(fs, dense_forward(space, idx, dims, scale=True)) < 1e-12


@pytest.mark.parametrize("dims", [(1, 1, 1), (2, 2, 2), (11, 12, 13), (12, 11, 13), (13, 13, 2),
                                  (100, 11, 2), (2, 100, 12), (12, 12, 100)])
@pytest.mark.parametrize("centered", [False, True])
def test_r2c(dims, centered):
    nx, ny, nz = dims
    rng = np.random.default_rng(42)
    space = rng.standard_normal((nz, ny, nx))
    idx = create_value_indices(rng, [1.0], 1.0, 1.0, nx, ny, nz, True)[0]
    if centered:
        # x stays non-negative for R2C (reference indices.hpp:137-141)
        c = center_indices(dims, [idx])[0]
        c[:, 0] = idx[:, 0]
        idx = c
    grid = sp.Grid(nx, ny, nz, nx * ny, HOST, 2)
    t = grid.create_transform(HOST, sp.TransformType.R2C, nx, ny, nz, nz, idx)
    f = t.forward(space)
    assert max_rel_error(f, dense_forward(space, idx, dims)) < 1e-12
    out = t.backward(f)
    assert max_rel_error(out, space * nx * ny * nz) < 1e-12


def test_readme_example_2x2x2():
    """Config 1 of BASELINE.json: 2x2x2 C2C on SPFFT_PU_HOST (reference README example)."""
    dims = (2, 2, 2)
    idx = np.array([(x, y, z) for x in range(2) for y in range(2) for z in range(2)], np.int32)
    vals = np.array([complex(i, -i) for i in range(8)])
    grid = sp.Grid(2, 2, 2, 4, HOST, -1)
    t = grid.create_transform(HOST, sp.TransformType.C2C, 2, 2, 2, 2, idx)
    out = t.backward(vals)
    assert max_rel_error(out, dense_backward(idx, vals, dims)) < 1e-14
    back = t.forward(None, scaling=sp.Scaling.FULL)
    assert max_rel_error(back, vals) < 1e-14


def test_single_precision_host():
    rng = np.random.default_rng(1)
    dims = (12, 11, 13)
    nx, ny, nz = dims
    idx = create_value_indices(rng, [1.0], 0.7, 0.7, nx, ny, nz, False)[0]
    vals = (rng.standard_normal(len(idx)) + 1j * rng.standard_normal(len(idx))).astype(np.complex64)
    grid = sp.GridFloat(nx, ny, nz, nx * ny, HOST, 2)
    t = grid.create_transform(HOST, sp.TransformType.C2C, nx, ny, nz, nz, idx)
    out = t.backward(vals)
    assert out.dtype == np.complex64
    assert max_rel_error(out, dense_backward(idx, vals, dims)) < 1e-5


@pytest.mark.parametrize("dims", [(67, 3, 2), (101, 103, 4), (127, 2, 131), (2, 257, 3), (199, 1, 1),
                                  (202, 3, 2), (3, 134, 5), (4, 3, 206)])
@pytest.mark.parametrize("r2c", [False, True])
def test_large_prime_bluestein(dims, r2c):
    """Lengths with a prime factor > 61 (host, batched): primes whose n - 1 has a
    direct plan run Rader's algorithm (67, 101, 103, 127, 131, 199, 257), other
    lengths (2 * 101, 2 * 67, 2 * 103) Bluestein's chirp-z convolution."""
    nx, ny, nz = dims
    rng = np.random.default_rng(3)
    idx = create_value_indices(rng, [1.0], 0.8, 0.9, nx, ny, nz, r2c)[0]
    space = rng.standard_normal((nz, ny, nx))
    if not r2c:
        space = space + 1j * rng.standard_normal((nz, ny, nx))
    vals = dense_forward(space, idx, dims, r2c=r2c)
    g = sp.Grid(nx, ny, nz, nx * ny, sp.ProcessingUnit.HOST, 2)
    t = g.create_transform(sp.ProcessingUnit.HOST, sp.TransformType.R2C if r2c else sp.TransformType.C2C,
                           nx, ny, nz, nz, idx)
    out = np.array(t.backward(vals))
    assert max_rel_error(out, dense_backward(idx, vals, dims, r2c=r2c)) < 1e-12
    f = np.array(t.forward(space))
    assert max_rel_error(f, vals) < 1e-12


def test_reference_size_sweep_full():
    """All 216 combinations of the reference sweep on the host engine in one loop
    (C2C alternating centred indices, run twice, scaled forward)."""
    rng = np.random.default_rng(216)
    failures = []
    for n, dims in enumerate(itertools.product(SIZES, SIZES, SIZES)):
        nx, ny, nz = dims
        idx = create_value_indices(rng, [1.0], 0.7, 0.7, nx, ny, nz, False)[0]
        centered = n % 2 == 1
        if centered:
            idx = center_indices(dims, [idx])[0]
        vals = rng.standard_normal(len(idx)) + 1j * rng.standard_normal(len(idx))
        grid = sp.Grid(nx, ny, nz, nx * ny, HOST, 4)
        t = grid.create_transform(HOST, sp.TransformType.C2C, nx, ny, nz, nz, idx)
        ref = dense_backward(idx, vals, dims)
        errs = [max_rel_error(t.backward(vals), ref) for _ in range(2)]
        space = rng.standard_normal((nz, ny, nx)) + 1j * rng.standard_normal((nz, ny, nx))
        errs.append(max_rel_error(t.forward(space, scaling=sp.Scaling.FULL),
                                  dense_forward(space, idx, dims, scale=True)))
        if max(errs) > 1e-11:
            failures.append((dims, centered, errs))
    assert not failures, failures[:5]


@pytest.mark.parametrize("fuse", ["0", "1"])
@pytest.mark.parametrize("ttype", ["c2c", "r2c"])
@pytest.mark.parametrize("dims", [(24, 20, 17), (67, 9, 10), (15, 67, 12), (9, 10, 131),
                                  (33, 18, 26), (8, 8, 9)])
@pytest.mark.parametrize("single", [False, True])
def test_batched_engine_paths(dims, ttype, fuse, single, monkeypatch):
    """The batched SIMD host engine: fused plane-block y/x path and separate
    stages (SPFFT_HOST_FUSE), packed-real (even dimX) and complex (odd dimX)
    C2R/R2C x lines, partial batches (plane / row / stick counts that are not a
    multiple of the SIMD width), prime lengths (67, 131: Rader) on SIMD lanes too."""
    monkeypatch.setenv("SPFFT_HOST_FUSE", fuse)
    nx, ny, nz = dims
    r2c = ttype == "r2c"
    rng = np.random.default_rng(5)
    idx = create_value_indices(rng, [1.0], 0.8, 0.8, nx, ny, nz, r2c)[0]
    G = sp.GridFloat if single else sp.Grid
    grid = G(nx, ny, nz, nx * ny, HOST, 3)
    t = grid.create_transform(HOST, sp.TransformType.R2C if r2c else sp.TransformType.C2C,
                              nx, ny, nz, nz, idx)
    tol = 2e-4 if single else 1e-11
    space = rng.standard_normal((nz, ny, nx))
    if not r2c:
        space = space + 1j * rng.standard_normal((nz, ny, nx))
    space = space.astype((np.float32 if r2c else np.complex64) if single else
                         (np.float64 if r2c else np.complex128))
    f = t.forward(space)
    assert max_rel_error(f, dense_forward(space.astype(np.complex128 if not r2c else np.float64),
                                          idx, dims, r2c=r2c)) < tol
    b = t.backward(f)
    ref = dense_backward(idx, np.asarray(f).astype(np.complex128), dims, r2c=r2c)
    assert max_rel_error(b, ref) < tol


@pytest.mark.parametrize("single", [False, True])
def test_step_api_distributed_host(single):
    """The step-wise API (backward_z / backward_exchange / backward_xy, forward_xy /
    forward_exchange / forward_z) of both precisions on 2 in-process ranks matches the
    whole calls and the dense oracle (reference: transform_internal.cpp step functions)."""
    from spfft_amd.parallel import make_distributed, run_ranks
    from spfft_amd.utils.indices import distribute_sticks, sphere_indices
    dims = (14, 12, 10)
    gidx = sphere_indices(*dims, 0.45)
    parts = distribute_sticks(gidx, 2, dims)
    rng = np.random.default_rng(3)
    vals = rng.standard_normal(len(gidx)) + 1j * rng.standard_normal(len(gidx))
    ref = dense_backward(gidx, vals, dims)
    tol = 2e-5 if single else 1e-12
    cdt = np.complex64 if single else np.complex128

    def body(rank, comm):
        s = make_distributed(comm, dims, gidx, processing_unit=HOST, single=single)
        start = sum(len(p) for p in parts[:rank])
        mine = np.ascontiguousarray(vals[start:start + len(s.indices)], dtype=cdt)
        t = s.transform
        t.backward_z(mine)
        t.backward_exchange()
        out = np.array(t.backward_xy())
        e1 = max_rel_error(out, ref[s.z_offset:s.z_offset + s.z_length])
        t.forward_xy()
        t.forward_exchange()
        f = t.forward_z(scaling=sp.Scaling.FULL)
        e2 = max_rel_error(f, mine)
        whole = t.forward(None, scaling=sp.Scaling.FULL)
        return e1, e2, max_rel_error(f, whole)

    for e1, e2, e3 in run_ranks(2, body):
        assert e1 < tol and e2 < tol and e3 < 1e-6, (e1, e2, e3)

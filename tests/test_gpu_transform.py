"""GPU numerics: the hand-written HIP stage kernels against fp64 references
(numpy for small sizes, torch.fft on the GPU for large ones)."""
import os

import numpy as np
import pytest

import spfft_amd as sp
from spfft_amd.utils.indices import (center_indices, create_value_indices, sphere_indices)
from spfft_amd.utils.oracle import dense_backward, dense_forward, max_rel_error

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

GPU = sp.ProcessingUnit.GPU
HOST = sp.ProcessingUnit.HOST


def _rand_vals(rng, n, single=False):
    v = rng.standard_normal(n) + 1j * rng.standard_normal(n)
    return v.astype(np.complex64 if single else np.complex128)


# lengths with a compile-time kernel (16..1024 powers of two) and run-time ones
SIZES = [(2, 2, 2), (11, 12, 13), (16, 32, 64), (100, 13, 12), (1, 1, 7), (128, 1, 256),
         (64, 100, 16), (13, 256, 1), (512, 3, 5), (36, 40, 45)]


@pytest.mark.parametrize("dims", SIZES)
@pytest.mark.parametrize("centered", [False, True])
def test_c2c_sweep(gpu, dims, centered):
    import torch
    rng = np.random.default_rng(7)
    nx, ny, nz = dims
    idx = create_value_indices(rng, [1.0], 0.7, 0.7, nx, ny, nz, False)[0]
    if centered:
        idx = center_indices(dims, [idx])[0]
    vals = _rand_vals(rng, len(idx))
    grid = sp.Grid(nx, ny, nz, nx * ny, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.C2C, nx, ny, nz, nz, idx)
    ref = dense_backward(idx, vals, dims)
    dv = torch.as_tensor(vals, device=gpu)
    for _ in range(2):  # twice: catches missing zero-fill (reference test_transform.hpp:129-131)
        out = t.backward(dv)
        assert max_rel_error(out.cpu().numpy(), ref) < 1e-12
    space = rng.standard_normal((nz, ny, nx)) + 1j * rng.standard_normal((nz, ny, nx))
    f = t.forward(torch.as_tensor(space, device=gpu))
    assert max_rel_error(f.cpu().numpy(), dense_forward(space, idx, dims)) < 1e-12


@pytest.mark.parametrize("dims", [(8, 8, 8), (11, 12, 13), (16, 16, 32), (12, 11, 4), (2, 13, 11),
                                  (256, 16, 16), (15, 64, 128), (4, 5, 6), (6, 7, 5), (200, 9, 8),
                                  (1024, 4, 4)])
def test_r2c(gpu, dims):
    import torch
    rng = np.random.default_rng(3)
    nx, ny, nz = dims
    space = rng.standard_normal((nz, ny, nx))
    idx = create_value_indices(rng, [1.0], 1.0, 1.0, nx, ny, nz, True)[0]
    grid = sp.Grid(nx, ny, nz, nx * ny, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.R2C, nx, ny, nz, nz, idx)
    f = t.forward(torch.as_tensor(space, device=gpu))
    assert max_rel_error(f.cpu().numpy(), dense_forward(space, idx, dims)) < 1e-12
    out = t.backward(f)
    assert max_rel_error(out.cpu().numpy(), space * (nx * ny * nz)) < 1e-12


@pytest.mark.parametrize("dims", [(16, 12, 10), (64, 32, 48), (30, 8, 9)])
def test_r2c_sparse_columns_single(gpu, dims):
    """Sparse R2C in fp32: x-columns present at k but absent at n/2-k exercise the
    packed-real pre/post passes' zero handling."""
    import torch
    rng = np.random.default_rng(8)
    nx, ny, nz = dims
    idx = create_value_indices(rng, [1.0], 0.5, 0.8, nx, ny, nz, True)[0]
    vals = dense_forward(rng.standard_normal((nz, ny, nx)), idx, dims).astype(np.complex64)
    grid = sp.GridFloat(nx, ny, nz, nx * ny, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.R2C, nx, ny, nz, nz, idx)
    out = t.backward(torch.as_tensor(vals, device=gpu))
    ref = dense_backward(idx, vals.astype(np.complex128), dims, r2c=True)
    assert max_rel_error(out.cpu().numpy(), ref) < 2e-5
    space = rng.standard_normal((nz, ny, nx)).astype(np.float32)
    f = t.forward(torch.as_tensor(space, device=gpu))
    assert max_rel_error(f.cpu().numpy(), dense_forward(space.astype(np.float64), idx, dims)) < 2e-5


def test_r2c_sphere_256(gpu):
    """Config 3 of BASELINE.json: 256^3 R2C spherical cutoff, fp64, vs torch.fft on the GPU."""
    import torch
    n = 256
    dims = (n, n, n)
    idx = sphere_indices(*dims, 0.5, r2c=True)
    rng = np.random.default_rng(13)
    space = torch.as_tensor(rng.standard_normal((n, n, n)), device=gpu)
    grid = sp.Grid(n, n, n, n * n, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.R2C, n, n, n, n, idx)
    f = t.forward(space)
    full = torch.fft.fftn(space.permute(2, 1, 0))  # [x][y][z]
    s = torch.as_tensor(np.where(idx < 0, idx + n, idx).astype(np.int64), device=gpu)
    ref = full[s[:, 0], s[:, 1], s[:, 2]]
    err = (f - ref).abs().max() / ref.abs().max()
    assert err.item() < 1e-12
    # backward of a hermitian-consistent spectrum (the forward output) is real and exact
    out = t.backward(f)
    F = torch.zeros((n // 2 + 1, n, n), dtype=torch.complex128, device=gpu)
    F[s[:, 0], s[:, 1], s[:, 2]] = f
    ref_b = torch.fft.irfftn(F.permute(2, 1, 0), s=(n, n, n), dim=(0, 1, 2)) * n ** 3
    err_b = (out - ref_b).abs().max() / ref_b.abs().max()
    assert err_b.item() < 1e-11


def test_r2c_half_plane_symmetry(gpu):
    """Only half of the x=0 plane / (0,0) stick given: hermitian fill on the GPU."""
    import torch
    rng = np.random.default_rng(5)
    dims = (12, 10, 14)
    nx, ny, nz = dims
    space = rng.standard_normal((nz, ny, nx))
    idx = create_value_indices(rng, [1.0], 1.0, 1.0, nx, ny, nz, True)[0]
    # keep the x = 0 plane only for y <= ny/2 and the (0,0) stick only for z <= nz/2 (generator does)
    vals = dense_forward(space, idx, dims)
    grid = sp.Grid(nx, ny, nz, nx * ny, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.R2C, nx, ny, nz, nz, idx)
    out = t.backward(torch.as_tensor(vals, device=gpu))
    ref = dense_backward(idx, vals, dims, r2c=True)
    assert max_rel_error(out.cpu().numpy(), ref) < 1e-12
    assert max_rel_error(out.cpu().numpy(), space * nx * ny * nz) < 1e-12


@pytest.mark.parametrize("n", [64, 128])
def test_sphere_c2c_large(gpu, n):
    """Config 2 of BASELINE.json: n^3 C2C spherical cutoff, fp64, checked with torch.fft."""
    import torch
    dims = (n, n, n)
    idx = sphere_indices(*dims, 0.5)
    rng = np.random.default_rng(11)
    vals = _rand_vals(rng, len(idx))
    grid = sp.Grid(n, n, n, n * n, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.C2C, n, n, n, n, idx)
    out = t.backward(torch.as_tensor(vals, device=gpu))
    s = torch.as_tensor(np.where(idx < 0, idx + n, idx).astype(np.int64), device=gpu)
    F = torch.zeros((n, n, n), dtype=torch.complex128, device=gpu)
    F[s[:, 0], s[:, 1], s[:, 2]] = torch.as_tensor(vals, device=gpu)
    ref = torch.fft.ifftn(F) * (n ** 3)
    ref = ref.permute(2, 1, 0)
    err = (out - ref).abs().max() / ref.abs().max()
    assert err.item() < 1e-12
    f = t.forward(None, scaling=sp.Scaling.FULL)
    assert (f.cpu() - torch.as_tensor(vals)).abs().max().item() < 1e-12 * np.abs(vals).max() * 10


@pytest.mark.parametrize("dims", [(11, 12, 13), (32, 32, 32), (64, 16, 36)])
def test_single_precision(gpu, dims):
    import torch
    rng = np.random.default_rng(2)
    nx, ny, nz = dims
    idx = create_value_indices(rng, [1.0], 0.7, 0.7, nx, ny, nz, False)[0]
    vals = _rand_vals(rng, len(idx), single=True)
    grid = sp.GridFloat(nx, ny, nz, nx * ny, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.C2C, nx, ny, nz, nz, idx)
    out = t.backward(torch.as_tensor(vals, device=gpu))
    ref = dense_backward(idx, vals.astype(np.complex128), dims)
    assert max_rel_error(out.cpu().numpy(), ref) < 2e-5


@pytest.mark.parametrize("dims", [(240, 6, 10), (15, 20, 30), (60, 90, 12), (120, 45, 7),
                                  (180, 36, 20), (100, 30, 16)])
@pytest.mark.parametrize("ttype", ["c2c", "r2c"])
@pytest.mark.parametrize("single", [False, True])
def test_composite_radices(gpu, dims, ttype, single):
    """Mixed-radix lengths in every stage (z row engine, y/x line-fast engines,
    packed-real x); the fp64 plans use the prime-factor codelets 6, 10, 12, 15,
    20 (rt_pfa), the fp32 plans the prime radices."""
    import torch
    rng = np.random.default_rng(17)
    nx, ny, nz = dims
    r2c = ttype == "r2c"
    idx = create_value_indices(rng, [1.0], 0.8, 0.8, nx, ny, nz, r2c)[0]
    if r2c:
        vals = dense_forward(rng.standard_normal((nz, ny, nx)), idx, dims)
    else:
        vals = _rand_vals(rng, len(idx))
    vals = vals.astype(np.complex64 if single else np.complex128)
    grid = (sp.GridFloat if single else sp.Grid)(nx, ny, nz, nx * ny, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.R2C if r2c else sp.TransformType.C2C,
                              nx, ny, nz, nz, idx)
    out = t.backward(torch.as_tensor(vals, device=gpu))
    ref = dense_backward(idx, vals.astype(np.complex128), dims, r2c=r2c)
    tol = 2e-5 if single else 1e-12
    assert max_rel_error(out.cpu().numpy(), ref) < tol
    space = rng.standard_normal((nz, ny, nx))
    if not r2c:
        space = space + 1j * rng.standard_normal((nz, ny, nx))
    space = space.astype((np.float32 if r2c else np.complex64) if single else
                         (np.float64 if r2c else np.complex128))
    f = t.forward(torch.as_tensor(space, device=gpu))
    assert max_rel_error(f.cpu().numpy(), dense_forward(space.astype(np.complex128), idx, dims)) < tol


@pytest.mark.parametrize("dims", [(240, 12, 10), (10, 200, 12), (12, 10, 192), (192, 240, 200),
                                  (96, 144, 216), (360, 8, 10), (6, 480, 8), (10, 6, 384),
                                  (100, 108, 125), (150, 135, 12), (250, 10, 100),
                                  (48, 60, 72), (80, 90, 12), (180, 8, 60)])
@pytest.mark.parametrize("ttype", ["c2c", "r2c"])
@pytest.mark.parametrize("single", [False, True])
def test_mixed_radix_ct_lengths(gpu, dims, ttype, single):
    """The compile-time mixed-radix kernels (FftMR, SPFFT_MR_SIZES: 2- and 3-pass
    plans such as 240 = 16*15, 200 = 20*10 / 10*10*2, 216 = 12*6*3) on every axis:
    z row engine, y/x line-fast engines, packed-real x stage on N/2."""
    import torch
    rng = np.random.default_rng(29)
    nx, ny, nz = dims
    r2c = ttype == "r2c"
    idx = create_value_indices(rng, [1.0], 0.8, 0.8, nx, ny, nz, r2c)[0]
    if r2c:
        vals = dense_forward(rng.standard_normal((nz, ny, nx)), idx, dims)
    else:
        vals = _rand_vals(rng, len(idx))
    vals = vals.astype(np.complex64 if single else np.complex128)
    grid = (sp.GridFloat if single else sp.Grid)(nx, ny, nz, nx * ny, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.R2C if r2c else sp.TransformType.C2C,
                              nx, ny, nz, nz, idx)
    out = t.backward(torch.as_tensor(vals, device=gpu))
    ref = dense_backward(idx, vals.astype(np.complex128), dims, r2c=r2c)
    tol = 2e-5 if single else 1e-12
    assert max_rel_error(out.cpu().numpy(), ref) < tol
    space = rng.standard_normal((nz, ny, nx))
    if not r2c:
        space = space + 1j * rng.standard_normal((nz, ny, nx))
    space = space.astype((np.float32 if r2c else np.complex64) if single else
                         (np.float64 if r2c else np.complex128))
    f = t.forward(torch.as_tensor(space, device=gpu))
    assert max_rel_error(f.cpu().numpy(), dense_forward(space.astype(np.complex128), idx, dims)) < tol


def test_host_pointers_on_gpu_transform(gpu):
    """GPU transform with host input/output and host space domain (staging paths)."""
    rng = np.random.default_rng(4)
    dims = (16, 12, 20)
    nx, ny, nz = dims
    idx = create_value_indices(rng, [1.0], 0.8, 0.8, nx, ny, nz, False)[0]
    vals = _rand_vals(rng, len(idx))
    grid = sp.Grid(nx, ny, nz, nx * ny, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.C2C, nx, ny, nz, nz, idx)
    out = t.backward(vals, HOST)
    assert isinstance(out, np.ndarray)
    assert max_rel_error(out, dense_backward(idx, vals, dims)) < 1e-12
    res = np.empty(len(idx), dtype=np.complex128)
    t.forward(None, output=res, input_location=HOST, scaling=sp.Scaling.FULL)
    assert max_rel_error(res, vals) < 1e-12


@pytest.mark.parametrize("exchange", list(sp.ExchangeType))
def test_gpu_virtual_ranks(gpu, exchange):
    """P virtual ranks on one GPU (in-process group, peer-copy data plane) through the
    distributed pack/unpack layouts of every exchange type."""
    import torch
    from spfft_amd.parallel import make_distributed, run_ranks
    from spfft_amd.utils.indices import distribute_sticks
    dims = (24, 20, 18)
    gidx = sphere_indices(*dims, 0.5)
    rng = np.random.default_rng(9)
    vals = _rand_vals(rng, len(gidx))
    ref = dense_backward(gidx, vals, dims)
    P = 3
    parts = distribute_sticks(gidx, P, dims)
    tol = 1e-6 if exchange in (sp.ExchangeType.BUFFERED_FLOAT,
                               sp.ExchangeType.COMPACT_BUFFERED_FLOAT) else 1e-12

    def body(rank, comm):
        torch.cuda.set_device(0)
        s = make_distributed(comm, dims, gidx, processing_unit=GPU, exchange_type=exchange)
        start = sum(len(p) for p in parts[:rank])
        v = torch.as_tensor(vals[start:start + len(s.indices)], device="cuda")
        out = s.transform.backward(v).cpu().numpy()
        e1 = max_rel_error(out, ref[s.z_offset:s.z_offset + s.z_length])
        f = s.transform.forward(None, scaling=sp.Scaling.FULL).cpu().numpy()
        e2 = max_rel_error(f, v.cpu().numpy())
        return e1, e2

    for e1, e2 in run_ranks(P, body):
        assert e1 < tol and e2 < tol


@pytest.mark.parametrize("exchange", ["COMPACT_BUFFERED", "BUFFERED"])
@pytest.mark.parametrize("nz", [4000, 5000])
def test_gpu_virtual_ranks_z_near_lds_limit(gpu, exchange, nz):
    """Distributed plan whose z engine nearly fills the 160 KB LDS (fp64 run-time
    engine, dimZ 4000 / 5000): the per-plane exchange segment table no longer fits
    next to it and is read from global memory instead (z_args_for_lds)."""
    import torch
    from spfft_amd.parallel import make_distributed, run_ranks
    from spfft_amd.utils.indices import distribute_sticks
    dims = (6, 5, nz)
    gidx = sphere_indices(*dims, 0.5)
    rng = np.random.default_rng(19)
    vals = _rand_vals(rng, len(gidx))
    ref = dense_backward(gidx, vals, dims)
    P = 2
    parts = distribute_sticks(gidx, P, dims)
    ex = getattr(sp.ExchangeType, exchange)

    def body(rank, comm):
        torch.cuda.set_device(0)
        s = make_distributed(comm, dims, gidx, processing_unit=GPU, exchange_type=ex)
        start = sum(len(p) for p in parts[:rank])
        v = torch.as_tensor(vals[start:start + len(s.indices)], device="cuda")
        out = s.transform.backward(v).cpu().numpy()
        e1 = max_rel_error(out, ref[s.z_offset:s.z_offset + s.z_length])
        f = s.transform.forward(None, scaling=sp.Scaling.FULL).cpu().numpy()
        e2 = max_rel_error(f, v.cpu().numpy())
        return e1, e2

    for e1, e2 in run_ranks(P, body):
        assert e1 < 1e-11 and e2 < 1e-11


def test_multi_transform_gpu(gpu):
    import torch
    rng = np.random.default_rng(12)
    dims = (32, 24, 20)
    nx, ny, nz = dims
    idx = sphere_indices(*dims, 0.5)
    grid = sp.Grid(nx, ny, nz, nx * ny, GPU, 1)
    t0 = grid.create_transform(GPU, sp.TransformType.C2C, nx, ny, nz, nz, idx)
    ts = [t0, t0.clone(), t0.clone()]
    vals = [_rand_vals(rng, len(idx)) for _ in ts]
    outs = sp.multi_transform_backward(ts, [torch.as_tensor(v, device=gpu) for v in vals])
    for o, v in zip(outs, vals):
        assert max_rel_error(o.cpu().numpy(), dense_backward(idx, v, dims)) < 1e-12
    res = sp.multi_transform_forward(ts, scalings=[sp.Scaling.FULL] * 3)
    for r, v in zip(res, vals):
        assert max_rel_error(r.cpu().numpy(), v) < 1e-12
    with pytest.raises(sp.InvalidParameterError):
        sp.multi_transform_backward([t0, t0], [vals[0], vals[0]])


@pytest.mark.parametrize("ttype,single", [("C2C", False), ("R2C", False), ("C2C", True),
                                           ("R2C", True)])
@pytest.mark.parametrize("dims", [(32, 24, 20), (64, 64, 64)])
def test_multi_transform_batched(gpu, ttype, single, dims):
    """Batched multi_transform: transforms with identical plans share one launch per
    stage (blockIdx.z = transform, groups of at most 8). 10 clones (a batch of 8 and one
    of 2) plus a transform with another index set (unbatched path) in the middle; every
    result equals the one-at-a-time result of a separate transform."""
    import torch
    rng = np.random.default_rng(21)
    tt = getattr(sp.TransformType, ttype)
    r2c = tt == sp.TransformType.R2C
    nx, ny, nz = dims
    GridCls = sp.GridFloat if single else sp.Grid
    idx = sphere_indices(*dims, 0.5, r2c=r2c)
    idx_o = sphere_indices(*dims, 0.3, r2c=r2c)

    def make(ix):
        g = GridCls(nx, ny, nz, nx * ny, GPU, 1)
        return g, g.create_transform(GPU, tt, nx, ny, nz, nz, ix)

    g0, t0 = make(idx)
    go, to = make(idx_o)
    ts = [t0] + [t0.clone() for _ in range(9)]
    ts.insert(5, to)
    vals = [torch.as_tensor(_rand_vals(rng, len(idx_o if t is to else idx), single), device=gpu)
            for t in ts]
    sp.timing_reset()
    sp.timing_enable(True)
    try:
        spaces = [s.clone() for s in sp.multi_transform_backward(ts, vals)]
        outs = sp.multi_transform_forward(ts, scalings=[sp.Scaling.FULL] * len(ts))
        torch.cuda.synchronize()
        rep = sp.timing_report()
    finally:
        sp.timing_enable(False)
    assert "gpu_backward_batch" in rep and "gpu_forward_batch" in rep, rep
    _, ref = make(idx)
    _, ref_o = make(idx_o)
    tol = 1e-5 if single else 1e-13
    for t, v, s, o in zip(ts, vals, spaces, outs):
        r = ref_o if t is to else ref
        rs = r.backward(v).clone()
        ro = r.forward(None, scaling=sp.Scaling.FULL)
        assert max_rel_error(s.cpu().numpy(), rs.cpu().numpy()) <= tol
        assert max_rel_error(o.cpu().numpy(), ro.cpu().numpy()) <= tol
        if not r2c:
            ix = idx_o if t is to else idx
            ref_space = dense_backward(ix, v.cpu().numpy().astype(np.complex128), dims)
            assert max_rel_error(s.cpu().numpy(), ref_space) < (1e-4 if single else 1e-12)
            assert max_rel_error(o.cpu().numpy(), v.cpu().numpy()) < (1e-4 if single else 1e-12)


@pytest.mark.parametrize("split", ["2", "3"])
def test_multi_transform_batched_streams(gpu, monkeypatch, split):
    """Large-grid batching (SPFFT_BATCH_LARGE=0 makes every grid "large"): transforms on
    their own async user streams run in sub-batches of SPFFT_BATCH_SPLIT on the
    sub-batch leader's stream, joined to the members' streams by events; later work
    on each member's stream sees the results."""
    import torch
    monkeypatch.setenv("SPFFT_BATCH_LARGE", "0")
    monkeypatch.setenv("SPFFT_BATCH_SPLIT", split)
    rng = np.random.default_rng(23)
    dims = (48, 40, 36)
    idx = sphere_indices(*dims, 0.5)
    grid = sp.Grid(*dims, 48 * 40, GPU, 1)
    t0 = grid.create_transform(GPU, sp.TransformType.C2C, *dims, 36, idx)
    ts = [t0] + [t0.clone() for _ in range(4)]
    streams = [torch.cuda.Stream() for _ in ts]
    for t, st in zip(ts, streams):
        t.set_stream(st, synchronous=False)
    vals = [torch.as_tensor(_rand_vals(rng, len(idx)), device=gpu) for _ in ts]
    outs = [torch.empty_like(v) for v in vals]
    sp.timing_reset()
    sp.timing_enable(True)
    try:
        for _ in range(2):
            spaces = sp.multi_transform_backward(ts, vals)
            copies = []
            for s_, st in zip(spaces, streams):
                with torch.cuda.stream(st):  # ordered after the batch on each stream
                    copies.append(s_.clone())
            sp.multi_transform_forward(ts, outputs=outs, scalings=[sp.Scaling.FULL] * len(ts))
        torch.cuda.synchronize()
        rep = sp.timing_report()
    finally:
        sp.timing_enable(False)
    assert "gpu_backward_batch" in rep and "gpu_forward_batch" in rep, rep
    for c, o, v in zip(copies, outs, vals):
        assert max_rel_error(c.cpu().numpy(), dense_backward(idx, v.cpu().numpy(), dims)) < 1e-12
        assert max_rel_error(o.cpu().numpy(), v.cpu().numpy()) < 1e-12


def test_multi_transform_batched_mixed_scaling(gpu):
    """Forward batches group transforms of equal scaling only ([NONE, FULL, FULL, NONE]
    -> two batches); each output matches its scaling."""
    import torch
    rng = np.random.default_rng(24)
    dims = (32, 32, 32)
    idx = sphere_indices(*dims, 0.5)
    grid = sp.Grid(*dims, 32 * 32, GPU, 1)
    t0 = grid.create_transform(GPU, sp.TransformType.C2C, *dims, 32, idx)
    ts = [t0] + [t0.clone() for _ in range(3)]
    vals = [torch.as_tensor(_rand_vals(rng, len(idx)), device=gpu) for _ in ts]
    sp.multi_transform_backward(ts, vals)
    sc = [sp.Scaling.NONE, sp.Scaling.FULL, sp.Scaling.FULL, sp.Scaling.NONE]
    outs = sp.multi_transform_forward(ts, scalings=sc)
    n = float(np.prod(dims))
    for o, v, s_ in zip(outs, vals, sc):
        ref = v.cpu().numpy() * (1.0 if s_ == sp.Scaling.FULL else n)
        assert max_rel_error(o.cpu().numpy(), ref) < 1e-12


def test_multi_transform_batch_disabled(gpu, monkeypatch):
    """SPFFT_BATCH=0 (read at transform creation) keeps every transform on its own
    launches; results are unchanged."""
    import torch
    monkeypatch.setenv("SPFFT_BATCH", "0")
    rng = np.random.default_rng(22)
    dims = (32, 32, 32)
    idx = sphere_indices(*dims, 0.5)
    grid = sp.Grid(*dims, 32 * 32, GPU, 1)
    t0 = grid.create_transform(GPU, sp.TransformType.C2C, *dims, 32, idx)
    ts = [t0, t0.clone()]
    vals = [torch.as_tensor(_rand_vals(rng, len(idx)), device=gpu) for _ in ts]
    sp.timing_reset()
    sp.timing_enable(True)
    try:
        outs = [s.clone() for s in sp.multi_transform_backward(ts, vals)]
        torch.cuda.synchronize()
        rep = sp.timing_report()
    finally:
        sp.timing_enable(False)
    assert "gpu_backward_batch" not in rep
    for o, v in zip(outs, vals):
        assert max_rel_error(o.cpu().numpy(), dense_backward(idx, v.cpu().numpy(), dims)) < 1e-12


def test_user_stream_async(gpu):
    import torch
    rng = np.random.default_rng(13)
    dims = (64, 64, 64)
    idx = sphere_indices(*dims, 0.4)
    vals = torch.as_tensor(_rand_vals(rng, len(idx)), device=gpu)
    grid = sp.Grid(*dims, 64 * 64, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.C2C, *dims, 64, idx)
    s = torch.cuda.Stream()
    t.set_stream(s, synchronous=False)
    with torch.cuda.stream(s):
        t.backward(vals)
        out = t.forward(None, scaling=sp.Scaling.FULL)
    t.synchronize()
    assert (out - vals).abs().max().item() < 1e-12


@pytest.mark.parametrize("chunks,exchange,blocks", [
    (1, "COMPACT_BUFFERED", 1), (3, "COMPACT_BUFFERED", 1), (8, "COMPACT_BUFFERED", 1),
    (3, "COMPACT_BUFFERED_FLOAT", 1), (3, "BUFFERED", 1), (1, "COMPACT_BUFFERED", 2),
    (2, "COMPACT_BUFFERED", 2), (2, "BUFFERED", 4), (4, "COMPACT_BUFFERED_FLOAT", 2)])
@pytest.mark.parametrize("dist", ["uniform", "rank0", "rank0_planes_last", "r2c"])
def test_gpu_virtual_ranks_distributions(gpu, dist, chunks, exchange, blocks, monkeypatch):
    """Reference distribution sweep (tests/mpi_tests/test_transform.cpp) on P=3 virtual
    ranks of one GPU, through the pipelined exchange's 2D grid of stick blocks x plane
    chunks (1..8 chunks, 1..4 stick blocks; ranks with few or no planes or sticks get
    empty messages and every rank issues the same steps), also with fp32 exchange
    buffers and the padded BUFFERED layout."""
    import torch
    from spfft_amd.parallel import run_ranks
    from spfft_amd.utils.indices import calculate_num_local_xy_planes
    monkeypatch.setenv("SPFFT_EXCH_CHUNKS", str(chunks))
    monkeypatch.setenv("SPFFT_EXCH_STICK_BLOCKS", str(blocks))
    dims = (20, 18, 17)
    nx, ny, nz = dims
    P = 3
    r2c = dist == "r2c"
    stick_dist = {"uniform": [1, 1, 1], "rank0": [1, 0, 0], "rank0_planes_last": [1, 0, 0],
                  "r2c": [1, 2, 1]}[dist]
    plane_dist = {"uniform": [1, 1, 1], "rank0": [1, 0, 0], "rank0_planes_last": [0, 0, 1],
                  "r2c": [1, 1, 1]}[dist]
    rng = np.random.default_rng(21)
    parts = create_value_indices(rng, stick_dist, 0.7, 0.8, nx, ny, nz, r2c)
    planes = [calculate_num_local_xy_planes(r, nz, plane_dist) for r in range(P)]
    offsets = np.concatenate([[0], np.cumsum(planes)])
    all_idx = np.concatenate(parts)
    space = rng.standard_normal((nz, ny, nx))
    if r2c:
        vals_all = dense_forward(space, all_idx, dims, r2c=True)
    else:
        vals_all = _rand_vals(rng, len(all_idx))
    ref = dense_backward(all_idx, vals_all, dims, r2c=r2c)
    field = space if r2c else space + 1j * rng.standard_normal((nz, ny, nx))
    ref_fwd = dense_forward(field, all_idx, dims, r2c=r2c)
    starts = np.concatenate([[0], np.cumsum([len(p) for p in parts])])
    ttype = sp.TransformType.R2C if r2c else sp.TransformType.C2C
    max_sticks = max(len(np.unique(p[:, 0] * ny + p[:, 1])) if len(p) else 0 for p in parts)

    def body(rank, comm):
        torch.cuda.set_device(0)
        grid = sp.Grid(nx, ny, nz, max(1, max_sticks), GPU, 1, max_local_z_length=max(planes),
                       comm=comm, exchange_type=getattr(sp.ExchangeType, exchange))
        t = grid.create_transform(GPU, ttype, nx, ny, nz, planes[rank], parts[rank])
        v = torch.as_tensor(vals_all[starts[rank]:starts[rank + 1]], device="cuda")
        errs = []
        for _ in range(2):
            out = t.backward(v).cpu().numpy()
            errs.append(max_rel_error(out, ref[offsets[rank]:offsets[rank + 1]]) if planes[rank]
                        else 0.0)
        # forward of this rank's slab of a known field
        slab = torch.as_tensor(np.ascontiguousarray(field[offsets[rank]:offsets[rank + 1]]),
                               device="cuda")
        f = t.forward(slab).cpu().numpy()
        errs.append(max_rel_error(f, ref_fwd[starts[rank]:starts[rank + 1]]) if len(f) else 0.0)
        return max(errs)

    tol = 1e-5 if exchange.endswith("FLOAT") else 1e-11
    for e in run_ranks(P, body):
        assert e < tol


@pytest.mark.parametrize("dims,sticks,planes", [
    ((2, 64, 5), [1, 1], [1, 1]), ((2, 64, 5), [1, 1], [0, 1]), ((2, 64, 5), [1, 0], [0, 1]),
    ((4, 32, 6), [1, 2, 1], [1, 0, 2]), ((3, 128, 4), [0, 1, 1], [1, 1, 0])])
def test_unbuffered_skewed_distributions(gpu, dims, sticks, planes):
    """UNBUFFERED (peer writes) with y lengths on the compile-time engines, whose y stage
    reads the stick bases from an LDS table: a peer's buffer below the local one gives a
    negative base, which the table's old -1 "no entry" marker dropped (found by
    tools/fuzz_gpu.py). Every rank with planes writes into every rank with sticks."""
    import torch
    from spfft_amd.parallel import run_ranks
    from spfft_amd.utils.indices import calculate_num_local_xy_planes
    nx, ny, nz = dims
    P = len(sticks)
    rng = np.random.default_rng(64)
    parts = create_value_indices(rng, sticks, 0.9, 0.8, nx, ny, nz, False)
    pl = [calculate_num_local_xy_planes(r, nz, planes) for r in range(P)]
    offsets = np.concatenate([[0], np.cumsum(pl)])
    all_idx = np.concatenate(parts)
    field = rng.standard_normal((nz, ny, nx)) + 1j * rng.standard_normal((nz, ny, nx))
    vals = dense_forward(field, all_idx, dims)
    ref = dense_backward(all_idx, vals, dims)
    starts = np.concatenate([[0], np.cumsum([len(p) for p in parts])])
    ms = max(len(np.unique(p[:, 0].astype(np.int64) * ny + p[:, 1])) if len(p) else 0 for p in parts)

    def body(rank, comm):
        torch.cuda.set_device(0)
        grid = sp.Grid(nx, ny, nz, max(1, ms), GPU, 1, max_local_z_length=max(pl), comm=comm,
                       exchange_type=sp.ExchangeType.UNBUFFERED)
        t = grid.create_transform(GPU, sp.TransformType.C2C, nx, ny, nz, pl[rank], parts[rank])
        errs = []
        for _ in range(2):
            v = torch.as_tensor(vals[starts[rank]:starts[rank + 1]], device="cuda")
            out = t.backward(v).cpu().numpy()
            errs.append(max_rel_error(out, ref[offsets[rank]:offsets[rank + 1]]) if pl[rank] else 0.0)
            slab = torch.as_tensor(np.ascontiguousarray(field[offsets[rank]:offsets[rank + 1]]),
                                   device="cuda")
            f = t.forward(slab).cpu().numpy()
            errs.append(max_rel_error(f, vals[starts[rank]:starts[rank + 1]]) if len(f) else 0.0)
        return max(errs)

    for e in run_ranks(P, body):
        assert e < 1e-11


@pytest.mark.parametrize("dims,ttype", [((16, 12, 20), "c2c"), ((11, 13, 12), "c2c"),
                                        ((16, 10, 14), "r2c"), ((15, 8, 9), "r2c"),
                                        ((64, 64, 64), "c2c")])
def test_nan_poison(gpu, dims, ttype, monkeypatch):
    """SPFFT_POISON=1 fills every work buffer with NaN before each direction: a kernel
    reading an element no stage wrote would leak NaN into the result."""
    import torch
    monkeypatch.setenv("SPFFT_POISON", "1")
    rng = np.random.default_rng(17)
    nx, ny, nz = dims
    r2c = ttype == "r2c"
    idx = create_value_indices(rng, [1.0], 0.6, 0.6, nx, ny, nz, r2c)[0]
    space = rng.standard_normal((nz, ny, nx))
    if not r2c:
        space = space + 1j * rng.standard_normal((nz, ny, nx))
    vals = dense_forward(space, idx, dims, r2c=r2c)
    grid = sp.Grid(nx, ny, nz, nx * ny, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.R2C if r2c else sp.TransformType.C2C,
                              nx, ny, nz, nz, idx)
    out = t.backward(torch.as_tensor(vals, device=gpu))
    assert not torch.isnan(out).any()
    assert max_rel_error(out.cpu().numpy(), dense_backward(idx, vals, dims, r2c=r2c)) < 1e-12
    f = t.forward(torch.as_tensor(space, device=gpu))
    assert not torch.isnan(f).any()
    assert max_rel_error(f.cpu().numpy(), dense_forward(space, idx, dims, r2c=r2c)) < 1e-12


@pytest.mark.parametrize("dims,r2c,single", [((67, 8, 101), False, False), ((127, 3, 2), False, False),
                                             ((103, 16, 67), True, False), ((2, 257, 5), False, True),
                                             ((1021, 2, 3), False, False), ((97, 89, 4), True, True)])
def test_gpu_bluestein(gpu, dims, r2c, single):
    """GPU lengths with a prime factor > 61: Bluestein engine (chirp-z, power-of-two
    convolution in LDS) inside the stage kernels."""
    import torch
    nx, ny, nz = dims
    rng = np.random.default_rng(31)
    idx = create_value_indices(rng, [1.0], 0.8, 0.9, nx, ny, nz, r2c)[0]
    space = rng.standard_normal((nz, ny, nx))
    if not r2c:
        space = space + 1j * rng.standard_normal((nz, ny, nx))
    vals = dense_forward(space, idx, dims, r2c=r2c)
    tol = 2e-5 if single else 1e-11
    cls = sp.GridFloat if single else sp.Grid
    g = cls(nx, ny, nz, nx * ny, GPU, 1)
    t = g.create_transform(GPU, sp.TransformType.R2C if r2c else sp.TransformType.C2C,
                           nx, ny, nz, nz, idx)
    vdt = np.complex64 if single else np.complex128
    out = t.backward(torch.as_tensor(vals.astype(vdt), device=gpu))
    assert max_rel_error(out.cpu().numpy(), dense_backward(idx, vals, dims, r2c=r2c)) < tol
    sdt = (np.float32 if r2c else np.complex64) if single else space.dtype
    f = t.forward(torch.as_tensor(space.astype(sdt), device=gpu))
    assert max_rel_error(f.cpu().numpy(), vals) < tol


@pytest.mark.parametrize("ttype", ["c2c", "r2c"])
def test_graph_replay(gpu, ttype, monkeypatch):
    """Whole-direction hipGraph replay (opt-in SPFFT_GRAPH=1, private stream):
    the first call of a direction runs step-wise, the second is captured, later
    calls replay; buffers are refilled in place between calls (a graph must read
    them afresh) and a new output buffer triggers a new capture."""
    import torch
    monkeypatch.setenv("SPFFT_GRAPH", "1")
    rng = np.random.default_rng(21)
    dims = (64, 48, 40)
    nx, ny, nz = dims
    r2c = ttype == "r2c"
    idx = sphere_indices(*dims, 0.45, r2c=r2c)
    grid = sp.Grid(*dims, nx * ny, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.R2C if r2c else sp.TransformType.C2C,
                              *dims, nz, idx)
    t.set_stream(None)  # the library's private stream (torch's default stream is not capturable)
    sp.timing_reset()
    sp.timing_enable(True)
    try:
        vbuf = torch.empty(len(idx), dtype=torch.complex128, device=gpu)
        outs = [torch.empty_like(vbuf), torch.empty_like(vbuf)]
        for it in range(5):
            out = outs[it // 3]
            if r2c:
                space = rng.standard_normal((nz, ny, nx))
                f = t.forward(torch.as_tensor(space, device=gpu), output=out)
                ref = dense_forward(space, idx, dims)
                assert max_rel_error(f.cpu().numpy(), ref) < 1e-12
                vbuf.copy_(f)
                back = t.backward(vbuf)
                ref = dense_backward(idx, f.cpu().numpy(), dims, r2c=True)
                assert max_rel_error(back.cpu().numpy(), ref) < 1e-12
            else:
                vals = _rand_vals(rng, len(idx))
                vbuf.copy_(torch.as_tensor(vals, device=gpu))
                back = t.backward(vbuf)
                assert max_rel_error(back.cpu().numpy(), dense_backward(idx, vals, dims)) < 1e-12
                f = t.forward(None, output=out, scaling=sp.Scaling.FULL)
                assert max_rel_error(f.cpu().numpy(), vals) < 1e-12
        report = sp.timing_report()
    finally:
        sp.timing_enable(False)
    assert "gpu_backward_graph" in report and "gpu_forward_graph" in report, report


def test_gpu_stage_timing(gpu):
    """SPFFT_TIMING: hipEvent intervals of every stage land in the timing tree
    (gpu/<direction>/<stage>) once the calls completed; SURVEY.md section 5."""
    import torch
    rng = np.random.default_rng(31)
    dims = (64, 64, 64)
    idx = sphere_indices(*dims, 0.5)
    grid = sp.Grid(*dims, 64 * 64, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.C2C, *dims, 64, idx)
    vals = torch.as_tensor(_rand_vals(rng, len(idx)), device=gpu)
    sp.timing_reset()
    sp.timing_enable(True)
    try:
        for _ in range(3):
            t.backward(vals)
            t.forward(None, scaling=sp.Scaling.FULL)
        t.synchronize()
        tree = sp.timing_json()
    finally:
        sp.timing_enable(False)
    gpu_node = [n for n in tree["timings"] if n["identifier"] == "gpu"]
    assert gpu_node, tree
    dirs = {d["identifier"]: {s["identifier"]: s for s in d["sub-timings"]}
            for d in gpu_node[0]["sub-timings"]}
    assert set(dirs) == {"backward", "forward"}, dirs
    for d, stages in (("backward", ("z", "exchange", "y+x")), ("forward", ("x+y", "exchange", "z"))):
        for st in stages:
            node = dirs[d][st]
            assert node["count"] == 3, (d, st, node)
            assert node["min"] >= 0.0
        # the FFT stages of a 64^3 transform take measurable GPU time
        assert dirs[d]["z"]["total"] > 0.0


def test_reference_size_sweep_full(gpu):
    """The reference's complete local sweep on the GPU: X, Y, Z in {1, 2, 11, 12, 13, 100}
    (all 216 combinations; tests/local_tests/test_local_transform.cpp), C2C with and
    without centred indices (run twice: zero-fill), forward with full scaling, and R2C
    forward/backward against numpy."""
    import itertools

    import torch
    sizes = [1, 2, 11, 12, 13, 100]
    rng = np.random.default_rng(216)
    failures = []
    for n, dims in enumerate(itertools.product(sizes, sizes, sizes)):
        nx, ny, nz = dims
        centered = n % 2 == 1
        idx = create_value_indices(rng, [1.0], 0.7, 0.7, nx, ny, nz, False)[0]
        if centered:
            idx = center_indices(dims, [idx])[0]
        vals = _rand_vals(rng, len(idx))
        grid = sp.Grid(nx, ny, nz, nx * ny, GPU, 1)
        t = grid.create_transform(GPU, sp.TransformType.C2C, nx, ny, nz, nz, idx)
        ref = dense_backward(idx, vals, dims)
        dv = torch.as_tensor(vals, device=gpu)
        errs = [max_rel_error(t.backward(dv).cpu().numpy(), ref) for _ in range(2)]
        space = rng.standard_normal((nz, ny, nx)) + 1j * rng.standard_normal((nz, ny, nx))
        f = t.forward(torch.as_tensor(space, device=gpu), scaling=sp.Scaling.FULL)
        errs.append(max_rel_error(f.cpu().numpy(), dense_forward(space, idx, dims, scale=True)))
        # R2C on the same grid shape (hermitian half of the indices)
        ridx = create_value_indices(rng, [1.0], 1.0, 1.0, nx, ny, nz, True)[0]
        rgrid = sp.Grid(nx, ny, nz, nx * ny, GPU, 1)
        rt = rgrid.create_transform(GPU, sp.TransformType.R2C, nx, ny, nz, nz, ridx)
        rspace = rng.standard_normal((nz, ny, nx))
        rf = rt.forward(torch.as_tensor(rspace, device=gpu))
        errs.append(max_rel_error(rf.cpu().numpy(), dense_forward(rspace, ridx, dims)))
        rb = rt.backward(rf)
        errs.append(max_rel_error(rb.cpu().numpy(), dense_backward(ridx, rf.cpu().numpy(), dims,
                                                                   r2c=True)))
        if max(errs) > 1e-11:
            failures.append((dims, centered, errs))
    assert not failures, failures[:5]


@pytest.mark.parametrize("exchange,chunks", [("COMPACT_BUFFERED", 3), ("UNBUFFERED", 1),
                                             ("BUFFERED", 1)])
def test_gpu_virtual_ranks_empty_transform(gpu, exchange, chunks, monkeypatch):
    """No frequency values on any rank (a valid SpFFT transform): backward gives a zero
    space domain, forward returns nothing, through every data plane and the chunk plan."""
    import torch
    from spfft_amd.parallel import run_ranks
    monkeypatch.setenv("SPFFT_EXCH_CHUNKS", str(chunks))
    dims = (16, 12, 10)
    nx, ny, nz = dims
    planes = [5, 5]

    def body(rank, comm):
        torch.cuda.set_device(0)
        grid = sp.Grid(nx, ny, nz, 1, GPU, 1, max_local_z_length=5, comm=comm,
                       exchange_type=getattr(sp.ExchangeType, exchange))
        t = grid.create_transform(GPU, sp.TransformType.C2C, nx, ny, nz, planes[rank],
                                  np.zeros((0, 3), dtype=np.int32))
        out = t.backward(torch.zeros(0, dtype=torch.complex128, device="cuda"))
        zero = float(out.abs().max().item()) if out.numel() else 0.0
        f = t.forward(None)
        return zero, len(f)

    for zero, nf in run_ranks(2, body):
        assert zero == 0.0 and nf == 0


@pytest.mark.parametrize("dims", [(1024, 8, 12), (16, 1024, 8), (8, 12, 1024), (512, 16, 10),
                                  (10, 512, 6)])
@pytest.mark.parametrize("single", [False, True])
@pytest.mark.parametrize("ttype", ["c2c", "r2c"])
def test_long_lines(gpu, dims, single, ttype):
    """Lengths 512 and 1024 along each axis: the wide (512-thread, up to 139 KB LDS)
    line-fast shapes of the x/y stages and the row-mapped z shapes, fp64 and fp32."""
    import torch
    rng = np.random.default_rng(1024)
    nx, ny, nz = dims
    r2c = ttype == "r2c"
    idx = create_value_indices(rng, [1.0], 0.6, 0.8, nx, ny, nz, r2c)[0]
    G = sp.GridFloat if single else sp.Grid
    grid = G(nx, ny, nz, nx * ny, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.R2C if r2c else sp.TransformType.C2C,
                              nx, ny, nz, nz, idx)
    tol = 1e-4 if single else 1e-11
    cdt = torch.complex64 if single else torch.complex128
    if r2c:
        space = rng.standard_normal((nz, ny, nx))
        f = t.forward(torch.as_tensor(space.astype(np.float32 if single else np.float64), device=gpu))
        assert max_rel_error(f.cpu().numpy(), dense_forward(space, idx, dims)) < tol
        b = t.backward(f)
        ref = dense_backward(idx, f.cpu().numpy().astype(np.complex128), dims, r2c=True)
        assert max_rel_error(b.cpu().numpy(), ref) < tol
    else:
        vals = _rand_vals(rng, len(idx), single)
        out = t.backward(torch.as_tensor(vals, device=gpu, dtype=cdt))
        assert max_rel_error(out.cpu().numpy(), dense_backward(idx, vals, dims)) < tol
        space = rng.standard_normal((nz, ny, nx)) + 1j * rng.standard_normal((nz, ny, nx))
        f = t.forward(torch.as_tensor(space, device=gpu, dtype=cdt))
        assert max_rel_error(f.cpu().numpy(), dense_forward(space, idx, dims)) < tol


@pytest.mark.parametrize("exchange", ["COMPACT_BUFFERED", "COMPACT_BUFFERED_FLOAT", "BUFFERED",
                                      "BUFFERED_FLOAT", "UNBUFFERED"])
@pytest.mark.parametrize("P,chunks,blocks", [(8, 1, 1), (8, 2, 1), (8, 4, 1), (4, 3, 1), (2, 4, 1),
                                             (8, 2, 2), (4, 2, 4), (2, 1, 2)])
def test_gpu_virtual_ranks_scale_configs(gpu, P, chunks, blocks, exchange, monkeypatch):
    """The driver's scaling configurations (2/4/8 ranks, the chunk counts the automatic
    rule picks at 256^3) on virtual ranks of one GPU, with a sphere split evenly like
    bench.py, for every exchange type (BUFFERED chunks are padded blocks; UNBUFFERED
    uses peer writes, which are never chunked): multi_transform of 2 transforms per
    rank, backward vs numpy, round trip."""
    import torch
    from spfft_amd.parallel import TorchDistComm, make_distributed, run_ranks  # noqa: F401
    from spfft_amd.utils.indices import distribute_sticks
    monkeypatch.setenv("SPFFT_EXCH_CHUNKS", str(chunks))
    monkeypatch.setenv("SPFFT_EXCH_STICK_BLOCKS", str(blocks))
    dims = (48, 40, 64)
    nx, ny, nz = dims
    gidx = sphere_indices(*dims, 0.5)
    parts = distribute_sticks(gidx, P, dims)
    planes = [nz // P + (1 if r < nz % P else 0) for r in range(P)]
    offsets = np.concatenate([[0], np.cumsum(planes)])
    rng = np.random.default_rng(88)
    vals = [_rand_vals(rng, len(gidx)) for _ in range(2)]
    refs = [dense_backward(gidx, v, dims) for v in vals]
    starts = np.concatenate([[0], np.cumsum([len(p) for p in parts])])
    max_sticks = max(len(np.unique(p[:, 0] * ny + p[:, 1])) for p in parts)

    def body(rank, comm):
        torch.cuda.set_device(0)
        ts = []
        for _ in range(2):
            g = sp.Grid(nx, ny, nz, max_sticks, GPU, 1, max_local_z_length=max(planes), comm=comm,
                        exchange_type=getattr(sp.ExchangeType, exchange))
            ts.append(g.create_transform(GPU, sp.TransformType.C2C, nx, ny, nz, planes[rank],
                                         parts[rank]))
        ins = [torch.as_tensor(v[starts[rank]:starts[rank + 1]], device="cuda") for v in vals]
        outs = sp.multi_transform_backward(ts, ins)
        e = max(max_rel_error(o.cpu().numpy(), r[offsets[rank]:offsets[rank + 1]])
                for o, r in zip(outs, refs))
        back = sp.multi_transform_forward(ts, scalings=[sp.Scaling.FULL] * 2)
        e2 = max(max_rel_error(b.cpu().numpy(), i.cpu().numpy()) for b, i in zip(back, ins))
        return max(e, e2)

    tol = 1e-5 if exchange.endswith("FLOAT") else 1e-11
    for e in run_ranks(P, body):
        assert e < tol


# ------------------------------------------------------------ RCCL data plane
# SPFFT_GPU_EXCHANGE=rccl on an in-process group: every exchange block of every
# virtual rank moves through RCCL (grouped ncclSend/ncclRecv to self on a size-1
# communicator per virtual rank, on the shared channel stream, with the real
# counts and displacements). RCCL refuses two ranks of one communicator on one
# device (profiles/r3/rccl_duplicate_device.txt), so this is how the RCCL data
# path runs on the one-GPU box.
@pytest.mark.parametrize("exchange,chunks,blocks", [
    ("COMPACT_BUFFERED", 1, 1), ("COMPACT_BUFFERED", 2, 1), ("COMPACT_BUFFERED", 4, 1),
    ("COMPACT_BUFFERED_FLOAT", 1, 1), ("COMPACT_BUFFERED_FLOAT", 3, 1), ("BUFFERED", 1, 1),
    ("BUFFERED", 2, 1), ("BUFFERED_FLOAT", 1, 1), ("UNBUFFERED", 1, 1), ("UNBUFFERED", 2, 1),
    ("COMPACT_BUFFERED", 2, 2), ("COMPACT_BUFFERED", 2, 4), ("BUFFERED", 2, 2),
    ("COMPACT_BUFFERED_FLOAT", 1, 2)])
@pytest.mark.parametrize("P", [3, 8])
def test_gpu_virtual_ranks_rccl(gpu, P, exchange, chunks, blocks, monkeypatch):
    import torch
    from spfft_amd.parallel import make_distributed, run_ranks
    from spfft_amd.utils.indices import distribute_sticks
    monkeypatch.setenv("SPFFT_GPU_EXCHANGE", "rccl")
    monkeypatch.setenv("SPFFT_EXCH_CHUNKS", str(chunks))
    monkeypatch.setenv("SPFFT_EXCH_STICK_BLOCKS", str(blocks))
    dims = (24, 20, 18) if P == 3 else (32, 28, 40)
    gidx = sphere_indices(*dims, 0.5)
    rng = np.random.default_rng(31 + P)
    vals = _rand_vals(rng, len(gidx))
    ref = dense_backward(gidx, vals, dims)
    parts = distribute_sticks(gidx, P, dims)
    tol = 1e-6 if exchange.endswith("FLOAT") else 1e-12
    ex = getattr(sp.ExchangeType, exchange)

    def body(rank, comm):
        torch.cuda.set_device(0)
        s = make_distributed(comm, dims, gidx, processing_unit=GPU, exchange_type=ex)
        plane = s.grid.data_plane
        start = sum(len(p) for p in parts[:rank])
        v = torch.as_tensor(vals[start:start + len(s.indices)], device="cuda")
        errs = []
        for _ in range(2):  # run twice: stale or missing blocks show up
            out = s.transform.backward(v).cpu().numpy()
            errs.append(max_rel_error(out, ref[s.z_offset:s.z_offset + s.z_length]))
            f = s.transform.forward(None, scaling=sp.Scaling.FULL).cpu().numpy()
            errs.append(max_rel_error(f, v.cpu().numpy()))
        return plane, max(errs)

    for plane, e in run_ranks(P, body):
        assert plane == "rccl-self"
        assert e < tol


def test_rccl_channel_shared_across_grids(gpu, monkeypatch):
    """Grids of one rank share one RCCL communicator: 3 grids per virtual rank
    (multi_transform of 3 transforms) create one communicator per rank, not 3."""
    import torch
    from spfft_amd.parallel import run_ranks
    from spfft_amd.utils.indices import distribute_sticks
    monkeypatch.setenv("SPFFT_GPU_EXCHANGE", "rccl")
    dims = (20, 16, 12)
    nx, ny, nz = dims
    P = 2
    gidx = sphere_indices(*dims, 0.5)
    parts = distribute_sticks(gidx, P, dims)
    planes = [nz // P] * P
    rng = np.random.default_rng(5)
    vals = [_rand_vals(rng, len(gidx)) for _ in range(3)]
    refs = [dense_backward(gidx, v, dims) for v in vals]
    starts = np.concatenate([[0], np.cumsum([len(p) for p in parts])])
    max_sticks = max(len(np.unique(p[:, 0] * ny + p[:, 1])) for p in parts)
    import gc
    gc.collect()  # grids of earlier tests release their channels
    before = sp.rccl_communicators()

    def body(rank, comm):
        torch.cuda.set_device(0)
        ts = []
        for _ in range(3):
            g = sp.Grid(nx, ny, nz, max_sticks, GPU, 1, max_local_z_length=max(planes), comm=comm,
                        exchange_type=sp.ExchangeType.COMPACT_BUFFERED)
            ts.append(g.create_transform(GPU, sp.TransformType.C2C, nx, ny, nz, planes[rank],
                                         parts[rank]))
        ins = [torch.as_tensor(v[starts[rank]:starts[rank + 1]], device="cuda") for v in vals]
        outs = sp.multi_transform_backward(ts, ins)
        z0 = rank * planes[0]
        e = max(max_rel_error(o.cpu().numpy(), r[z0:z0 + planes[rank]]) for o, r in zip(outs, refs))
        back = sp.multi_transform_forward(ts, scalings=[sp.Scaling.FULL] * 3)
        e2 = max(max_rel_error(b.cpu().numpy(), i.cpu().numpy()) for b, i in zip(back, ins))
        return max(e, e2)

    for e in run_ranks(P, body):
        assert e < 1e-12
    # one per virtual rank (fewer if an earlier test's channel is still alive), not 3P
    assert 0 <= sp.rccl_communicators() - before <= P


def test_rccl_abort_is_reported(gpu):
    """Failure detection on the RCCL plane: the 2nd exchange aborts the communicator
    (ncclCommAbort on a live RCCL communicator, fault injection EXCHANGE_ABORT=2 of the
    testing library); that call and every later exchange raise MPIError instead of
    hanging (tools/fault_rccl_abort.py, in its own process)."""
    import subprocess
    import sys
    from conftest import TESTING_ENV
    e = dict(os.environ, **TESTING_ENV)
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "fault_rccl_abort.py")], cwd=REPO, env=e,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ABORT OK" in r.stdout, (r.stdout + r.stderr)[-4000:]


@pytest.mark.parametrize("ttype", ["c2c", "r2c"])
@pytest.mark.parametrize("single", [False, True])
def test_capped_intermediate(gpu, ttype, single, monkeypatch):
    """SPFFT_INTER_BYTES caps the grid's [z][column][y] intermediate (large-grid
    memory mode): the y/x stages run over plane ranges that reuse it. 5 planes of
    room for a 21-plane slab: ranges of 5, 5, 5, 5, 1 planes."""
    import torch
    dims = (24, 20, 21)
    nx, ny, nz = dims
    esize = 8 if single else 16
    monkeypatch.setenv("SPFFT_INTER_BYTES", str(5 * nx * (ny + 8) * esize))
    rng = np.random.default_rng(77)
    r2c = ttype == "r2c"
    idx = create_value_indices(rng, [1.0], 0.8, 0.8, nx, ny, nz, r2c)[0]
    G = sp.GridFloat if single else sp.Grid
    grid = G(nx, ny, nz, nx * ny, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.R2C if r2c else sp.TransformType.C2C,
                              nx, ny, nz, nz, idx)
    tol = 1e-4 if single else 1e-11
    cdt = torch.complex64 if single else torch.complex128
    space = rng.standard_normal((nz, ny, nx))
    if not r2c:
        space = space + 1j * rng.standard_normal((nz, ny, nx))
    rdt = torch.float32 if single else torch.float64
    f = t.forward(torch.as_tensor(space, device=gpu, dtype=rdt if r2c else cdt))
    assert max_rel_error(f.cpu().numpy(), dense_forward(space, idx, dims, r2c=r2c)) < tol
    b = t.backward(f)
    ref = dense_backward(idx, f.cpu().numpy().astype(np.complex128), dims, r2c=r2c)
    assert max_rel_error(b.cpu().numpy(), ref) < tol


@pytest.mark.parametrize("exchange,chunks", [("COMPACT_BUFFERED", 1), ("COMPACT_BUFFERED", 2),
                                             ("BUFFERED", 2), ("UNBUFFERED", 1)])
def test_capped_intermediate_distributed(gpu, exchange, chunks, monkeypatch):
    """Capped intermediate on 3 virtual ranks, inside the pipelined exchange chunks."""
    import torch
    from spfft_amd.parallel import make_distributed, run_ranks
    from spfft_amd.utils.indices import distribute_sticks
    monkeypatch.setenv("SPFFT_EXCH_CHUNKS", str(chunks))
    dims = (24, 20, 30)
    nx, ny, nz = dims
    monkeypatch.setenv("SPFFT_INTER_BYTES", str(3 * nx * (ny + 8) * 16))
    gidx = sphere_indices(*dims, 0.5)
    rng = np.random.default_rng(78)
    vals = _rand_vals(rng, len(gidx))
    ref = dense_backward(gidx, vals, dims)
    P = 3
    parts = distribute_sticks(gidx, P, dims)

    def body(rank, comm):
        torch.cuda.set_device(0)
        s = make_distributed(comm, dims, gidx, processing_unit=GPU,
                             exchange_type=getattr(sp.ExchangeType, exchange))
        start = sum(len(p) for p in parts[:rank])
        v = torch.as_tensor(vals[start:start + len(s.indices)], device="cuda")
        out = s.transform.backward(v).cpu().numpy()
        e1 = max_rel_error(out, ref[s.z_offset:s.z_offset + s.z_length])
        f = s.transform.forward(None, scaling=sp.Scaling.FULL).cpu().numpy()
        return max(e1, max_rel_error(f, v.cpu().numpy()))

    for e in run_ranks(P, body):
        assert e < 1e-11


# ------------------------------------------------------------- long lines
# Axes beyond one workgroup's LDS run the global four-step engine (6144 = 64 x 96,
# 8192 = 64 x 128, 12288) or Bluestein over it (the prime 4099: m = 16384 = 128 x 128),
# fp64 and fp32, on the z, y and x axes, C2C and R2C (packed-real long x for even
# lengths, hermitian-extended complex rows for odd ones).
@pytest.mark.parametrize("dims,ttype,single", [
    ((6, 5, 6144), "c2c", False), ((4, 6, 8192), "c2c", False), ((5, 4, 4099), "c2c", False),
    ((6144, 4, 6), "c2c", False), ((8192, 3, 5), "c2c", False), ((4099, 4, 5), "c2c", False),
    ((4, 6144, 5), "c2c", False), ((5, 4099, 4), "c2c", False),
    ((4, 5, 12288), "c2c", True), ((5, 4, 4099), "c2c", True), ((12288, 3, 4), "c2c", True),
    ((4099, 3, 4), "c2c", True), ((3, 4099, 4), "c2c", True),
    ((12288, 4, 5), "r2c", False), ((4099, 4, 5), "r2c", False), ((6, 5, 6144), "r2c", False),
    ((4, 4099, 5), "r2c", False), ((24576, 3, 4), "r2c", True), ((4099, 3, 4), "r2c", True),
    # fp32 8192 fits one workgroup's LDS as a line but not next to the x stage's column
    # table; 4096 / 2048 on the line-fast axes take the four-step (one-line run-time
    # workgroups); z at 4096 stays in LDS
    ((8192, 3, 4), "c2c", True), ((4, 8192, 3), "c2c", True), ((4096, 4, 5), "c2c", False),
    ((4, 2048, 5), "c2c", False), ((4096, 3, 4), "r2c", True), ((6, 4, 4096), "c2c", True),
])
def test_long_lines_any_length(gpu, dims, ttype, single):
    import torch
    rng = np.random.default_rng(4099)
    nx, ny, nz = dims
    r2c = ttype == "r2c"
    idx = create_value_indices(rng, [1.0], 0.8, 0.7, nx, ny, nz, r2c)[0]
    G = sp.GridFloat if single else sp.Grid
    grid = G(nx, ny, nz, nx * ny, GPU, 1)
    t = grid.create_transform(GPU, sp.TransformType.R2C if r2c else sp.TransformType.C2C,
                              nx, ny, nz, nz, idx)
    tol = 2e-5 if single else 1e-12
    cdt = torch.complex64 if single else torch.complex128
    rdt = torch.float32 if single else torch.float64
    space = rng.standard_normal((nz, ny, nx))
    if not r2c:
        space = space + 1j * rng.standard_normal((nz, ny, nx))
    f = t.forward(torch.as_tensor(space, device=gpu, dtype=rdt if r2c else cdt))
    assert max_rel_error(f.cpu().numpy(), dense_forward(space, idx, dims, r2c=r2c)) < tol
    vals = f.cpu().numpy().astype(np.complex128)
    b = t.backward(f)
    assert max_rel_error(b.cpu().numpy(), dense_backward(idx, vals, dims, r2c=r2c)) < tol


@pytest.mark.parametrize("dims,ttype,exchange,chunks", [
    ((4, 5, 6144), "c2c", "COMPACT_BUFFERED", 1), ((4, 5, 6144), "c2c", "BUFFERED", 2),
    ((5, 2048, 4), "c2c", "COMPACT_BUFFERED", 2), ((5, 2048, 4), "r2c", "COMPACT_BUFFERED", 1),
    ((4096, 4, 6), "c2c", "COMPACT_BUFFERED_FLOAT", 2), ((4096, 4, 6), "r2c", "BUFFERED", 1),
    ((4, 4099, 5), "r2c", "COMPACT_BUFFERED", 2), ((5, 4, 4099), "c2c", "UNBUFFERED", 1)])
def test_long_lines_distributed(gpu, dims, ttype, exchange, chunks, monkeypatch):
    """Four-step axes on P = 2 virtual ranks: the fused long-line IO through the
    exchange layouts (z: per-rank segments; y: the received column entries, chunked;
    x: the column tables), against the dense numpy oracle."""
    import torch
    from spfft_amd.parallel import run_ranks
    from spfft_amd.utils.indices import calculate_num_local_xy_planes
    monkeypatch.setenv("SPFFT_EXCH_CHUNKS", str(chunks))
    nx, ny, nz = dims
    P = 2
    r2c = ttype == "r2c"
    rng = np.random.default_rng(6144)
    parts = create_value_indices(rng, [1, 1], 0.8, 0.7, nx, ny, nz, r2c)
    planes = [calculate_num_local_xy_planes(r, nz, [1, 1]) for r in range(P)]
    offsets = np.concatenate([[0], np.cumsum(planes)])
    all_idx = np.concatenate(parts)
    space = rng.standard_normal((nz, ny, nx))
    field = space if r2c else space + 1j * rng.standard_normal((nz, ny, nx))
    vals_all = dense_forward(field, all_idx, dims, r2c=r2c)
    ref = dense_backward(all_idx, vals_all, dims, r2c=r2c)
    starts = np.concatenate([[0], np.cumsum([len(p) for p in parts])])
    ttype_e = sp.TransformType.R2C if r2c else sp.TransformType.C2C
    max_sticks = max(len(np.unique(p[:, 0] * ny + p[:, 1])) if len(p) else 0 for p in parts)

    def body(rank, comm):
        torch.cuda.set_device(0)
        grid = sp.Grid(nx, ny, nz, max(1, max_sticks), GPU, 1, max_local_z_length=max(planes),
                       comm=comm, exchange_type=getattr(sp.ExchangeType, exchange))
        t = grid.create_transform(GPU, ttype_e, nx, ny, nz, planes[rank], parts[rank])
        v = torch.as_tensor(vals_all[starts[rank]:starts[rank + 1]], device="cuda")
        out = t.backward(v).cpu().numpy()
        e = max_rel_error(out, ref[offsets[rank]:offsets[rank + 1]]) if planes[rank] else 0.0
        slab = torch.as_tensor(np.ascontiguousarray(field[offsets[rank]:offsets[rank + 1]]),
                               device="cuda")
        f = t.forward(slab).cpu().numpy()
        return max(e, max_rel_error(f, vals_all[starts[rank]:starts[rank + 1]]) if len(f) else 0.0)

    tol = 2e-5 if exchange.endswith("FLOAT") else 1e-11
    for e in run_ranks(P, body):
        assert e < tol


def test_grid_device_footprint(gpu):
    """Grid memory (tools/memory_model.py): stick side (dimZ + 32) x maxSticks, slab
    side sum(maxSticks) x maxLocalZ (distributed only), space maxX (maxY + 32) maxLocalZ,
    intermediate min(that, 2 GiB); complex elements. A local 64^3 grid with a sphere's
    sticks holds ~1.8 slabs, 4 virtual ranks ~2.6 slabs each."""
    import torch
    from spfft_amd.parallel import run_ranks
    n = 64
    sticks = 3217
    g = sp.Grid(n, n, n, sticks, GPU, 1)
    plane = n * (n + 32) * n
    assert g.device_bytes == 16 * ((n + 32) * sticks + 2 * plane)
    P = 4

    def body(rank, comm):
        torch.cuda.set_device(0)
        gd = sp.Grid(n, n, n, sticks // P + 1, GPU, 1, max_local_z_length=n // P, comm=comm,
                     exchange_type=sp.ExchangeType.COMPACT_BUFFERED)
        pl = n * (n + 32) * (n // P)
        want = 16 * ((n + 32) * (sticks // P + 1) + P * (sticks // P + 1) * (n // P) + 2 * pl)
        return gd.device_bytes, want

    for got, want in run_ranks(P, body):
        assert got == want


def test_peer_write_offsets_both_signs(gpu, monkeypatch, capfd):
    """Peer-write plans address the peers' buffers as signed element offsets from the
    local ones (round 2's y base table dropped negative ones). Three virtual ranks
    allocate in rank order, so rank 0 sees positive and rank 2 negative offsets; the
    transform must be exact with both (SPFFT_LOG prints each plan's offset range)."""
    import re
    import torch
    from spfft_amd.parallel import make_distributed, run_ranks
    from spfft_amd.utils.indices import distribute_sticks
    monkeypatch.setenv("SPFFT_LOG", "1")
    dims = (20, 18, 16)
    gidx = sphere_indices(*dims, 0.5)
    rng = np.random.default_rng(2)
    vals = _rand_vals(rng, len(gidx))
    ref = dense_backward(gidx, vals, dims)
    parts = distribute_sticks(gidx, 3, dims)

    def body(rank, comm):
        torch.cuda.set_device(0)
        s = make_distributed(comm, dims, gidx, processing_unit=GPU,
                             exchange_type=sp.ExchangeType.UNBUFFERED)
        start = sum(len(p) for p in parts[:rank])
        v = torch.as_tensor(vals[start:start + len(s.indices)], device="cuda")
        e1 = max_rel_error(s.transform.backward(v).cpu().numpy(),
                           ref[s.z_offset:s.z_offset + s.z_length])
        e2 = max_rel_error(s.transform.forward(None, scaling=sp.Scaling.FULL).cpu().numpy(),
                           v.cpu().numpy())
        return max(e1, e2)

    for e in run_ranks(3, body):
        assert e < 1e-12
    err = capfd.readouterr().err
    ranges = [(int(a), int(b)) for a, b in re.findall(r"peer_offsets=\[(-?\d+), (-?\d+)\]", err)]
    assert len(ranges) == 3, err[-2000:]
    assert min(r[0] for r in ranges) < 0 < max(r[1] for r in ranges), ranges


@pytest.mark.parametrize("single", [False, True])
def test_grid_host_and_gpu(gpu, single):
    """A grid created with SPFFT_PU_HOST | SPFFT_PU_GPU holds both memories and serves a
    HOST transform and a GPU transform (reference: grid_internal.cpp:60-77,
    transform_internal.cpp:69-77); both match the dense oracle, and the GPU transform's
    host-located output matches too."""
    import torch
    dims = (24, 20, 18)
    nx, ny, nz = dims
    rng = np.random.default_rng(11)
    idx = create_value_indices(rng, [1.0], 0.6, 0.8, nx, ny, nz, False)[0]
    vals = rng.standard_normal(len(idx)) + 1j * rng.standard_normal(len(idx))
    ref = dense_backward(idx, vals, dims)
    G = sp.GridFloat if single else sp.Grid
    cdt = np.complex64 if single else np.complex128
    tol = 2e-5 if single else 1e-12
    both = int(sp.ProcessingUnit.HOST) | int(sp.ProcessingUnit.GPU)
    grid = G(nx, ny, nz, nx * ny, both, 2)
    th = grid.create_transform(sp.ProcessingUnit.HOST, sp.TransformType.C2C, nx, ny, nz, nz, idx)
    tg = grid.create_transform(sp.ProcessingUnit.GPU, sp.TransformType.C2C, nx, ny, nz, nz, idx)
    v = vals.astype(cdt)
    assert max_rel_error(np.array(th.backward(v)), ref) < tol
    out = tg.backward(torch.as_tensor(v, device="cuda"))
    torch.cuda.synchronize()
    assert max_rel_error(out.cpu().numpy(), ref) < tol
    # GPU transform, output in host memory
    hout = tg.backward(torch.as_tensor(v, device="cuda"), output_location=sp.ProcessingUnit.HOST)
    assert max_rel_error(np.array(hout), ref) < tol
    # forward of both from their own space domains
    space = (rng.standard_normal((nz, ny, nx)) + 1j * rng.standard_normal((nz, ny, nx))).astype(cdt)
    fref = dense_forward(space.astype(np.complex128), idx, dims)
    assert max_rel_error(np.array(th.forward(space)), fref) < tol * 10
    fg = tg.forward(torch.as_tensor(space, device="cuda"))
    torch.cuda.synchronize()
    assert max_rel_error(fg.cpu().numpy(), fref) < tol * 10

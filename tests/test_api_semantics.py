"""API semantics and error contract of SURVEY.md §7.7 (reference:
src/spfft/grid_internal.cpp:47-229, transform_internal.cpp:52-83,
compression/indices.hpp:49-186, parameters.cpp:95-109,
multi_transform_internal.hpp:53-59), checked on the host engine, plus the
distributed checks on in-process rank groups."""
import numpy as np
import pytest

import spfft_amd as sp
from spfft_amd.parallel import run_ranks
from spfft_amd.utils.indices import create_value_indices, sphere_indices
from spfft_amd.utils.oracle import dense_backward, dense_forward, max_rel_error

HOST = sp.ProcessingUnit.HOST
C2C, R2C = sp.TransformType.C2C, sp.TransformType.R2C


def _idx(nx, ny, nz, r2c=False, seed=0):
    return create_value_indices(np.random.default_rng(seed), [1.0], 0.8, 0.8, nx, ny, nz, r2c)[0]


# ---------------------------------------------------------------- Grid
@pytest.mark.parametrize("args", [(0, 4, 4, 16), (4, -1, 4, 16), (4, 4, 0, 16), (4, 4, 4, -1)])
def test_grid_invalid_dims(args):
    with pytest.raises(sp.InvalidParameterError):
        sp.Grid(*args, HOST, 1)


def test_grid_invalid_processing_unit():
    with pytest.raises(sp.InvalidParameterError):
        sp.Grid(4, 4, 4, 16, sp.ProcessingUnit(1) & 0 or 4, 1)


def test_grid_getters_and_threads_default():
    g = sp.Grid(8, 6, 4, 20, HOST, -1)
    assert (g.max_dim_x, g.max_dim_y, g.max_dim_z) == (8, 6, 4)
    assert g.max_num_local_z_columns == 20
    assert g.max_local_z_length == 4
    assert g.processing_unit == HOST
    assert g.num_threads >= 1  # < 1 -> runtime default (reference: grid_internal.cpp:69-72)


# ----------------------------------------------------------- Transform
def test_transform_dims_exceed_grid():
    g = sp.Grid(8, 8, 8, 64, HOST, 1)
    with pytest.raises(sp.InvalidParameterError):
        g.create_transform(HOST, C2C, 9, 8, 8, 8, _idx(8, 8, 8))


def test_local_grid_requires_full_z():
    g = sp.Grid(8, 8, 8, 64, HOST, 1)
    with pytest.raises(sp.InvalidParameterError):
        g.create_transform(HOST, C2C, 8, 8, 8, 7, _idx(8, 8, 8))


def test_too_many_sticks_for_grid():
    g = sp.Grid(8, 8, 8, 3, HOST, 1)
    with pytest.raises(sp.InvalidParameterError):
        g.create_transform(HOST, C2C, 8, 8, 8, 8, _idx(8, 8, 8))


def test_gpu_transform_on_host_grid():
    g = sp.Grid(8, 8, 8, 64, HOST, 1)
    with pytest.raises(sp.SpfftError):
        g.create_transform(sp.ProcessingUnit.GPU, C2C, 8, 8, 8, 8, _idx(8, 8, 8))


def test_host_transform_rejects_gpu_location():
    g = sp.Grid(8, 8, 8, 64, HOST, 1)
    idx = _idx(8, 8, 8)
    t = g.create_transform(HOST, C2C, 8, 8, 8, 8, idx)
    with pytest.raises(sp.InvalidParameterError):
        t.backward(np.zeros(len(idx), np.complex128), sp.ProcessingUnit.GPU)


@pytest.mark.parametrize("bad", [(8, 0, 0), (0, 8, 0), (0, 0, 8), (-5, 0, 0)])
def test_out_of_bounds_indices(bad):
    g = sp.Grid(8, 8, 8, 64, HOST, 1)
    idx = np.array([[0, 0, 0], list(bad)], dtype=np.int32)
    with pytest.raises(sp.InvalidIndicesError):
        g.create_transform(HOST, C2C, 8, 8, 8, 8, idx)


def test_duplicate_triplets_within_rank():
    """As in the reference (duplicates are checked per stick across ranks only,
    compression/indices.hpp:105-117), a repeated triplet within one rank is accepted
    and both output slots receive that frequency's value."""
    g = sp.Grid(8, 8, 8, 64, HOST, 1)
    idx = np.array([[1, 2, 3], [1, 2, 3], [0, 0, 0]], dtype=np.int32)
    t = g.create_transform(HOST, C2C, 8, 8, 8, 8, idx)
    rng = np.random.default_rng(0)
    space = rng.standard_normal((8, 8, 8)) + 1j * rng.standard_normal((8, 8, 8))
    f = np.array(t.forward(space))
    assert f[0] == f[1]


def test_r2c_rejects_negative_x():
    g = sp.Grid(8, 8, 8, 64, HOST, 1)
    idx = np.array([[-1, 0, 0]], dtype=np.int32)
    with pytest.raises(sp.InvalidIndicesError):
        g.create_transform(HOST, R2C, 8, 8, 8, 8, idx)


def test_centered_mode_triggered_by_any_negative_index():
    """One negative index switches the whole set to centred interpretation, so an index
    valid only in shifted mode (x = 6 of 8) becomes invalid."""
    g = sp.Grid(8, 8, 8, 64, HOST, 1)
    idx = np.array([[6, 0, 0], [0, -1, 0]], dtype=np.int32)
    with pytest.raises(sp.InvalidIndicesError):
        g.create_transform(HOST, C2C, 8, 8, 8, 8, idx)


def test_transform_getters_and_clone():
    nx, ny, nz = 10, 9, 8
    idx = _idx(nx, ny, nz)
    g = sp.Grid(nx, ny, nz, nx * ny, HOST, 2)
    t = g.create_transform(HOST, C2C, nx, ny, nz, nz, idx)
    assert (t.dim_x, t.dim_y, t.dim_z) == (nx, ny, nz)
    assert t.local_z_length == nz and t.local_z_offset == 0
    assert t.local_slice_size == nx * ny * nz
    assert t.global_size == nx * ny * nz
    assert t.num_local_elements == len(idx) == t.num_global_elements
    assert t.type == C2C and t.processing_unit == HOST
    c = t.clone()  # deep copy with a new grid: independent space domain
    rng = np.random.default_rng(1)
    v = rng.standard_normal(len(idx)) + 1j * rng.standard_normal(len(idx))
    a = np.array(t.backward(v))
    b = np.array(c.backward(v))
    assert np.array_equal(a, b)
    c.backward(np.zeros_like(v))
    assert np.array_equal(np.array(t.space_domain(HOST)), a)


def test_transforms_share_grid_space_domain():
    """Transforms of one Grid share its memory (reference semantics)."""
    nx = ny = nz = 6
    idx = _idx(nx, ny, nz)
    g = sp.Grid(nx, ny, nz, nx * ny, HOST, 1)
    t1 = g.create_transform(HOST, C2C, nx, ny, nz, nz, idx)
    t2 = g.create_transform(HOST, C2C, nx, ny, nz, nz, idx)
    assert t1.space_domain_ptr(HOST) == t2.space_domain_ptr(HOST)


def test_multi_transform_rejects_shared_grid():
    nx = ny = nz = 6
    idx = _idx(nx, ny, nz)
    g = sp.Grid(nx, ny, nz, nx * ny, HOST, 1)
    t1 = g.create_transform(HOST, C2C, nx, ny, nz, nz, idx)
    t2 = g.create_transform(HOST, C2C, nx, ny, nz, nz, idx)
    v = np.zeros(len(idx), np.complex128)
    with pytest.raises(sp.InvalidParameterError):
        sp.multi_transform_backward([t1, t2], [v, v])


def test_multi_transform_reference_values():
    """Reference test_multi_transform.cpp: 3 transforms (grid + 2 clones), constant
    values (i, i); backward then unscaled forward gives (i N, i N)."""
    nx, ny, nz = 8, 7, 6
    idx = sphere_indices(nx, ny, nz, 0.5)
    g = sp.Grid(nx, ny, nz, nx * ny, HOST, 1)
    t0 = g.create_transform(HOST, C2C, nx, ny, nz, nz, idx)
    ts = [t0, t0.clone(), t0.clone()]
    vals = [np.full(len(idx), i + 1j * i, np.complex128) for i in range(3)]
    sp.multi_transform_backward(ts, vals)
    outs = sp.multi_transform_forward(ts)
    for i, o in enumerate(outs):
        assert np.allclose(o, (i + 1j * i) * nx * ny * nz, atol=1e-8)


def test_full_scaling_roundtrip_and_step_api():
    nx, ny, nz = 12, 10, 9
    idx = _idx(nx, ny, nz, seed=3)
    g = sp.Grid(nx, ny, nz, nx * ny, HOST, 2)
    t = g.create_transform(HOST, C2C, nx, ny, nz, nz, idx)
    rng = np.random.default_rng(2)
    v = rng.standard_normal(len(idx)) + 1j * rng.standard_normal(len(idx))
    t.backward(v)
    out = np.array(t.forward(None, scaling=sp.Scaling.FULL))
    assert max_rel_error(out, v) < 1e-13


@pytest.mark.parametrize("r2c", [False, True])
def test_host_poison_mode(r2c, monkeypatch):
    monkeypatch.setenv("SPFFT_POISON", "1")
    nx, ny, nz = 10, 8, 6
    idx = _idx(nx, ny, nz, r2c=r2c, seed=5)
    rng = np.random.default_rng(6)
    space = rng.standard_normal((nz, ny, nx))
    if not r2c:
        space = space + 1j * rng.standard_normal((nz, ny, nx))
    vals = dense_forward(space, idx, (nx, ny, nz), r2c=r2c)
    g = sp.Grid(nx, ny, nz, nx * ny, HOST, 1)
    t = g.create_transform(HOST, R2C if r2c else C2C, nx, ny, nz, nz, idx)
    out = np.array(t.backward(vals))
    assert not np.isnan(out).any()
    assert max_rel_error(out, dense_backward(idx, vals, (nx, ny, nz), r2c=r2c)) < 1e-12
    f = np.array(t.forward(space))
    assert not np.isnan(f).any()


# -------------------------------------------------- distributed contract
def _dist_grid(comm, nx, ny, nz, sticks, planes, exch=sp.ExchangeType.DEFAULT):
    return sp.Grid(nx, ny, nz, sticks, HOST, 1, max_local_z_length=planes, comm=comm,
                   exchange_type=exch)


def test_distributed_dims_mismatch():
    def body(rank, comm):
        g = _dist_grid(comm, 8, 8, 8, 64, 4)
        nx = 8 if rank == 0 else 6
        with pytest.raises(sp.MPIParameterMismatchError):
            g.create_transform(HOST, C2C, nx, 8, 8, 4, np.zeros((0, 3), np.int32))
    run_ranks(2, body)


def test_distributed_plane_sum_mismatch():
    def body(rank, comm):
        g = _dist_grid(comm, 8, 8, 8, 64, 8)
        with pytest.raises(sp.MPIParameterMismatchError):
            g.create_transform(HOST, C2C, 8, 8, 8, 3, np.zeros((0, 3), np.int32))
    run_ranks(2, body)


def test_distributed_duplicate_sticks_across_ranks():
    def body(rank, comm):
        g = _dist_grid(comm, 8, 8, 8, 64, 4)
        idx = np.array([[1, 1, rank]], dtype=np.int32)  # same stick (1,1) on both ranks
        with pytest.raises(sp.DuplicateIndicesError):
            g.create_transform(HOST, C2C, 8, 8, 8, 4, idx)
    run_ranks(2, body)


def test_distributed_exchange_type_mismatch():
    def body(rank, comm):
        exch = sp.ExchangeType.BUFFERED if rank == 0 else sp.ExchangeType.UNBUFFERED
        with pytest.raises(sp.MPIParameterMismatchError):
            _dist_grid(comm, 8, 8, 8, 64, 4, exch)
    run_ranks(2, body)


def test_distributed_errors_do_not_hang_other_ranks():
    """An invalid index on one rank fails every rank (agreement by allgather)."""
    def body(rank, comm):
        g = _dist_grid(comm, 8, 8, 8, 64, 4)
        idx = np.array([[0, 0, 9 if rank == 1 else 0]], dtype=np.int32)
        with pytest.raises(sp.SpfftError):
            g.create_transform(HOST, C2C, 8, 8, 8, 4, idx)
    run_ranks(2, body)


def test_default_exchange_is_compact():
    def body(rank, comm):
        g = _dist_grid(comm, 8, 8, 8, 64, 4)
        return g.exchange_type
    assert run_ranks(2, body) == [sp.ExchangeType.COMPACT_BUFFERED] * 2


def test_bench_model_relay_shares():
    """bench.py's exchange model (config.model_ms): link time of a direct exchange,
    and of the relay plane, whose shares cut every link's load to (N-1)/(N-1+K) in
    two hops."""
    import importlib.util
    import os
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench", os.path.join(repo, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    stages = {"backward": {"z": 0.07, "y+x": 0.18, "exchange": 0.7, "total": 0.95},
              "forward": {"x+y": 0.17, "z": 0.06, "exchange": 0.7, "total": 0.93}}
    direct = b._model(stages, 52.7e6, 2, 1, 1)
    relay = b._model(stages, 52.7e6, 2, 1, 1, relays=6)
    assert abs(direct["backward"]["link_ms"] - 52.7e6 / 70e9 * 1e3) < 1e-9
    assert abs(relay["backward"]["link_ms"] - 2 * direct["backward"]["link_ms"] / 7 - b.RELAY_BARRIER_MS) < 1e-9
    assert direct["backward"]["bound"] == "link" and relay["relay_gpus"] == 6
    assert abs(direct["backward"]["compute_ms"] - 0.25) < 1e-12
    # pipelined grid: all but one step's compute hidden behind the link
    piped = b._model(stages, 52.7e6, 2, 2, 2)
    assert abs(piped["backward"]["predicted_ms"] - (direct["backward"]["link_ms"] + 0.25 / 4)) < 1e-9
    # a measured link rate replaces the assumption
    meas = b._model(stages, 52.7e6, 2, 1, 1, link_gbps=50.0)
    assert meas["link_GBps_source"] == "measured"
    assert abs(meas["backward"]["link_ms"] - 52.7e6 / 50e9 * 1e3) < 1e-9
    # the pipelined relay: shares, two hops, overlap
    rp = b._model(stages, 52.7e6, 2, 4, 2, relays=6)
    assert abs(rp["forward"]["predicted_ms"] - (max(rp["forward"]["link_ms"], 0.23) + 0.23 / 8)) < 1e-9


def test_release_library_has_no_test_hooks():
    """The release library exports no test probe and reads no fault-injection switch;
    both live in the testing library only (CMake SPFFT_TESTING_LIBRARY,
    src/core/fault.hpp, src/testing/)."""
    import os
    import shutil
    import subprocess
    from conftest import TESTING_LIB
    from spfft_amd.ops._lib import NATIVE_DIR
    rel = os.path.join(NATIVE_DIR, "libspfft_amd.so")
    nm = shutil.which("nm") or "/usr/bin/nm"
    syms = subprocess.run([nm, "-D", "--defined-only", rel], capture_output=True, text=True, check=True).stdout
    assert "spfft_amd_test_" not in syms and "shm_check" not in syms
    with open(rel, "rb") as f:
        assert b"SPFFT_FAULT_" not in f.read()
    tsyms = subprocess.run([nm, "-D", "--defined-only", TESTING_LIB], capture_output=True, text=True,
                           check=True).stdout
    assert "spfft_amd_test_comm_shm_check" in tsyms and "spfft_amd_test_fault_injection" in tsyms


def test_stage_kernels_keep_nt_hints():
    """The z/y stage kernels' stick-side accesses keep the cache policy they were
    written with in the built gfx950 code: streaming (nt) stores in the z backward
    kernels unless instantiated Plain, nt stick stores in the y forward kernels. A
    run-time plain/nt branch had the compiler drop the hints (profiles/r6/ntmerge);
    tools/nt_audit.py reads the library's code objects."""
    import os
    import shutil
    import sys
    from spfft_amd.ops._lib import NATIVE_DIR
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import nt_audit
    if not shutil.which("objcopy") or not nt_audit._tool("clang-offload-bundler") or not nt_audit._tool("llvm-objdump"):
        pytest.skip("objcopy / clang-offload-bundler / llvm-objdump not available")
    lib = os.path.join(NATIVE_DIR, "libspfft_amd.so")
    res = nt_audit.audit(lib, r"(z_backward_desc|z_forward_desc|y_forward|y_backward)_kernel.*CtEngI[fd]Li(256|512)E",
                         needles=(b"z_backward_desc_kernel", b"y_forward_kernel"))
    zb = {k: c for k, c in res.items() if "z_backward_desc" in k}
    zf = {k: c for k, c in res.items() if "z_forward_desc" in k}
    yf = {k: c for k, c in res.items() if "y_forward" in k}
    yb = {k: c for k, c in res.items() if "y_backward" in k}
    assert len(zb) >= 8 and len(zf) >= 8 and len(yf) >= 4 and len(yb) >= 8, sorted(res)
    flag = lambda k: "Lb1EEEvT_" in k  # the trailing bool template argument (Plain / NtValues)
    for k, c in zb.items():
        assert c["st"] > 0 and c["st_nt"] == (0 if flag(k) else c["st"]), (k, c)
        assert c["ld_nt"] > 0, (k, c)  # streamed value loads
    for k, c in zf.items():
        assert c["st"] > 0 and c["st_nt"] == (c["st"] if flag(k) else 0), (k, c)
        assert c["ld_nt"] > 0, (k, c)  # streamed stick loads
    for k, c in yf.items():
        assert c["st"] > 0 and c["st_nt"] == c["st"], (k, c)
    for k, c in yb.items():
        if not flag(k):  # the Plain instantiation loads its sticks without the hint
            twin = yb[k.replace("Lb0EEEvT_", "Lb1EEEvT_")]
            assert c["ld_nt"] > twin["ld_nt"], (k, c, twin)


def test_bench_plane_choice(monkeypatch):
    """bench.py N > 1: the headline runs on the fastest probed plane that really ran
    as itself (a plane that fell back to another is no candidate); --plane forces one;
    plane switches set in the environment keep the library's own choice."""
    import importlib.util
    import os
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench", os.path.join(repo, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    for k in ("SPFFT_GPU_EXCHANGE", "SPFFT_RELAY"):
        monkeypatch.delenv(k, raising=False)
    probe = {"rccl": {"ms_per_step": 1.2, "plane": "rccl"},
             "ipc": {"ms_per_step": 0.9, "plane": "ipc"},
             "relay": {"ms_per_step": 0.5, "plane": "rccl"}}  # relay fell back to RCCL
    assert b._choose_plane("auto", probe)["plane"] == "ipc"
    assert b._choose_plane("rccl", probe)["plane"] == "rccl"
    assert b._choose_plane("auto", {"ipc": {"error": "MPIError"}})["plane"] == "default"
    assert b._choose_plane("auto", None)["plane"] == "default"
    monkeypatch.setenv("SPFFT_RELAY", "force")
    assert b._choose_plane("auto", probe)["plane"] == "default"
    assert b._plane_env("relay", True)["SPFFT_RELAY"] == "force"
    assert b._plane_env("relay", False)["SPFFT_RELAY"] == "auto"

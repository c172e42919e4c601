"""Runs the native (C/C++/Fortran) test programs and examples built by
spfft_amd.build: the C++ unit-test runner, the MPI test runner under
mpiexec with 1-4 ranks (reference: tests/CMakeLists.txt runs run_mpi_tests
with mpiexec -n 1..4), and the C, C++ and Fortran examples (reference:
examples/example.{c,cpp,f90}).

GPU sub-cases inside the native runners skip themselves when no device is
visible, so these tests are CPU-runnable; the GPU variant re-runs them on the
MI355X box.
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(REPO, "spfft_amd", "_native")
MPIEXEC = shutil.which("mpiexec") or "/opt/conda/bin/mpiexec"


def _prog(name):
    path = os.path.join(NATIVE, name)
    if not os.path.exists(path):
        pytest.skip(f"{name} not built")
    return path


def _run(cmd, timeout=600):
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "2")
    r = subprocess.run(cmd, cwd=NATIVE, env=env, capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    assert r.returncode == 0, f"{cmd} exited {r.returncode}:\n{out[-4000:]}"
    return out


def test_native_unit_tests():
    out = _run([_prog("spfft_native_tests")])
    assert " 0 failed" in out


@pytest.mark.parametrize("nranks", [1, 2, 3, 4])
def test_mpi_tests(nranks):
    prog = _prog("spfft_mpi_tests")
    if not os.path.exists(MPIEXEC):
        pytest.skip("mpiexec not available")
    out = _run([MPIEXEC, "-n", str(nranks), prog])
    assert " 0 failed" in out


@pytest.mark.parametrize("name", ["example_c", "example_cpp", "example_f90"])
def test_examples(name):
    out = _run([_prog(name)])
    assert out.strip()


@pytest.mark.gpu
def test_native_unit_tests_gpu(gpu):
    out = _run([_prog("spfft_native_tests")])
    assert " 0 failed" in out and "SKIP" not in out


@pytest.mark.gpu
@pytest.mark.parametrize("nranks", [1, 2, 3, 4])
def test_mpi_tests_gpu(gpu, nranks):
    """MPI front end with GPU grids (mpi_gpu_c2c runs every exchange type, mpi_gpu_churn
    every exchange and transform type with grids re-created per case and dropped by the
    ranks at different times): ranks share the box's GPU through the IPC peer-write
    plane, the production layout of plane-wave codes that run several ranks per GPU
    (reference: src/transpose/transpose_mpi_compact_buffered_gpu.cpp:195-219); nothing
    may be skipped."""
    prog = _prog("spfft_mpi_tests")
    if not os.path.exists(MPIEXEC):
        pytest.skip("mpiexec not available")
    out = _run([MPIEXEC, "-n", str(nranks), prog])
    assert " 0 failed" in out and "SKIP" not in out


def test_bench_cli_host(tmp_path):
    """C++ benchmark CLI (reference flags -d -r -o -m -s -t -e -p) on the host engine."""
    import json
    out = tmp_path / "b.json"
    _run([_prog("spfft_bench"), "-d", "24", "20", "18", "-r", "2", "-o", str(out), "-e", "all",
          "-p", "cpu", "--cutoff", "0.5", "-m", "2"])
    j = json.loads(out.read_text())
    assert [r["exchange"] for r in j["results"]] == ["buffered", "compact", "unbuffered"]
    assert all(r["transforms_per_second"] > 0 for r in j["results"])
    assert j["parameters"]["num_transforms"] == 2


def test_bench_cli_mpi_r2c(tmp_path):
    if not os.path.exists(MPIEXEC):
        pytest.skip("mpiexec not available")
    out = _run([MPIEXEC, "-n", "2", _prog("spfft_bench"), "-d", "20", "18", "16", "-r", "2",
                "-o", "", "-e", "compactFloat", "-p", "cpu", "-t", "r2c", "-s", "0.6"])
    assert "transforms/s" in out and "ranks: 2" in out


@pytest.mark.gpu
def test_bench_cli_gpu(gpu, tmp_path):
    import json
    out = tmp_path / "g.json"
    _run([_prog("spfft_bench"), "-d", "64", "64", "64", "-r", "5", "-o", str(out), "-e", "compact",
          "-p", "gpu-gpu", "--cutoff", "0.5"])
    j = json.loads(out.read_text())
    assert j["results"][0]["transforms_per_second"] > 0


def test_host_multi_transform_nonblocking_exchange_mpi(tmp_path):
    """Host multi_transform under mpiexec -n 2: each transform's exchange starts as an
    MPI_Ialltoallv (backward_exchange_start / forward_exchange_start) and completes in
    the next stage (exchange_wait), so the second transform's z / xy stage runs while
    the first one's exchange is in flight (reference:
    src/spfft/multi_transform_internal.hpp:61-94)."""
    import json
    if not os.path.exists(MPIEXEC):
        pytest.skip("mpiexec not available")
    out = tmp_path / "nb.json"
    _run([MPIEXEC, "-n", "2", _prog("spfft_bench"), "-d", "32", "30", "28", "-r", "3", "-m", "2",
          "-o", str(out), "-e", "compact", "-p", "cpu", "--cutoff", "0.5"])
    text = out.read_text()
    j = json.loads(text)
    assert j["results"][0]["transforms_per_second"] > 0
    for name in ("backward_exchange_start", "forward_exchange_start", "exchange_wait"):
        assert name in text, name


@pytest.mark.parametrize("nranks", [2, 3])
def test_host_unbuffered_alltoallw_mpi(tmp_path, nranks):
    """Host UNBUFFERED under mpiexec: the z stage keeps whole sticks and the exchange
    is one MPI_(I)alltoallw with hvector datatypes per peer (no pack or unpack pass;
    reference: src/transpose/transpose_mpi_unbuffered_host.cpp:66-181). The bench's
    timing tree shows the alltoallw scopes, non-blocking under multi_transform."""
    import json
    if not os.path.exists(MPIEXEC):
        pytest.skip("mpiexec not available")
    out = tmp_path / "unbuf.json"
    _run([MPIEXEC, "-n", str(nranks), _prog("spfft_bench"), "-d", "30", "28", "26", "-r", "3",
          "-m", "2", "-o", str(out), "-e", "unbuffered", "-p", "cpu", "--cutoff", "0.5"])
    text = out.read_text()
    j = json.loads(text)
    assert j["results"][0]["transforms_per_second"] > 0
    assert "alltoallw" in text
    assert "pack" not in text


@pytest.mark.gpu
def test_bench_cli_mpi_4ranks_shared_gpu(gpu, tmp_path):
    """Four MPI ranks on the box's one GPU (the several-ranks-per-GPU layout of
    plane-wave codes), every exchange type through the IPC peer-write plane, two
    transforms per step: the C++ benchmark's rates (profiles/r5/ipc/)."""
    import json
    if not os.path.exists(MPIEXEC):
        pytest.skip("mpiexec not available")
    out = tmp_path / "m4.json"
    _run([MPIEXEC, "-n", "4", _prog("spfft_bench"), "-d", "128", "128", "128", "-r", "10", "-m", "2",
          "-o", str(out), "-e", "all", "-p", "gpu-gpu", "--cutoff", "0.5"])
    j = json.loads(out.read_text())
    assert len(j["results"]) >= 3
    assert all(r["transforms_per_second"] > 0 for r in j["results"])
    # keep the record next to the profiles when asked (the GPU runs of the round)
    keep = os.environ.get("SPFFT_KEEP_BENCH")
    if keep:
        os.makedirs(os.path.dirname(keep), exist_ok=True)
        with open(keep, "w") as f:
            f.write(out.read_text())

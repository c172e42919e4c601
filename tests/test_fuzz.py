"""Randomised sweeps of tools/fuzz_gpu.py inside the suites: every engine path, type,
precision, 1-3 ranks with random distributions, every exchange type, centred indices
and multi_transform batches, against the dense numpy oracle."""
import importlib.util
import os

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fuzz():
    spec = importlib.util.spec_from_file_location("fuzz_gpu", os.path.join(REPO, "tools", "fuzz_gpu.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _sweep(host, cases, seed, max_elems):
    mod = _fuzz()
    rng = np.random.default_rng(seed)
    bad = []
    for c in range(cases):
        desc, err, tol = mod.run_case(rng, c, max_elems, host=host)
        if not err < tol:
            bad.append(f"{desc} err={err:.2e}")
    assert not bad, "\n".join(bad)


def test_fuzz_host():
    _sweep(True, 40, 2024, 1 << 17)


@pytest.mark.gpu
def test_fuzz_gpu(gpu):
    _sweep(False, 150, 2025, 1 << 20)


def _launch_dist(nproc, *args, env_extra=None):
    import subprocess
    import sys
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr=127.0.0.1",
           f"--nproc-per-node={nproc}", os.path.join(REPO, "tools", "fuzz_dist.py"), *args]
    env = dict(os.environ, OMP_NUM_THREADS="1", **(env_extra or {}))
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "passed" in out and "FAIL" not in out, out[-4000:]


def test_fuzz_dist_host_3ranks():
    """The random cases on three OS processes over torch.distributed (host engine)."""
    _launch_dist(3, "--host", "--cases", "20", "--seed", "31", "--max-elems", "65536")


@pytest.mark.gpu
def test_fuzz_dist_gpu_ipc_lazy_teardown(gpu):
    """Three processes sharing the GPU over the IPC peer-write plane, grids dropped
    lazily (each rank's previous grid lives until the next one exists). This is the
    sweep that failed in round 4 (seed 8: wrong results at cases 27/29, then a hang)."""
    _launch_dist(3, "--cases", "40", "--seed", "8")

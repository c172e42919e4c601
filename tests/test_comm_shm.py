"""Node-local shared-memory collectives (src/comm/shm_group.cpp), the host
synchronisation of the relay data plane: checked allgather + barrier rounds
against the communicator's own collectives, in-process and across processes."""
import json
import os
import re
import subprocess
import sys

from conftest import TESTING_ENV

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shm_collectives_threads():
    """4 in-process ranks (local group) through the testing library's probe."""
    code = ("from spfft_amd.parallel.comm import run_ranks\n"
            "res = run_ranks(4, lambda r, c: c.shm_check(500))\n"
            "assert all(s is not None and s > 0 and c > 0 for s, c in res), res\n"
            "print('THREADS OK')\n")
    e = dict(os.environ, OMP_NUM_THREADS="1", **TESTING_ENV)
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=e, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and "THREADS OK" in r.stdout, (r.stdout + r.stderr)[-4000:]


def test_shm_probe_absent_from_release_library():
    """The probe is not part of the release library's ABI."""
    code = ("from spfft_amd.parallel.comm import run_ranks\n"
            "try:\n"
            "    run_ranks(2, lambda r, c: c.shm_check(5))\n"
            "except Exception as e:\n"
            "    print('REFUSED', e)\n")
    e = {k: v for k, v in os.environ.items() if k != "SPFFT_AMD_LIBRARY"}
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=e, capture_output=True, text=True,
                       timeout=300)
    assert "REFUSED" in r.stdout and "testing library" in r.stdout, (r.stdout + r.stderr)[-4000:]


def _probe(nproc, env=None):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr=127.0.0.1",
           f"--nproc-per-node={nproc}", os.path.join(REPO, "tools", "shm_probe.py"), "--iters", "300"]
    e = dict(os.environ, OMP_NUM_THREADS="1", **TESTING_ENV, **(env or {}))
    r = subprocess.run(cmd, cwd=REPO, env=e, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    # (the ranks' lines may interleave on the shared pipe)
    found = dict(re.findall(r"SHM OK rank=(\d+) (\{[^}]*\})", r.stdout))
    assert len(found) == nproc, out[-4000:]
    return [json.loads(v) for v in found.values()]


def test_shm_collectives_processes():
    """3 processes over gloo: the shared segment carries the allgathers correctly
    (checked inside) and is faster than the gloo control plane."""
    for d in _probe(3):
        assert d["shm_us"] is not None and d["shm_us"] < d["comm_us"], d


def test_shm_collectives_disabled():
    for d in _probe(2, {"SPFFT_SHM_COLLECTIVES": "0"}):
        assert d["shm_us"] is None, d


def test_shm_segment_unlinked():
    """Nothing is left in /dev/shm after the processes end."""
    before = set(n for n in os.listdir("/dev/shm") if n.startswith("spfft-"))
    _probe(2)
    after = set(n for n in os.listdir("/dev/shm") if n.startswith("spfft-"))
    assert after <= before, after - before


def test_shm_peer_exit_detected():
    """A rank that leaves while the others wait in a shared-memory barrier: the
    waits end with an error naming the exited rank (liveness check), not a hang."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr=127.0.0.1",
           "--nproc-per-node=2", os.path.join(REPO, "tools", "shm_probe.py"), "--iters", "300"]
    e = dict(os.environ, OMP_NUM_THREADS="1", SPFFT_FAULT_SHM_EXIT="1", **TESTING_ENV)
    r = subprocess.run(cmd, cwd=REPO, env=e, capture_output=True, text=True, timeout=120)
    out = r.stdout + r.stderr
    assert "SHM ERROR rank=0" in out and "has exited" in out, out[-4000:]


def test_relay_skips_busy_gpus(tmp_path):
    """Idle-GPU relaying leases memory only on GPUs nothing else uses: the driver's
    mem_info_vram_used (sysfs, faked here) must show at most a few MiB; a GPU another
    process holds memory on, or whose usage is unknown, is not a relay candidate."""
    # (an idle MI355X reports 297766912 B: the driver's reservation)
    for pci, used in (("0000:05:00.0", 297766912), ("0000:26:00.0", 1545904128)):
        d = tmp_path / "bus" / "pci" / "devices" / pci
        d.mkdir(parents=True)
        (d / "mem_info_vram_used").write_text(f"{used}\n")
    code = ("import ctypes\n"
            "from spfft_amd.ops._lib import lib\n"
            "f = lib().spfft_amd_test_relay_candidate_idle\n"
            "f.argtypes = [ctypes.c_int] * 3\n"
            "print('IDLE', f(0, 0x05, 0), f(0, 0x26, 0), f(0, 0x45, 0))\n")
    e = dict(os.environ, SPFFT_SYSFS_ROOT=str(tmp_path), **TESTING_ENV)
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=e, capture_output=True, text=True,
                       timeout=120)
    assert "IDLE 1 0 0" in r.stdout, (r.stdout + r.stderr)[-4000:]


def test_shm_group_needs_one_pid_namespace():
    """Ranks that share /dev/shm from different pid namespaces cannot use the pid
    liveness check of the shared-memory waits: the group is not created on any rank
    (fault injection SHM_PIDNS: the last rank reports another namespace), and the
    plane falls back to the communicator's collectives."""
    for d in _probe(2, {"SPFFT_FAULT_SHM_PIDNS": "1"}):
        assert d["shm_us"] is None and d["comm_us"] > 0, d

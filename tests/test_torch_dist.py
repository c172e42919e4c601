"""Multi-process distributed transforms over torch.distributed (gloo control
plane, one OS process per rank), the same launch path bench.py uses.

CPU: host transforms, every exchange type, 2 and 3 ranks.
GPU: 2-4 ranks sharing the box's single MI355X. RCCL refuses two ranks of one
host on one device (profiles/r3/rccl_duplicate_device.txt): by default such
ranks move data with the IPC peer-write plane; with SPFFT_RCCL_VIRTUAL_HOSTS=1
every rank claims its own host id and the ranks run one multi-rank RCCL
communicator over RCCL's socket transport (test_torch_dist_rccl_multirank,
test_bench_driver_launch_2ranks_rccl). The RCCL initialisation-failure
agreement and fallback are covered by fault injection.
"""
import os
import socket
import subprocess
import sys

import pytest

from conftest import TESTING_ENV, TESTING_LIB

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(REPO, "tools", "rccl_probe.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(nproc, *args, timeout=300, expect=None):
    # standalone rendezvous: the launcher binds its own free port (a port picked
    # here and released could be taken again before the launcher binds it)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr=127.0.0.1",
           f"--nproc-per-node={nproc}", PROBE, *args]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert out.count(" OK") == nproc, out[-4000:]
    if expect:
        assert out.count(f"[{expect}]") == nproc, out[-4000:]


@pytest.mark.parametrize("exchange", ["COMPACT_BUFFERED", "COMPACT_BUFFERED_FLOAT", "BUFFERED",
                                      "BUFFERED_FLOAT", "UNBUFFERED"])
def test_torch_dist_host(exchange):
    _launch(2, exchange, "--host")


def test_torch_dist_host_3ranks():
    _launch(3, "COMPACT_BUFFERED", "--host")


# Ranks sharing the box's single GPU: RCCL refuses duplicate devices, so the
# library picks the IPC peer-write data plane (stage kernels store into the
# other processes' exchange buffers; stream-ordered barrier kernels).
@pytest.mark.gpu
@pytest.mark.parametrize("exchange", ["COMPACT_BUFFERED", "BUFFERED_FLOAT", "UNBUFFERED",
                                      "COMPACT_BUFFERED_FLOAT", "BUFFERED"])
def test_torch_dist_ipc_shared_gpu(gpu, exchange):
    _launch(2, exchange, "--iters=4", expect="ipc")


@pytest.mark.gpu
def test_torch_dist_ipc_3ranks_repeated(gpu):
    # many back-to-back transforms with fresh data: a stale read of an earlier
    # exchange (missing barrier / visibility) shows as a mismatch
    _launch(3, "UNBUFFERED", "--iters=12", "--dims=64,60,48", expect="ipc")


# Ranks sharing the box's single GPU through ONE multi-rank RCCL communicator:
# SPFFT_RCCL_VIRTUAL_HOSTS=1 gives every rank a host id of its own (RCCL's
# duplicate-device check is per host), so the ranks talk over RCCL's socket
# transport on loopback. This runs RcclDeviceComm, the class that moves the
# data between distinct GPUs on an 8-GPU node (peer ids, staggered send/recv
# order, grouped calls, channel stream hand-offs), through the pipelined 2D
# grid of stick blocks x plane chunks.
@pytest.mark.gpu
@pytest.mark.parametrize("nproc,exchange,chunks,blocks", [
    (2, "COMPACT_BUFFERED", 1, 1), (2, "COMPACT_BUFFERED", 2, 2), (3, "BUFFERED_FLOAT", 1, 1),
    (3, "COMPACT_BUFFERED_FLOAT", 4, 2), (4, "BUFFERED", 2, 2), (4, "COMPACT_BUFFERED", 1, 3)])
def test_torch_dist_rccl_multirank(gpu, monkeypatch, nproc, exchange, chunks, blocks):
    monkeypatch.setenv("SPFFT_EXCH_CHUNKS", str(chunks))
    monkeypatch.setenv("SPFFT_EXCH_STICK_BLOCKS", str(blocks))
    _launch(nproc, exchange, "--iters=3", "--rccl-net", expect="rccl", timeout=240)


@pytest.mark.gpu
def test_rccl_init_failure_falls_back_to_peer_writes(gpu, monkeypatch):
    """Fault injection: every rank's RCCL initialisation fails. The ranks agree on
    the outcome (allgather) and move the exchange with IPC peer writes instead."""
    monkeypatch.setenv("SPFFT_FAULT_RCCL_INIT", "1")
    monkeypatch.setenv("SPFFT_AMD_LIBRARY", TESTING_LIB)
    _launch(2, "COMPACT_BUFFERED", "--iters=2", expect="ipc")


@pytest.mark.gpu
def test_rccl_init_failure_one_rank(gpu, monkeypatch):
    """Fault injection on one rank only (SPFFT_FAULT_RCCL_INIT=2: the last rank never
    calls ncclCommInitRankConfig). The other rank's non-blocking initialisation waits
    until SPFFT_COMM_TIMEOUT, aborts, and both ranks agree on the peer-write fallback
    instead of one of them blocking inside RCCL."""
    monkeypatch.setenv("SPFFT_FAULT_RCCL_INIT", "2")
    monkeypatch.setenv("SPFFT_AMD_LIBRARY", TESTING_LIB)
    monkeypatch.setenv("SPFFT_COMM_TIMEOUT", "5")
    _launch(2, "COMPACT_BUFFERED", "--iters=2", expect="ipc", timeout=180)


@pytest.mark.gpu
def test_rccl_init_failure_strict(gpu, monkeypatch):
    """With SPFFT_GPU_EXCHANGE=rccl there is no fallback: every rank raises MPIError
    (with the cause) instead of hanging."""
    monkeypatch.setenv("SPFFT_FAULT_RCCL_INIT", "1")
    monkeypatch.setenv("SPFFT_AMD_LIBRARY", TESTING_LIB)
    monkeypatch.setenv("SPFFT_GPU_EXCHANGE", "rccl")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", PROBE, "COMPACT_BUFFERED"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
    out = r.stdout + r.stderr
    assert r.returncode != 0, out[-4000:]
    assert "MPIError" in out and "fault injection RCCL_INIT" in out, out[-4000:]


def _bench_json(out):
    import json
    lines = [l for l in out.splitlines() if l.startswith("{") and '"metric"' in l]
    assert len(lines) == 1, out[-4000:]  # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_driver_launch_2ranks(gpu):
    # the round driver's multi-GPU launch line, rehearsed with 2 ranks on one
    # device: JSON contract fields and a checked round trip on every rank
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--size", "96", "--check"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    rec = _bench_json(r.stdout)
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["higher_is_better"] is True
    # the reported round-trip error is the MAX over both ranks
    assert rec["config"]["check_error"]["ranks_checked"] == 2
    assert rec["config"]["check_error"]["roundtrip"] < 1e-12
    assert rec["config"]["check_error"]["ok"]
    # both ranks ran on the one card of the test box: flagged as a rehearsal
    import torch
    ndev = torch.cuda.device_count()
    assert rec["config"]["distinct_devices"] == min(2, ndev)
    assert rec["config"]["shared_device"] is (ndev < 2)


@pytest.mark.gpu
def test_bench_driver_launch_2ranks_rccl(gpu, monkeypatch):
    """The driver's multi-GPU launch line with the RCCL data plane between the two
    ranks (virtual hosts on one device): the record carries a passing on-GPU
    round-trip check from both ranks, per-direction stage times and the exchange
    rate, without --check."""
    monkeypatch.setenv("SPFFT_RCCL_VIRTUAL_HOSTS", "1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--size", "64", "--transforms", "2"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    rec = _bench_json(r.stdout)
    cfg = rec["config"]
    assert cfg["data_plane"] == "rccl" and cfg["exchange"] == "compact"
    chk = cfg["check_error"]
    assert chk["ranks_checked"] == 2 and chk["ok"] and chk["roundtrip"] < 1e-12
    for d in ("backward", "forward"):
        assert cfg["stage_ms"][d]["z"] > 0
        assert cfg["exchange_stats"]["ms"][d] > 0 and cfg["exchange_stats"]["GBps_per_rank"][d] > 0
    assert "64^3" in rec["metric"]
    # the record predicts itself: modelled link / compute / pipelined times per direction
    m = cfg["model_ms"]
    assert m["chunks"] >= 1 and m["stick_blocks"] >= 1 and m["bytes_per_peer"] > 0
    for d in ("backward", "forward"):
        assert m[d]["link_ms"] > 0 and m[d]["compute_ms"] > 0 and m[d]["predicted_ms"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("queues", [1, 2])
def test_bench_rccl_few_hw_queues(gpu, monkeypatch, queues):
    """T = 4 transforms per rank on per-transform streams with K = 2 plane chunks and
    2 stick blocks, every exchange on the process's one RCCL channel stream (T + 1
    streams), with only 1 or 2 hardware queues per process: streams that share a
    queue serialise in issue order, which must never put a wait in front of the
    work it waits for."""
    monkeypatch.setenv("SPFFT_RCCL_VIRTUAL_HOSTS", "1")
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", str(queues))
    monkeypatch.setenv("SPFFT_EXCH_CHUNKS", "2")
    monkeypatch.setenv("SPFFT_EXCH_STICK_BLOCKS", "2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
           "--size", "64", "--transforms", "4", "--streams", "per-transform"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    rec = _bench_json(r.stdout)
    cfg = rec["config"]
    assert cfg["data_plane"] == "rccl" and cfg["check_error"]["ok"], cfg
    # the transforms run on the 4 torch streams; the library owns only the channel stream
    assert cfg["library_streams"] == 1, cfg


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["host-timeout", "peer-timeout"])
def test_exchange_failure_detected(gpu, mode):
    """A rank that never joins the exchange: the other rank's call raises MPIError
    within seconds (data plane aborted) instead of hanging."""
    probe = os.path.join(REPO, "tools", "failure_probe.py")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", probe, mode]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=120)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    line = [l for l in out.splitlines() if l.startswith("DETECTED")]
    assert line, out[-4000:]
    seconds = float(line[0].split()[1])
    assert seconds < 5.0, line[0]
    assert ("SPFFT_COMM_TIMEOUT" in line[0]) if mode == "host-timeout" else ("barrier" in line[0])


def _launch_tool(nproc, tool, *args, env_extra=None, timeout=300):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr=127.0.0.1",
           f"--nproc-per-node={nproc}", os.path.join(REPO, "tools", tool), *args]
    env = dict(os.environ, OMP_NUM_THREADS="1", **(env_extra or {}))
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    return r.returncode, r.stdout + r.stderr


@pytest.mark.gpu
def test_ipc_grid_churn_uneven_teardown(gpu):
    """Grids created collectively and destroyed by the ranks at different times
    (one rank drops its grid at once, the others keep it past the next grid's
    creation), two transforms per grid on different streams, empty sides, every
    exchange type, ending with a fresh UNBUFFERED grid. Destroying a grid must need
    no peer (reference: src/memory/gpu_array.hpp:88)."""
    code, out = _launch_tool(3, "ipc_churn.py", "--rounds", "14")
    assert code == 0, out[-4000:]
    assert "14/14 rounds passed" in out and "plane=ipc" in out, out[-4000:]


@pytest.mark.gpu
def test_ipc_peer_self_test(gpu):
    """The peer-write plane checks its route at setup (every receiver's L2 warmed
    with the old contents, stage-kernel-style remote stores, one barrier round, every
    word checked) and records the outcome in the plane info."""
    code, out = _launch_tool(3, "rccl_probe.py", "UNBUFFERED", "--iters=2", timeout=180)
    assert code == 0, out[-4000:]
    assert out.count("[ipc] self-test: ok") == 3, out[-4000:]
    # ranks sharing the GPU: normal-priority channel streams (profiles/r6/probe_state)
    assert out.count("channel priority: normal") == 3, out[-4000:]


@pytest.mark.gpu
def test_ipc_peer_self_test_failure_detected(gpu):
    """A wrong word in the self-test (fault injection: the last rank corrupts its
    message to rank 0) fails the plane on every rank. Ranks that share one GPU have no
    other plane (RCCL refuses them), so grid setup raises MPIError everywhere; ranks
    on distinct GPUs fall back to RCCL (DeviceComm::create)."""
    code, out = _launch_tool(2, "rccl_probe.py", "UNBUFFERED",
                             env_extra={"SPFFT_FAULT_PEER_SELFTEST": "1", **TESTING_ENV}, timeout=180)
    assert code != 0, out[-4000:]
    assert out.count("route self-test failed") >= 2, out[-4000:]


@pytest.mark.gpu
def test_ipc_stale_mapping_detected(gpu, monkeypatch):
    """A mapping whose header does not carry the owner's announced nonce (fault
    injection: the last rank announces a wrong one) is reported as MPIError on
    every rank at grid setup; nothing is computed on it."""
    code, out = _launch_tool(2, "rccl_probe.py", "UNBUFFERED",
                             env_extra={"SPFFT_FAULT_IPC_NONCE": "1", **TESTING_ENV}, timeout=180)
    assert code != 0, out[-4000:]
    assert out.count("stale IPC mapping") >= 2, out[-4000:]


@pytest.mark.gpu
@pytest.mark.parametrize("queues,barrier", [(1, "stream"), (2, "stream"), (1, "channel"), (2, "host")])
def test_bench_ipc_unbuffered_few_hw_queues(gpu, monkeypatch, queues, barrier):
    """UNBUFFERED over the IPC peer-write plane, 3 processes, T = 4 transforms per rank
    on per-transform streams with only 1 or 2 hardware queues per process: every
    barrier round of a plane keeps its issue order across the streams (stream mode:
    an event from the previous round's stream; channel mode: one ordered stream per
    process), so no barrier waits for work queued behind it. SPFFT_PEER_BARRIER=host
    runs the rounds on the host instead (stream synchronise + communicator barrier)."""
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", str(queues))
    monkeypatch.setenv("SPFFT_PEER_BARRIER", barrier)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(REPO, "bench.py"), "--gpus", "3", "--steps", "4", "--warmup", "1",
           "--size", "64", "--transforms", "4", "--streams", "per-transform", "--exchange", "unbuffered"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    rec = _bench_json(r.stdout)
    cfg = rec["config"]
    assert cfg["data_plane"] == "ipc" and cfg["check_error"]["ok"], cfg
    # the transforms run on the 4 torch streams; the library owns only the peer
    # channel stream in channel mode
    assert cfg["library_streams"] == (1 if barrier == "channel" else 0), cfg


# Relay routing (RelayDeviceComm): on an 8-GPU node with ranks on fewer GPUs, each
# peer message is split between the direct xGMI link and two-hop routes through the
# idle GPUs. On the one-GPU box, SPFFT_RELAY=force relays through virtual relay
# buffers on the rank's own GPU: the same layouts, shares, two phases and barriers.
@pytest.mark.gpu
@pytest.mark.parametrize("nproc,exchange,relays", [(2, "COMPACT_BUFFERED", 2), (3, "BUFFERED_FLOAT", 3),
                                                   (2, "BUFFERED", 1), (3, "COMPACT_BUFFERED_FLOAT", 2)])
def test_torch_dist_relay_forced(gpu, monkeypatch, nproc, exchange, relays):
    monkeypatch.setenv("SPFFT_RELAY", "force")
    monkeypatch.setenv("SPFFT_RELAY_VIRTUAL", str(relays))
    monkeypatch.setenv("SPFFT_RELAY_MIN_BYTES", "0")
    _launch(nproc, exchange, "--iters=3", "--dims=48,40,36", expect="relay")


@pytest.mark.gpu
def test_fuzz_dist_relay_forced(gpu):
    """The random distributions (empty ranks included) through the relay plane."""
    code, out = _launch_tool(3, "fuzz_dist.py", "--cases", "30", "--seed", "12",
                             env_extra={"SPFFT_RELAY": "force", "SPFFT_RELAY_MIN_BYTES": "0",
                                        "SPFFT_RELAY_VIRTUAL": "2"})
    assert code == 0, out[-4000:]
    assert "30/30 passed" in out and "plane=relay" in out, out[-4000:]


@pytest.mark.gpu
def test_fuzz_dist_relay_pipelined(gpu):
    """The relay plane's registered, stream-ordered exchanges (device barrier rounds
    on the plane's ordered stream, no host round trip) with pipelined plans: 2 plane
    chunks x 2 stick blocks per direction, random distributions with empty ranks."""
    code, out = _launch_tool(3, "fuzz_dist.py", "--cases", "24", "--seed", "31",
                             env_extra={"SPFFT_RELAY": "force", "SPFFT_RELAY_MIN_BYTES": "0",
                                        "SPFFT_RELAY_VIRTUAL": "2", "SPFFT_EXCH_CHUNKS": "2",
                                        "SPFFT_EXCH_STICK_BLOCKS": "2"})
    assert code == 0, out[-4000:]
    assert "24/24 passed" in out and "plane=relay" in out, out[-4000:]


@pytest.mark.gpu
def test_bench_relay_model(gpu, monkeypatch):
    """bench.py over the forced relay plane: checked round trip on both ranks, and the
    modelled link time accounts for the relay shares."""
    monkeypatch.setenv("SPFFT_RELAY", "force")
    monkeypatch.setenv("SPFFT_RELAY_VIRTUAL", "3")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--size", "96", "--transforms", "2"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    cfg = _bench_json(r.stdout)["config"]
    assert cfg["data_plane"] == "relay" and cfg["check_error"]["ok"], cfg
    assert cfg["model_ms"]["relay_gpus"] == 3


@pytest.mark.gpu
def test_relay_self_test_failure_falls_back(gpu, monkeypatch):
    """The relay plane checks every route with a known pattern before it carries data;
    a wrong byte on any rank (fault injection) makes every rank drop the relay plane
    for the next one (here, ranks sharing the GPU: IPC peer writes), with the cause
    printed once."""
    monkeypatch.setenv("SPFFT_RELAY", "force")
    monkeypatch.setenv("SPFFT_FAULT_RELAY_SELFTEST", "1")
    monkeypatch.setenv("SPFFT_AMD_LIBRARY", TESTING_LIB)
    code, out = _launch_tool(2, "rccl_probe.py", "COMPACT_BUFFERED", "--iters=2")
    assert code == 0, out[-4000:]
    assert out.count("[ipc]") == 2 and "self-test exchange delivered wrong data" in out, out[-4000:]


@pytest.mark.gpu
@pytest.mark.parametrize("plane", ["ipc", "relay"])
def test_fuzz_dist_local_maxima(gpu, plane):
    """Every rank passes its own stick and plane counts as the grid maxima (zero on
    empty ranks), so the exchange sides differ per rank (the reference allows this,
    grid_internal.cpp:190): the relay split must use each sender's own capacity and
    the self-tests a message size every rank can hold."""
    env = {"SPFFT_RELAY": "force", "SPFFT_RELAY_MIN_BYTES": "0", "SPFFT_RELAY_VIRTUAL": "2"} \
        if plane == "relay" else {}
    code, out = _launch_tool(3, "fuzz_dist.py", "--cases", "24", "--seed", "21", "--maxima", "local",
                             env_extra=env)
    assert code == 0, out[-4000:]
    assert "24/24 passed" in out and f"plane={plane}" in out, out[-4000:]

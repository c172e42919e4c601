#!/usr/bin/env python3
"""Headline benchmark: 3D C2C transforms/sec, 256^3 spherical cutoff, 1/2/4/8 MI355X.

One step = one backward (frequency -> space) + one forward (space -> frequency)
transform of the 256^3 grid with the spherical cutoff |k| <= N/2 (≈8.78 M
frequency values, 51,431 z-sticks), fp64 complex, exactly like one repeat of
the reference benchmark (reference: tests/programs/benchmark.cpp:85-88).
Data is synthetic (random values),
inputs and outputs live in GPU memory ("gpu-gpu" mode of the reference).

A step runs 4 independent transforms of that problem (--transforms, the
reference benchmark's -m, tests/programs/benchmark.cpp:142, 84-96): multi_transform_backward +
multi_transform_forward, one HIP stream per transform, so one transform's
all-to-all and kernel tails overlap the others' kernels. transforms/sec =
2 * transforms * steps / elapsed. --transforms 1 times single calls.

Multi-GPU: launched by torch.distributed.run, one rank per GPU; z-sticks and
xy-planes are split evenly over ranks and the pencil <-> slab redistribution
runs inside the library over one of its data planes: RCCL all-to-all(v) over
xGMI, IPC peer writes from the stage kernels, or relay routing through idle
GPUs. Before the timed loop every eligible plane is timed on a few steps
(config.planes_ms) and the headline runs on the fastest (config.plane_choice;
--plane forces one). The problem size is fixed as N grows (strong scaling);
`value` is the whole-job rate.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

# transforms/s of the reference's vendor-FFT calls alone on one MI355X, 256^3
# C2C fp64 r = N/2 (tools/ref_pipeline_bench.py), by
# the number of transforms per step (T on T streams)
REF_FFT_ONLY_256_BY_T = {1: 2210.2, 4: 2418.3}  # profiles/r3/comparator/

# xGMI bandwidth one peer pair gets per direction (one link of an MI355X node:
# 153.6 GB/s per link both directions, ~70 GB/s usable one way): the model's
# assumption when the data plane has not measured it (plane info
# "link_GBps_measured": an 8 MiB copy into every rank's right neighbour at setup)
LINK_GBPS = 70.0
# two device barrier rounds per relay exchange (stream-ordered relay plane)
RELAY_BARRIER_MS = 0.02


def _model(stages, sent_per_rank, world, chunks, blocks, relays=0, link_gbps=None):
    """Modelled per-direction times of a distributed step (README, "Multi-GPU
    scaling"): every rank sends sent/(N-1) bytes to each peer over its own link, all
    links at once, so the exchange takes link_ms = sent/(N-1) / link rate; the
    compute is this run's own z and y/x stage times. The pipelined grid of K plane
    chunks x I stick blocks overlaps all but one step's compute with the link:
    predicted = max(link, compute) + compute / (K * I) (unpipelined: link + compute).
    The driver's measured ms_per_step / (2 T) can be read against `predicted_ms`."""
    rate = link_gbps if link_gbps else LINK_GBPS
    per_peer = sent_per_rank / max(1, world - 1)
    # relay plane: every link direction carries (N - 1) / (N - 1 + K) of a
    # peer message, in two stream-ordered hops (push, pull)
    share = (world - 1) / (world - 1 + relays) if relays else 1.0
    link_ms = per_peer * share / (rate * 1e9) * 1e3 * (2 if relays else 1)
    link_ms += RELAY_BARRIER_MS if relays else 0.0
    out = {"link_GBps_assumed": LINK_GBPS, "link_GBps_used": rate,
           "link_GBps_source": "measured" if link_gbps else "assumed", "bytes_per_peer": per_peer,
           "chunks": chunks, "stick_blocks": blocks, "relay_gpus": relays}
    for d in ("backward", "forward"):
        st = stages.get(d, {})
        compute = sum(v for k, v in st.items() if k not in ("exchange", "exchange-span", "exchange-tail", "total"))
        steps = max(1, chunks * blocks)
        pred = (max(link_ms, compute) + compute / steps) if steps > 1 else (link_ms + compute)
        out[d] = {"link_ms": link_ms, "compute_ms": compute, "predicted_ms": pred,
                  "bound": "link" if link_ms > compute else "compute"}
    out["predicted_pair_ms"] = out["backward"]["predicted_ms"] + out["forward"]["predicted_ms"]
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--cutoff", type=float, default=0.5)
    ap.add_argument("--exchange", default="compact",
                    choices=["compact", "compactFloat", "buffered", "bufferedFloat", "unbuffered"])
    ap.add_argument("--precision", default="double", choices=["double", "single"])
    ap.add_argument("--type", default="c2c", choices=["c2c", "r2c"])
    ap.add_argument("--transforms", type=int, default=4,
                    help="independent transforms per step, run with multi_transform_backward/"
                         "forward on one stream each (the reference benchmark's -m): one "
                         "transform's all-to-all overlaps the others' FFT kernels")
    ap.add_argument("--streams", default="auto", choices=["auto", "per-transform", "one"],
                    help="with --sync stream and T > 1: one stream per transform (their kernels "
                         "and exchanges overlap), or all transforms on torch's current stream "
                         "(identical single-GPU transforms then run batched, one launch per "
                         "stage for up to 8). auto: one stream on 1 GPU (batched launches "
                         "measured +2%% over 4 streams at 256^3, profiles/r3/t4_streams.txt), "
                         "per-transform streams on N > 1 GPUs (one transform's all-to-all "
                         "overlaps the others' kernels; distributed plans do not batch)")
    ap.add_argument("--timing", action="store_true", help="print the native timing tree")
    ap.add_argument("--check", action="store_true",
                    help="also compare the backward transform against the dense numpy oracle "
                         "(1 rank; the GPU round-trip check on every rank always runs)")
    ap.add_argument("--profile-reps", type=int, default=5,
                    help="backward+forward pairs of transform 0 timed per stage after the "
                         "timed loop (0 = no stage profile)")
    ap.add_argument("--planes-probe", type=int, default=1,
                    help="N > 1: before the timed loop, time a few steps (one transform per step) on "
                         "every eligible data plane (rccl / ipc / relay), record them in "
                         "config.planes_ms and run the headline on the fastest (--plane auto)")
    ap.add_argument("--probe-planes", default="rccl,ipc,relay",
                    help="comma-separated data planes the probe times (--planes-probe 1)")
    ap.add_argument("--plane", default="auto", choices=["auto", "default", "rccl", "ipc", "relay"],
                    help="N > 1: data plane of the headline transforms: auto = the fastest of the "
                         "probe (the library's default if the probe is off), default = the "
                         "library's own choice, or one plane forced")
    ap.add_argument("--sync", default="stream", choices=["stream", "call"],
                    help="stream: transforms are stream-ordered on torch's current stream (no host "
                         "wait per call; the timed loop still ends with a device synchronize); "
                         "call: every backward/forward call blocks until done (SpFFT default)")
    return ap.parse_args()


def _check(a, sp, t, values, gidx, dims, ttype, world):
    """Backward vs the dense numpy oracle (1 rank, --check): max relative error."""
    import torch
    from spfft_amd.utils.oracle import dense_backward, max_rel_error
    space = t.backward(values)
    torch.cuda.synchronize()
    ref = dense_backward(gidx, values.cpu().numpy(), dims, r2c=(ttype == sp.TransformType.R2C))
    return {"backward_vs_numpy": max_rel_error(space.cpu().numpy(), ref)}


def _roundtrip_gpu(sp, ts, vals, outs, r2c):
    """Round-trip error of every transform of this rank, computed on the GPU (no host
    copies): backward + forward with full scaling must reproduce the input. Random
    R2C input is not hermitian on the x = 0 plane, so R2C compares the second round
    trip with the first (the round trip is a projection)."""
    import torch
    worst = 0.0
    for t, v, o in zip(ts, vals, outs):
        if v.numel() == 0:
            continue
        t.backward(v)
        t.forward(None, output=o, scaling=sp.Scaling.FULL)
        base = v
        if r2c:
            torch.cuda.synchronize()
            base = o.clone()
            t.backward(base)
            t.forward(None, output=o, scaling=sp.Scaling.FULL)
        torch.cuda.synchronize()
        scale = float(base.abs().max().item()) or 1.0
        worst = max(worst, float((o - base).abs().max().item()) / scale)
    return worst


def _plane_env(name, shared):
    """The library's plane switches (read at grid setup) that select a data plane;
    ranks sharing a GPU relay through virtual relays (rehearsal)."""
    return {"rccl": {"SPFFT_GPU_EXCHANGE": "rccl", "SPFFT_RELAY": "0"},
            "ipc": {"SPFFT_GPU_EXCHANGE": "ipc", "SPFFT_RELAY": "0"},
            "relay": {"SPFFT_GPU_EXCHANGE": "", "SPFFT_RELAY": "force" if shared else "auto"}}.get(name, {})


def _gather_devices(torch, dev, dist, world):
    prop = torch.cuda.get_device_properties(dev)
    mine = f"{prop.pci_domain_id:04x}:{prop.pci_bus_id:02x}:{prop.pci_device_id:02x}"
    if dist is None:
        return [mine]
    out = [None] * world
    dist.all_gather_object(out, mine)
    return out


def _choose_plane(requested, planes_ms):
    """The headline's data plane: the forced one, or (auto) the fastest plane of the
    probe that really ran as itself (a plane that fell back to another is not a
    candidate); the library's default when nothing was probed."""
    if requested not in ("auto",):
        return {"plane": requested, "basis": "--plane"}
    if any(os.environ.get(k) for k in ("SPFFT_GPU_EXCHANGE", "SPFFT_RELAY")):
        return {"plane": "default", "basis": "the plane switches set in the environment"}
    ok = {k: v["ms_per_step"] for k, v in (planes_ms or {}).items()
          if "ms_per_step" in v and v.get("plane") == k}
    if not ok:
        return {"plane": "default", "basis": "no probe result: the library's default plane"}
    best = min(ok, key=ok.get)
    return {"plane": best, "basis": "fastest of planes_ms", "ms_per_step": ok[best]}


def _probe_planes(make_transform, dev, cdtype, world, shared, dist, steps=5, warmup=2,
                  names=("rccl", "ipc", "relay")):
    """ms per step (one backward + forward of one transform) on every eligible data
    plane, each forced through the library's plane switches (read at grid setup):
    rccl (not between ranks that share a GPU), ipc (peer writes) and relay (idle GPUs
    of the node, or virtual relays on a shared GPU). A plane the library cannot set up
    is recorded with its error (the failure is agreed on by every rank)."""
    import time as _t
    import torch
    planes = {name: _plane_env(name, shared) for name in names}
    out = {}
    for name, env in planes.items():
        if name == "rccl" and shared and os.environ.get("SPFFT_RCCL_VIRTUAL_HOSTS") != "1":
            out[name] = {"skipped": "ranks share a GPU (RCCL refuses duplicate devices)"}
            continue
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        g = t = None
        try:
            g, t, local, _ = make_transform()
            t.set_stream(torch.cuda.current_stream(), synchronous=False)
            v = torch.randn(len(local), dtype=cdtype, device=dev)
            o = torch.empty_like(v)
            for _ in range(warmup):
                t.backward(v)
                t.forward(None, output=o)
            torch.cuda.synchronize()
            dist.barrier()
            t0 = _t.perf_counter()
            for _ in range(steps):
                t.backward(v)
                t.forward(None, output=o)
            torch.cuda.synchronize()
            e = torch.tensor([_t.perf_counter() - t0], dtype=torch.float64)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            out[name] = {"ms_per_step": 1e3 * float(e.item()) / steps, "plane": g.data_plane}
        except Exception as ex:  # noqa: BLE001 - recorded
            out[name] = {"error": f"{type(ex).__name__}: {ex}"[:300]}
        finally:
            for k, val in saved.items():
                if val is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = val
            del t, g
            torch.cuda.synchronize()
    return out


def _timing_node(tree, path):
    nodes = tree.get("timings", [])
    node = None
    for name in path:
        node = next((n for n in nodes if n["identifier"] == name), None)
        if node is None:
            return None
        nodes = node.get("sub-timings", [])
    return node


def _stage_profile(sp, t, values, out, reps):
    """Per-direction GPU stage times of ONE transform run alone (outside the timed
    loop): hipEvent intervals at the stage boundaries on the transform's stream
    (gpu/<direction>/<stage>) and, for pipelined exchanges, the span of the exchange
    on the data plane's stream (exchange-span). Medians in milliseconds."""
    import torch
    sp.timing_reset()
    sp.timing_enable(True)
    for _ in range(reps):
        t.backward(values)
        t.forward(None, output=out)
    torch.cuda.synchronize()
    t.synchronize()  # completes the stage intervals
    sp.timing_enable(False)
    tree = sp.timing_json()
    prof = {}
    for direction in ("backward", "forward"):
        node = _timing_node(tree, ["gpu", direction])
        if node is None:
            continue
        prof[direction] = {c["identifier"]: 1e3 * c["median"] for c in node.get("sub-timings", [])}
        prof[direction]["total"] = sum(v for k, v in prof[direction].items() if k != "exchange-span")
    sp.timing_reset()
    return prof


def _metric(n, ttype, cutoff, single):
    headline = "3D C2C transforms/sec, 256^3 spherical cutoff, 1/2/4/8 MI355X"
    if n == 256 and ttype == "c2c" and cutoff == 0.5 and not single:
        return headline  # BASELINE.json's metric string
    prec = "fp32" if single else "fp64"
    return f"3D {ttype.upper()} {prec} transforms/sec, {n}^3 spherical cutoff r={cutoff}*N, MI355X"


def main():
    a = parse()
    import numpy as np
    import torch

    import spfft_amd as sp
    from spfft_amd.utils.indices import distribute_sticks, sphere_indices

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE {world}")
    # one rank per GPU; more ranks than GPUs (rehearsal on a small box) share
    # devices round-robin and the library then moves data by IPC peer writes
    ndev = max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank % ndev)
    dev = torch.device("cuda", local_rank % ndev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # torch.distributed is the control plane only (plan setup, barriers,
        # the timing reduction): gloo. The transform's all-to-all runs on the
        # library's own RCCL communicator over xGMI.
        dist.init_process_group("gloo")

    n = a.size
    dims = (n, n, n)
    ttype = sp.TransformType.R2C if a.type == "r2c" else sp.TransformType.C2C
    gidx = sphere_indices(*dims, a.cutoff, r2c=(ttype == sp.TransformType.R2C))
    exch = {"compact": sp.ExchangeType.COMPACT_BUFFERED,
            "compactFloat": sp.ExchangeType.COMPACT_BUFFERED_FLOAT,
            "buffered": sp.ExchangeType.BUFFERED,
            "bufferedFloat": sp.ExchangeType.BUFFERED_FLOAT,
            "unbuffered": sp.ExchangeType.UNBUFFERED}[a.exchange]
    single = a.precision == "single"
    GridCls = sp.GridFloat if single else sp.Grid
    cdtype = torch.complex64 if single else torch.complex128

    def make_transform():
        # every transform owns its grid (multi_transform rejects shared grids)
        if world == 1:
            g = GridCls(n, n, n, n * n, sp.ProcessingUnit.GPU, 1)
            return g, g.create_transform(sp.ProcessingUnit.GPU, ttype, n, n, n, n, gidx), gidx, n
        from spfft_amd.parallel import TorchDistComm, make_distributed
        setup = make_distributed(TorchDistComm(), dims, gidx, processing_unit=sp.ProcessingUnit.GPU,
                                 transform_type=ttype, exchange_type=exch, single=single)
        return setup.grid, setup.transform, setup.indices, setup.z_length

    # N > 1: time every eligible data plane first and run the headline on the
    # fastest (the library's plane switches are read at grid setup)
    planes_ms, plane_choice = None, None
    if world > 1:
        shared = len(set(_gather_devices(torch, dev, dist, world))) < world
        if a.planes_probe:
            planes_ms = _probe_planes(make_transform, dev, cdtype, world, shared, dist,
                                      names=tuple(x for x in a.probe_planes.split(",") if x))
        plane_choice = _choose_plane(a.plane, planes_ms)
        os.environ.update(_plane_env(plane_choice["plane"], shared))
    T = max(1, a.transforms)
    made = [make_transform() for _ in range(T)]
    grids = [m[0] for m in made]
    ts = [m[1] for m in made]
    local = made[0][2]
    grid, t = grids[0], ts[0]

    plane = grid.data_plane if world > 1 else "none"
    plane_info = grid.data_plane_info if world > 1 else {"kind": "none"}
    # every GPU the job touched: the ranks' devices (PCI locations, gathered) and
    # any relay GPUs the data plane uses besides them
    rank_devs = _gather_devices(torch, dev, dist, world)
    touched = list(dict.fromkeys(rank_devs + list(plane_info.get("devices", []))))
    if a.streams == "auto":
        a.streams = "one" if world == 1 else "per-transform"
    streams = []
    if a.sync == "stream":
        if T == 1 or a.streams == "one":
            for tr in ts:
                tr.set_stream(torch.cuda.current_stream(), synchronous=False)
        else:
            streams = [torch.cuda.Stream() for _ in range(T)]
            for tr, st in zip(ts, streams):
                tr.set_stream(st, synchronous=False)

    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    vals = [torch.randn(len(local), dtype=cdtype, device=dev, generator=gen) for _ in range(T)]
    outs = [torch.empty_like(v) for v in vals]
    values, out = vals[0], outs[0]

    def step():
        if T == 1:
            t.backward(values)
            t.forward(None, output=out)
        else:
            sp.multi_transform_backward(ts, vals)
            sp.multi_transform_forward(ts, outputs=outs)

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(a.warmup):
        step()
    barrier()
    if a.timing:
        sp.timing_reset()
        sp.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    if a.timing:
        for tr in ts:  # completes the GPU stage intervals (gpu/<direction>/<stage>)
            tr.synchronize()
        if rank == 0:
            print(sp.timing_report(), file=sys.stderr)
        sp.timing_enable(False)
    # Self-check outside the timed region, on every rank and every transform,
    # on the GPU: a multi-GPU record carries its own proof that the exchange
    # moved the right bytes. The worst rank is reported.
    check = {"roundtrip": _roundtrip_gpu(sp, ts, vals, outs, ttype == sp.TransformType.R2C),
             "ranks_checked": world, "transforms_checked": T,
             "method": "max |forward(backward(v)) - v| / max |v| with full scaling, on the GPU"}
    if dist is not None:
        e = torch.tensor([check["roundtrip"]], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        check["roundtrip"] = float(e.item())
    check["tolerance"] = 1e-4 if (single or "Float" in a.exchange) else 1e-10
    check["ok"] = check["roundtrip"] < check["tolerance"]
    if a.check and world == 1:
        check.update(_check(a, sp, t, values, gidx, dims, ttype, world))
    # per-direction stage times of transform 0 alone, and the exchange rate
    stages = _stage_profile(sp, t, values, out, a.profile_reps) if a.profile_reps > 0 else {}
    xstats = None
    if world > 1 and stages:
        eb = (8 if single or "Float" in a.exchange else 16)
        loc = np.asarray(local).reshape(-1, 3).astype(np.int64)
        local_sticks = int(np.unique((loc[:, 0] % n) * n + (loc[:, 1] % n)).size) if len(loc) else 0
        z_len = made[0][3]
        sent = local_sticks * (n - z_len) * eb  # compact layout: every non-local plane leaves
        ms = {}
        for d in ("backward", "forward"):
            st = stages.get(d, {})
            ms[d] = st.get("exchange-span", st.get("exchange"))
        xstats = {"bytes_sent_per_rank": sent,
                "ms": ms,
                "GBps_per_rank": {d: (sent / (v * 1e-3) / 1e9 if v else None) for d, v in ms.items()}}
        e = torch.tensor([float(sent)], dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        xstats["max_bytes_sent_per_rank"] = float(e.item())
    # ranks that share a device (rehearsal on a small box) are not a multi-GPU
    # measurement: record how many distinct devices the ranks ran on
    n_devices = len(set(rank_devs))
    model = None
    if world > 1 and stages:
        chunks, blocks, peer_writes, relays = t.exchange_plan()
        # (a same-device copy rate is no link rate: the model keeps its assumption)
        link = plane_info.get("link_GBps_measured") if plane_info.get("link_kind") == "xgmi" else None
        model = _model(stages, xstats["max_bytes_sent_per_rank"], world, chunks, blocks, relays, link)
        model["peer_writes"] = peer_writes
        model["shared_device"] = n_devices < world
    ms_per_step = 1e3 * elapsed / a.steps
    rate = 2.0 * T * a.steps / elapsed
    # the reference's FFT calls alone (rocFFT via
    # torch.fft) on one MI355X, an upper bound on its throughput for the headline config;
    # no measured reference exists for other configs or for N > 1 GPUs
    headline = (n == 256 and a.cutoff == 0.5 and a.type == "c2c" and not single)
    # comparator per protocol: the reference algorithm's rocFFT calls alone on one
    # MI355X, one transform at a time (T = 1) or T transforms on T streams
    # (tools/ref_pipeline_bench.py --transforms T), so the ratio does not mix the
    # multi-transform overlap into the per-transform speed-up
    ref_rate = REF_FFT_ONLY_256_BY_T.get(T) if (headline and world == 1) else None
    vs_baseline = rate / ref_rate if ref_rate else None
    if rank == 0:
        rec = {
            "metric": _metric(n, a.type, a.cutoff, single),
            "value": rate,
            "unit": "transforms/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": vs_baseline,
            "vs_baseline_basis": (f"value / {ref_rate:.1f}: the reference algorithm's rocFFT calls "
                                  f"alone on one MI355X with the same {T} transform(s) per step "
                                  f"(BASELINE.md {'B7' if T == 1 else 'B7-T4'}, tools/ref_pipeline_bench.py --transforms {T})"
                                  if vs_baseline else None),
            "dtype": "fp32" if single else "fp64",
            "data": "synthetic (random complex values on the spherical-cutoff index set)",
            "config": {
                "model": f"sparse 3D FFT {n}^3 {a.type.upper()} spherical cutoff r={a.cutoff}*N",
                "global_batch": 2 * T,
                "transforms_per_step": T,
                "seq_len": n,
                "parallelism": f"slab/pencil x{world} ({a.exchange} all-to-all)",
                "num_frequency_values": int(len(gidx)),
                "exchange": a.exchange,
                "data_plane": plane,
                "distinct_devices": n_devices,
                "devices_touched": touched,
                "plane_info": plane_info,
                "plane_self_test": plane_info.get("self_test"),
                "shared_device": n_devices < world,
                "sync": a.sync,
                "streams": a.streams if T > 1 else "one",
                "library_streams": sp.library_streams(),
                "check_error": check,
                "stage_ms": stages,
                "stage_ms_basis": (f"transform 0 alone, median of {a.profile_reps} backward+forward "
                                   "pairs after the timed loop (hipEvent stage marks)" if stages else None),
                "exchange_stats": xstats,
                "model_ms": model,
                "planes_ms": planes_ms,
                "planes_ms_basis": ("one transform per step, 2 warmup + 5 timed steps per plane, "
                                    "before the timed loop" if planes_ms else None),
                "plane_choice": plane_choice,
                "step": ("1 backward + 1 forward transform" if T == 1 else
                         f"multi_transform backward + forward of {T} independent transforms"),
            },
        }
        print(json.dumps(rec), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

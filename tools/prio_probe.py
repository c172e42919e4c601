"""Does a high-priority HIP stream in the process slow the transform's kernels?

One rank, 256^3 C2C fp64, one transform per step on torch's current stream:
transforms/s (a) as is, (b) while an idle high-priority torch stream exists,
(c) after it was destroyed, (d) with an idle normal-priority extra stream.
Motivation: 2 ranks sharing a GPU ran their stage kernels 2x slower after a
relay-plane grid (whose ordered channel stream is high priority) had been
created and destroyed (profiles/r6/probe_state/).
"""
import gc
import json
import time

import torch

import spfft_amd as sp
from spfft_amd.utils.indices import sphere_indices


def rate(t, v, o, steps=100):
    for _ in range(5):
        t.backward(v)
        t.forward(None, output=o)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        t.backward(v)
        t.forward(None, output=o)
    torch.cuda.synchronize()
    return 2 * steps / (time.perf_counter() - t0)


def main():
    n = 256
    gidx = sphere_indices(n, n, n, 0.5, r2c=False)
    g = sp.Grid(n, n, n, n * n, sp.ProcessingUnit.GPU, 1)
    t = g.create_transform(sp.ProcessingUnit.GPU, sp.TransformType.C2C, n, n, n, n, gidx)
    t.set_stream(torch.cuda.current_stream(), synchronous=False)
    v = torch.randn(len(gidx), dtype=torch.complex128, device="cuda")
    o = torch.empty_like(v)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    res = {"priority_range": [lo, hi]}
    res["a_plain"] = rate(t, v, o)
    s = torch.cuda.Stream(priority=hi)
    torch.cuda.synchronize()
    res["b_high_prio_alive"] = rate(t, v, o)
    with torch.cuda.stream(s):
        x = torch.ones(1 << 20, device="cuda")
        x.mul_(2)
    torch.cuda.synchronize()
    res["b2_high_prio_used"] = rate(t, v, o)
    # the library's own high-priority stream path: the transform on a stream of it
    t.set_stream(s, synchronous=False)
    res["b3_transform_on_high_prio"] = rate(t, v, o)
    t.set_stream(torch.cuda.current_stream(), synchronous=False)
    del s, x
    gc.collect()
    torch.cuda.synchronize()
    res["c_after_destroy"] = rate(t, v, o)
    s2 = torch.cuda.Stream()
    res["d_normal_extra"] = rate(t, v, o)
    del s2
    res["e_plain_again"] = rate(t, v, o)
    print(json.dumps({k: (round(x, 1) if isinstance(x, float) else x) for k, x in res.items()}))


if __name__ == "__main__":
    main()

"""Timeline of a rocprofv3 kernel_trace.csv: per kernel name, count / median /
total duration, the busy fraction of the traced span, and the idle gaps between
consecutive kernels (one process's trace). --tail N prints the last N kernels
with their start offsets and gaps.
    python tools/ktimeline.py run_kernel_trace.csv [--tail 40]"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--tail", type=int, default=0)
    ap.add_argument("--skip", type=int, default=0, help="ignore the first N kernels (setup, warmup)")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))[a.skip:]
    if not rows:
        return
    acc = collections.defaultdict(list)
    gaps = []
    prev_end = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("void spfft::dev::", "").split("<")[0].split("(")[0]
        acc[name].append((e - s) / 1e3)
        if prev_end is not None:
            gaps.append((s - prev_end) / 1e3)
        prev_end = max(prev_end or 0, e)
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    busy = sum(sum(v) for v in acc.values())
    print(f"kernels {len(rows)}  span {span:.1f} us  kernel time {busy:.1f} us ({100 * busy / span:.0f}%)")
    for name, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        v = sorted(v)
        print(f"  {name:32s} n={len(v):5d} median={v[len(v) // 2]:8.1f} us total={sum(v):10.1f} us")
    if gaps:
        g = sorted(gaps)
        print(f"gaps: median {g[len(g) // 2]:.1f} us, p90 {g[int(0.9 * len(g))]:.1f} us, "
              f"total {sum(x for x in g if x > 0):.1f} us")
    if a.tail:
        t0 = int(rows[-a.tail]["Start_Timestamp"])
        prev = None
        for r in rows[-a.tail:]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            name = r["Kernel_Name"].replace("void spfft::dev::", "").split("<")[0].split("(")[0]
            gap = "" if prev is None else f"gap {(s - prev) / 1e3:7.1f}"
            print(f"  +{(s - t0) / 1e3:9.1f} us {name:32s} {(e - s) / 1e3:8.1f} us {gap}")
            prev = e


if __name__ == "__main__":
    main()

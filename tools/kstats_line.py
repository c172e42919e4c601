"""One-line summary of a rocprofv3 kernel-stats CSV: avg us of the six stage
kernels (zb yb xb xf yf zf) and the bench value of the profiled run."""
import csv
import json
import sys

stats, bench, tag = sys.argv[1], sys.argv[2], sys.argv[3]
keys = [("zb", "z_backward"), ("yb", "y_backward"), ("xb", "x_backward"),
        ("xf", "x_forward"), ("yf", "y_forward"), ("zf", "z_forward")]
t = {}
with open(stats) as f:
    for row in csv.DictReader(f):
        name = row["Name"]
        for k, pat in keys:
            if pat in name:
                t[k] = t.get(k, 0.0) + float(row["TotalDurationNs"]) / 1e3 / max(1, int(row["Calls"]))
val = [l for l in open(bench) if l.startswith("{")]
v = json.loads(val[-1])["value"] if val else float("nan")
print(f"{tag:24s} " + " ".join(f"{k}={t.get(k, 0):6.1f}" for k, _ in keys) + f"  value={v:.0f}")

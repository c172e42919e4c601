"""HIP API calls of one process between the end of one kernel and the start of
the next (rocprofv3 --hip-trace + --kernel-trace CSVs): per API name, calls and
total host time over the last repeats, to find what fills the host gaps.
    python tools/api_between.py run_hip_api_trace.csv run_kernel_trace.csv"""
import collections
import csv
import sys

api = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ker = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
if len(ker) < 60:
    sys.exit(0)
t0, t1 = int(ker[-50]["Start_Timestamp"]), int(ker[-1]["End_Timestamp"])
acc = collections.defaultdict(lambda: [0, 0.0, 0.0])
for r in api:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t0 or s > t1:
        continue
    a = acc[r["Function"]]
    a[0] += 1
    a[1] += (e - s) / 1e3
    a[2] = max(a[2], (e - s) / 1e3)
span = (t1 - t0) / 1e3
print(f"host API calls over the last 50 kernels ({span:.0f} us):")
for name, (n, tot, mx) in sorted(acc.items(), key=lambda kv: -kv[1][1])[:18]:
    print(f"  {name:36s} n={n:5d} total={tot:9.1f} us max={mx:8.1f} us")

"""Per-kernel mean duration from a rocprofv3 kernel_trace.csv, split by the grid's
z extent (batched multi-transform launches carry one transform per z slice)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    if "spfft" not in r["Kernel_Name"]:
        continue
    name = r["Kernel_Name"].replace("void spfft::dev::", "").split("<")[0]
    z = int(r["Grid_Size_Z"])
    acc[(name, z)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot = collections.defaultdict(float)
for (name, z), v in sorted(acc.items(), key=lambda kv: (kv[0][1], kv[0][0])):
    m = sorted(v)[len(v) // 2]
    tot[z] += m
    print(f"z={z} {name:28s} n={len(v):4d} median_us={m:8.1f} per_transform={m / z:8.1f}")
for z, t in sorted(tot.items()):
    print(f"z={z} kernel sum per pair {t:.1f} us ({t / z:.1f} per transform)")

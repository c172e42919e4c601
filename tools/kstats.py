"""Summarise a rocprofv3 *_kernel_stats.csv (kernel, calls, avg us, share)."""
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = 0.0
for r in rows:
    name = re.sub(r"\(.*", "", r["Name"])
    name = name.replace("spfft::dev::", "").replace("spfft::", "")[:100]
    avg = float(r["AverageNs"]) / 1e3
    print(f"{name:100s} calls={int(r['Calls']):5d} avg_us={avg:9.1f} pct={float(r['Percentage']):5.1f}")

"""Per-kernel average times (us) for several rocprofv3 stats dirs, as a table."""
import csv, re, sys, os
dirs = sys.argv[1:]
tab = {}
for d in dirs:
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))):
        n = re.sub(r"\(.*", "", r["Name"])
        if "spfft" not in n:
            continue
        k = re.sub(r"^void spfft::dev::", "", n).split("<")[0]
        tab.setdefault(k, {})[d] = float(r["AverageNs"]) / 1e3
ks = sorted(tab)
print("variant".ljust(28) + "".join(k[:12].rjust(13) for k in ks) + "   total")
for d in dirs:
    vals = [tab[k].get(d, 0) for k in ks]
    print(os.path.basename(d).ljust(28) + "".join(f"{v:13.1f}" for v in vals) + f"{sum(vals):8.1f}")

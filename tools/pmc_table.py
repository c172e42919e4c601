"""Per-kernel table of a rocprofv3 --pmc counter_collection.csv (averaged over dispatches)."""
import collections
import csv
import sys


def table(path, kernel_filter="spfft"):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        k = r["Kernel_Name"]
        if kernel_filter not in k:
            continue
        k = k.split("(")[0].replace("void ", "").replace("spfft::dev::", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = []
    for k, d in agg.items():
        vals = {c: sum(v) / len(v) for c, v in d.items()}
        out.append((k, vals))
    return out


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print("==", p)
        for k, vals in table(p):
            print(f"  {k[:90]}")
            print("    " + "  ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))

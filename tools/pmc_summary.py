"""Aggregate rocprofv3 counter_collection.csv files: mean counter value per kernel."""
import csv, re, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("spfft::dev::", "").replace("spfft::", "")
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, ctrs in acc.items():
    if "at::" in name or "rocclr" in name:
        continue
    print(name[:90])
    for c, v in sorted(ctrs.items()):
        print(f"    {c:28s} {sum(v)/len(v):16.4g}")

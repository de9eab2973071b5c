"""Per-dispatch PMC table (dispatch order) across several rocprofv3 --pmc runs of the same
deterministic script: run k's i-th matching dispatch is aligned with run 1's i-th."""
import collections
import csv
import glob
import sys

pattern = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else "wino"
runs = []
for path in sorted(glob.glob(pattern)):
    per = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if key not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        per.setdefault(d, {"name": r["Kernel_Name"][:40]})
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    runs.append(list(per.values()))
n = min(len(r) for r in runs)
for i in range(n):
    merged = {}
    for r in runs:
        merged.update(r[i])
    name = merged.pop("name")
    print(f"{i:2d} {name:40s} " + " ".join(f"{k}={v:.3g}" for k, v in sorted(merged.items())))

"""Summarise rocprofv3 --pmc csv files: one row per kernel name (mean over dispatches)."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sys.argv[1:]:
    for path in glob.glob(f, recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(path)):
            per[(r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, k, c), v in per.items():
            agg[k][c].append(v)
for k, cs in agg.items():
    if "wino" not in k and "conv_igemm" not in k:
        continue
    print(k[:70])
    for c, vs in sorted(cs.items()):
        print(f"   {c:36s} {sum(vs) / len(vs):14.4g}")

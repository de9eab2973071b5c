"""Per-kernel PMC summary of the LAST engine step from rocprofv3 --pmc (+ --kernel-trace) passes.

usage: pmc_last_step.py <marker> <pass_dir> [<pass_dir> ...]
Each pass dir holds run_counter_collection.csv (and run_kernel_trace.csv). Dispatches after the
last launch of <marker> (e.g. nchw_to_nhwc_pad) are grouped by kernel name; reported:
mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs) (round-1 formula),
HBM read/write GB/s from FETCH_SIZE / WRITE_SIZE (KB) over the dispatch duration.
"""
import collections
import csv
import glob
import os
import re
import sys


def load(d):
    cnt = collections.defaultdict(dict)
    names = {}
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            i = int(r["Dispatch_Id"])
            names[i] = r["Kernel_Name"]
            cnt[i][r["Counter_Name"]] = cnt[i].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    dur = {}
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return names, cnt, dur


def main(marker, dirs):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    extra = set()
    for d in dirs:
        names, cnt, dur = load(d)
        ids = sorted(names)
        marks = [i for i in ids if any(m in names[i] for m in marker.split("|"))]
        if not marks:
            continue
        for i in ids:
            if i < marks[-1]:
                continue
            k = re.sub(r"\(.*", "", names[i])[:72]
            c = cnt[i]
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
                per[k]["mfma_util"].append(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024))
            us = dur.get(i)
            if us:
                per[k]["us"].append(us)
                if "FETCH_SIZE" in c:
                    per[k]["read_GBs"].append(c["FETCH_SIZE"] * 1024 / (us * 1e-6) / 1e9)
                if "WRITE_SIZE" in c:
                    per[k]["write_GBs"].append(c["WRITE_SIZE"] * 1024 / (us * 1e-6) / 1e9)
            for n in c:
                if n not in ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "FETCH_SIZE", "WRITE_SIZE"):
                    per[k][n].append(c[n])
                    extra.add(n)
    cols = ["us", "mfma_util", "read_GBs", "write_GBs"] + sorted(extra)
    print(f"{'kernel':72s} " + " ".join(f"{c[:12]:>12s}" for c in cols))
    for k, m in sorted(per.items(), key=lambda kv: -sum(kv[1].get("us", [0]))):
        vals = [(sum(m[c]) / len(m[c]) if m.get(c) else float("nan")) for c in cols]
        print(f"{k:72s} " + " ".join(f"{v:12.3g}" for v in vals))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])

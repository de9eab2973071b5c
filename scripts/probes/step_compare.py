"""Side-by-side per-dispatch durations of the last engine step of several rocprofv3 kernel traces
(e.g. TP_WINO_DBG experiments): python scripts/probes/step_compare.py dirA dirB ..."""
import csv
import glob
import re
import sys


def last_step(d, marker="nchw_to_nhwc"):
    path = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    a, b = idx[-2], idx[-1]
    return [(re.sub(r"\(.*", "", r["Kernel_Name"])[:48],
             (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows[a:b]]


def main(dirs):
    steps = [last_step(d) for d in dirs]
    n = min(len(s) for s in steps)
    print(" ".join(f"{d.split('/')[-1]:>10}" for d in dirs) + "  kernel")
    for i in range(n):
        print(" ".join(f"{s[i][1]:10.1f}" for s in steps) + f"  {steps[0][i][0]}")
    print(" ".join(f"{sum(t for _, t in s):10.1f}" for s in steps) + "  total")


if __name__ == "__main__":
    main(sys.argv[1:])

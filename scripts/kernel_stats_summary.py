"""Summarise a rocprofv3 ``*_kernel_stats.csv``: total GPU time per kernel (top N) and the share
of library (non-``tp::``) kernels, e.g. to show a workload runs only on the package's kernels."""
import csv
import re
import sys


def main(path, top=25):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lib = 0.0
    print(f"{'calls':>7} {'total_us':>11} {'share':>6}  kernel")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        name = re.sub(r"\(.*", "", r["Name"])[:100]
        print(f"{r['Calls']:>7} {float(r['TotalDurationNs']) / 1e3:11.1f} {float(r['TotalDurationNs']) / tot:6.1%}  {name}")
    for r in rows:
        if "tp::" not in r["Name"]:
            lib += float(r["TotalDurationNs"])
    libk = sorted({re.sub(r"\(.*", "", r["Name"])[:60] for r in rows if "tp::" not in r["Name"]})
    print(f"total {tot / 1e3:.1f} us; non-tp:: kernels {lib / tot:.1%} of GPU time: {libk}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)

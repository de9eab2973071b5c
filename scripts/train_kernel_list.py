"""Every launch of the LAST training step (rocprofv3 kernel trace of scripts/r50_train_probe.py)
whose name matches a pattern, in launch order: duration, grid, workgroup — per-shape efficiency
of the wgrad / BN kernels. python scripts/train_kernel_list.py trace.csv [pattern]"""
import csv
import re
import sys


def main(path, pat="wgrad|bn_"):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if re.search(r"conv_igemm<\d+, \d+, \d+, \d+, 7,", r["Kernel_Name"])]
    step = rows[idx[-2]:idx[-1]]
    tot = 0.0
    for r in step:
        n = re.sub(r"\(.*", "", r["Kernel_Name"])
        if not re.search(pat, n):
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        g = r.get("Grid_Size") or f"{r.get('Grid_Size_X')}x{r.get('Grid_Size_Y')}x{r.get('Grid_Size_Z')}"
        wg = r.get("Workgroup_Size") or r.get("Workgroup_Size_X")
        print(f"{d:8.1f} us  grid {g:>14}  wg {wg:>5}  {n[:90]}")
    print(f"total {tot:.1f} us")


if __name__ == "__main__":
    main(*sys.argv[1:])

"""Summarise one engine step from a rocprofv3 kernel_trace.csv: the kernels between the last two
occurrences of a marker kernel (default: conv_first), with durations and grid sizes."""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name[:110]


def main(path, marker="conv_first", which=-2):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if any(m in r["Kernel_Name"] for m in marker.split("|"))]
    if len(idx) < 2:
        print("marker not found twice")
        return
    a, b = idx[which], idx[which + 1]
    step = rows[a:b]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = int(rows[b]["Start_Timestamp"])
    busy = 0
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        busy += d
        grid = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])) * int(r["Grid_Size_Y"])
        print(f"{d:9.1f} us  wg={grid:6d}  vgpr={r['VGPR_Count']:>4}  lds={r['LDS_Block_Size']:>6}  {short(r['Kernel_Name'])}")
    print(f"step wall {(t1 - t0) / 1e3:.1f} us, kernel busy {busy:.1f} us, {len(step)} kernels")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3] or []))

"""Kernels of the last complete step in a rocprofv3 kernel trace, where a step starts at each
launch of a marker kernel (default: nchw_to_nhwc_pad, the first kernel of an engine forward):
per-kernel-name time, count and the step's wall/busy time."""
import collections
import csv
import re
import sys


def main(path, marker="nchw_to_nhwc_pad|conv_first_wave", top=30):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if any(m in r["Kernel_Name"] for m in marker.split("|"))]
    a, b = idx[-2], idx[-1]
    step = rows[a:b]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in step:
        n = re.sub(r"\(.*", "", r["Kernel_Name"])
        agg[n][0] += 1
        agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    busy = sum(v[1] for v in agg.values())
    wall = (int(rows[b]["Start_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
    print(f"last step: wall {wall:.1f} us, kernel busy {busy:.1f} us, {len(step)} kernels")
    for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{d:9.1f} us {d / busy:6.1%} {c:4d}x  {n[:110]}")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3] or []))

"""Per-category kernel time of the LAST training step in a rocprofv3 kernel trace of
scripts/r50_train_probe.py (a step starts at the ResNet stem's 7x7 conv kernel)."""
import collections
import csv
import re
import sys


def main(path, top=25):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if re.search(r"conv_igemm<\d+, \d+, \d+, \d+, 7,", r["Kernel_Name"])]
    a, b = idx[-2], idx[-1]
    step = rows[a:b]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in step:
        n = re.sub(r"\(.*", "", r["Kernel_Name"])
        if "conv_igemm" not in n and "conv_wgrad" not in n:
            n = re.sub(r"<.*", "<>", n)
        agg[n][0] += 1
        agg[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    busy = sum(v[1] for v in agg.values())
    wall = (int(rows[b]["Start_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
    print(f"last step: wall {wall:.1f} us, kernel busy {busy:.1f} us, {len(step)} kernels")
    cat = collections.defaultdict(float)
    for n, (c, d) in agg.items():
        k = ("wgrad" if "wgrad" in n else "conv fwd/dgrad" if "conv_igemm" in n else "batchnorm" if "bn_" in n
             else "aten elementwise" if "at::native" in n else "hipBLASLt" if "Cijk" in n else n[:40])
        cat[k] += d
    for k, v in sorted(cat.items(), key=lambda x: -x[1]):
        print(f"{v:10.1f} us {v / busy:6.1%}  {k}")
    for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{d:9.1f} us {c:4d}x  {n[:110]}")


if __name__ == "__main__":
    main(sys.argv[1])

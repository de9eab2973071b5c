"""Pivot a rocprofv3 counter_collection.csv: one row per dispatch of kernels matching a filter,
one column per counter, plus derived clock (GRBM_GUI_ACTIVE/8/duration) and MFMA busy share."""
import csv
import re
import sys
from collections import OrderedDict


def short(n):
    n = re.sub(r"\(.*", "", n)
    return n.replace("void ", "")[:70]


def main(path, filt="conv_igemm"):
    rows = csv.DictReader(open(path))
    disp = OrderedDict()
    for r in rows:
        if filt not in r["Kernel_Name"]:
            continue
        d = disp.setdefault(r["Dispatch_Id"], {"name": short(r["Kernel_Name"]), "grid": int(r["Grid_Size"]) // int(r["Workgroup_Size"]),
                                               "dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
    cols = None
    for k, d in disp.items():
        if cols is None:
            cols = [c for c in d if c not in ("name", "grid", "dur")]
            print("dispatch  dur_us  grid  clkGHz  " + "  ".join(cols) + "  kernel")
        clk = d.get("GRBM_GUI_ACTIVE", 0) / 8 / (d["dur"] * 1e3) if d["dur"] else 0
        extra = ""
        if "SQ_VALU_MFMA_BUSY_CYCLES" in d and "SQ_BUSY_CYCLES" in d and d["SQ_BUSY_CYCLES"]:
            extra = f" mfma/busy={d['SQ_VALU_MFMA_BUSY_CYCLES'] / d['SQ_BUSY_CYCLES']:.3f}"
        vals = "  ".join(f"{d.get(c, 0):.3g}" for c in cols)
        print(f"{k:>8} {d['dur']:7.1f} {d['grid']:5d} {clk:6.2f}  {vals}{extra}  {d['name']}")


if __name__ == "__main__":
    main(sys.argv[1], *(sys.argv[2:3]))

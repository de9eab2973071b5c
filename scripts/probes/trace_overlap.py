"""Kernel overlap in a rocprofv3 kernel trace: over the last ``frac`` of the trace's time span,
the wall span, the summed kernel time, the union of kernel intervals (time with >= 1 kernel
running) and the average number of kernels in flight; plus the per-kernel-name summed time.
Usage: python scripts/probes/trace_overlap.py <kernel_trace.csv> [frac=0.5] [top=15]"""
import collections
import csv
import re
import sys


def main(path, frac=0.5, top=15):
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), re.sub(r"\(.*", "", r["Kernel_Name"]))
            for r in csv.DictReader(open(path))]
    rows.sort()
    t_end = max(e for _, e, _ in rows)
    t_cut = rows[0][0] + (1 - frac) * (t_end - rows[0][0])
    win = [r for r in rows if r[0] >= t_cut]
    lo = win[0][0]
    wall = t_end - lo
    busy = sum(e - s for s, e, _ in win)
    union, cur_s, cur_e = 0, None, None
    for s, e, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    union += cur_e - cur_s
    print(f"window: last {frac:.0%} of the trace, {len(win)} kernels")
    print(f"wall {wall / 1e3:.1f} us, kernel time summed {busy / 1e3:.1f} us, GPU active (union) "
          f"{union / 1e3:.1f} us ({union / wall:.1%} of wall), average kernels in flight while active "
          f"{busy / union:.2f}")
    agg = collections.defaultdict(lambda: [0, 0])
    for s, e, n in win:
        agg[n][0] += 1
        agg[n][1] += e - s
    for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{d / 1e3:10.1f} us {d / busy:6.1%} {c:5d}x  {n[:100]}")


if __name__ == "__main__":
    main(sys.argv[1], *(float(a) if i == 0 else int(a) for i, a in enumerate(sys.argv[2:])))

"""Per-category kernel time of the LAST training step in a rocprofv3 (rocpd sqlite) kernel trace of
a ResNet-50 training probe (a step starts at the stem's 7x7 conv kernel, ``conv_igemm<..., 7, ...>``),
plus the library kernels the native path should not run (MIOpen / ATen BatchNorm, pad / slice /
copy kernels of channel padding).

    python scripts/rocpd_step.py gpurun_out/prof/x_results.db [top]
"""
import collections
import re
import sqlite3
import sys


def rows_of(path):
    c = sqlite3.connect(path)
    return [(n, int(s), int(e)) for n, s, e in c.execute("select name, start, end from kernels order by start")]


def category(n):
    if "wgrad" in n:
        return "wgrad"
    if "wino4" in n or "conv_igemm" in n or "conv_epilogue" in n or "conv_wino" in n:
        return "conv fwd/dgrad"
    if "bn_" in n:
        return "batchnorm (native)"
    if re.search(r"batch_norm|BatchNorm|MIOpenBatchNorm|bn_fwd|bnBwd", n, re.I):
        return "batchnorm (library)"
    if "pack_conv" in n or "weight_transform" in n:
        return "weight packs"
    if re.search(r"constant_pad|CatArray|copy_|direct_copy|elementwise_kernel.*copy", n):
        return "pad/slice/copy (ATen)"
    if "at::native" in n:
        return "aten other"
    return n[:48]


def main(path, top=30):
    rows = rows_of(path)
    idx = [i for i, r in enumerate(rows) if re.search(r"conv_igemm<\d+, \d+, \d+, \d+, 7,", r[0])]
    a, b = idx[-2], idx[-1]
    step = rows[a:b]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for n, s, e in step:
        k = re.sub(r"\(.*", "", n)
        if "conv_igemm" not in k and "conv_wgrad" not in k and "wino4" not in k:
            k = re.sub(r"<.*", "<>", k)
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e3
    busy = sum(v[1] for v in agg.values())
    wall = (rows[b][1] - step[0][1]) / 1e3
    print(f"last step: wall {wall:.1f} us, kernel busy {busy:.1f} us, {len(step)} kernels")
    cat = collections.defaultdict(lambda: [0, 0.0])
    for n, (c, d) in agg.items():
        cat[category(n)][0] += c
        cat[category(n)][1] += d
    for k, (c, v) in sorted(cat.items(), key=lambda x: -x[1][1]):
        print(f"{v:10.1f} us {v / busy:6.1%} {c:4d}x  {k}")
    print("top kernels:")
    for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{d:9.1f} us {c:4d}x  {n[:120]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30)

# wave-uniform first-layer kernel: tests + which first-layer candidate wins + headline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k "first" > gpurun_out/first2_tests.log 2>&1 || { tail -40 gpurun_out/first2_tests.log; exit 1; }
tail -2 gpurun_out/first2_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tr -o run --output-format csv -- python bench.py --steps 4 --warmup 2 --no-prune --no-baseline --teacher-steps 0 > gpurun_out/first2_tr.log 2>&1 || { tail -30 gpurun_out/first2_tr.log; exit 1; }
python - <<'PY' $(find /tmp/tr -name "*kernel_trace.csv" | head -1)
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "conv_first" in n or "wino_f2x3<0, 2>" in n or "nchw_to_nhwc_pad" in n:
        d[n.split("(")[0][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    v = sorted(v)
    print(f"{k:60s} n={len(v):4d} median {v[len(v)//2]:8.1f} us  min {v[0]:8.1f}")
PY
rm -rf /tmp/tr
timeout -k 10 300 python -u bench.py --no-prune --no-baseline > gpurun_out/first2_bench.log 2>&1 || { tail -30 gpurun_out/first2_bench.log; exit 1; }
grep "\[bench\] 1 GPU" gpurun_out/first2_bench.log

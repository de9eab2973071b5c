# final headline profile: rocprofv3 --kernel-trace --stats over a pipelined B=2048 run (stats kept,
# raw traces dropped) + the overlap of the two streams (sum of kernel time vs wall of the timed run)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/fp -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-prune --no-baseline --teacher-steps 0 > gpurun_out/final_prof.log 2>&1 || { tail -30 gpurun_out/final_prof.log; exit 1; }
python scripts/kernel_stats_summary.py $(find /tmp/fp -name "*kernel_stats.csv" | head -1) > gpurun_out/final_kernel_stats.txt
python - <<'PY' $(find /tmp/fp -name "*kernel_trace.csv" | head -1) >> gpurun_out/final_kernel_stats.txt
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "nchw_to_nhwc_pad" in r["Kernel_Name"]]
seg = rows[marks[-20]:]  # the timed run's 20 batches (first-layer launches)
t0 = int(seg[0]["Start_Timestamp"]); t1 = max(int(r["End_Timestamp"]) for r in seg)
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
print(f"timed run (20 batches): wall {(t1 - t0) / 1e3:.1f} us, sum of kernel durations {busy / 1e3:.1f} us "
      f"(> wall: kernels of the two streams overlap), {len(seg)} launches")
PY
rm -rf /tmp/fp
grep "\[bench\] 1 GPU" gpurun_out/final_prof.log
tail -3 gpurun_out/final_kernel_stats.txt

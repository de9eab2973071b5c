# Is the in-engine dgrad slowdown data-dependent? headline step trace with an untrained vs trained teacher
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for ts in 0 1500; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/tt$ts -o run --output-format csv -- python bench.py --steps 6 --warmup 2 --no-prune --no-baseline --teacher-steps $ts > gpurun_out/tt$ts.log 2>&1 || { tail -30 gpurun_out/tt$ts.log; exit 1; }
  python scripts/trace_step.py $(find gpurun_out/tt$ts -name "*kernel_trace.csv" | head -1) nchw_to_nhwc_pad 40 > gpurun_out/tt${ts}_step.txt
  head -30 gpurun_out/tt${ts}_step.txt
done

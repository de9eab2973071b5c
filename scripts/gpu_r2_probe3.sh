# headline step trace (ordered kernels with grids) at B=2048 and B=100, traces deleted after summarising
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for B in 2048 100; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tr$B -o run --output-format csv -- python bench.py --batch $B --steps 8 --warmup 2 --no-prune --no-baseline > gpurun_out/tr$B.log 2>&1 || { tail -30 gpurun_out/tr$B.log; exit 1; }
  python scripts/trace_step.py $(find /tmp/tr$B -name "*kernel_trace.csv" | head -1) nchw_to_nhwc_pad > gpurun_out/step_b$B.txt
  python scripts/step_breakdown.py $(find /tmp/tr$B -name "*kernel_trace.csv" | head -1) > gpurun_out/stepagg_b$B.txt
  rm -rf /tmp/tr$B
done

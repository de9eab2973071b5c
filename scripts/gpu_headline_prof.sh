# Headline step profile: bench (no extras) with tuner log, then a rocprofv3 kernel trace of the
# same run with one batch in flight (TORCHPRUNER_STREAMS=0: per-kernel times without overlap)
# and with the default two-stream pipeline; last-step breakdowns of both.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
TORCHPRUNER_TUNER_LOG=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-extras --no-prune --no-baseline --teacher-steps 0 > gpurun_out/hb.json 2> gpurun_out/hb.log || { tail -30 gpurun_out/hb.log; exit 1; }
grep "\[bench\]" gpurun_out/hb.log; grep "\[tuner\]" gpurun_out/hb.log | sort | uniq | head -60
cd /tmp && export TMPDIR=/tmp
for s in 0 1; do
  TORCHPRUNER_STREAMS=$s timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/hprof$s -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 --no-extras --no-prune --no-baseline --teacher-steps 0 > $R/gpurun_out/hprof$s.log 2>&1 || { tail -30 $R/gpurun_out/hprof$s.log; exit 1; }
  f=$(find $R/gpurun_out/hprof$s -name '*kernel_trace.csv' | head -1)
  echo "== streams=$s"; python3 $R/scripts/step_breakdown.py $f
done

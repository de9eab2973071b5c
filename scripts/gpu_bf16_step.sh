# Kernel breakdown of one opt-in bf16 engine step (B=2048) and of one fp32 step, one batch in flight.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bf16step
mkdir -p $O
for mode in bf16 fp32; do
  extra=""; [ $mode = fp32 ] && extra="--fp32"
  TORCHPRUNER_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$mode -o run --output-format csv -- python3 $R/scripts/probes/bf16_step_probe.py --steps 3 $extra > $O/$mode.log 2>&1 || { tail -20 $O/$mode.log; exit 1; }
  f=$(find $O/$mode -name '*kernel_trace.csv' | head -1)
  echo "== $mode"; python3 $R/scripts/step_breakdown.py $f
done

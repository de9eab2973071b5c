# ResNet-50 B=256 APoZ and Taylor engine steps (one batch in flight): last-step kernel breakdowns.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_rn2
mkdir -p $O
for metric in apoz taylor; do
  PYTHONPATH=$R TORCHPRUNER_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/$metric -o run --output-format csv -- python3 -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 3 --warmup 1 --metric $metric > $O/$metric.log 2>&1 || { tail -20 $O/$metric.log; exit 1; }
  f=$(find $O/$metric -name '*kernel_trace.csv' | head -1)
  echo "== $metric"; python3 $R/scripts/step_breakdown.py $f "nchw_to_nhwc_pad"
done

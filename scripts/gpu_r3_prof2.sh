#!/bin/bash
# Kernel traces: B=100 headline-variant step and the ResNet-50 Taylor/APoZ steps (B=256)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof2
mkdir -p $O
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/b100 -o run --output-format csv -- python3 $R/bench.py --batch 100 --steps 50 --warmup 10 --no-baseline --no-prune --no-extras --teacher-steps 0 > $O/b100.log 2>&1 || { echo "b100 failed"; tail -5 $O/b100.log; exit 1; }
python3 $R/scripts/step_breakdown.py $O/b100 nchw_to_nhwc_pad > $R/gpurun_out/b100_step_breakdown.txt 2>&1 || true
for m in taylor apoz; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/rn_$m -o run --output-format csv -- python3 -m torchpruner_amd.bench.resnet50_apoz --metric $m --steps 4 --warmup 2 > $O/rn_$m.log 2>&1 || { echo "resnet $m failed"; tail -5 $O/rn_$m.log; exit 2; }
  python3 $R/scripts/step_breakdown.py $O/rn_$m nchw_to_nhwc_pad > $R/gpurun_out/rn_${m}_step_breakdown.txt 2>&1 || true
done
cat $R/gpurun_out/b100_step_breakdown.txt | head -30
cat $R/gpurun_out/rn_taylor_step_breakdown.txt | head -25

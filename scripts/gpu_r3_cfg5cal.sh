#!/bin/bash
# Config #5 calibration: teacher accuracy / method separation for a few task difficulties (1 seed),
# then the B=100 headline-variant bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3
for cfg in ${CFG5_LIST:-"8 2.5" "16 3.0" "16 4.0"}; do
  set -- $cfg
  timeout -k 10 240 python -u experiments/prune_finetune.py --compare taylor,apoz,random --seeds 0 --modes $1 --noise $2 \
      --rounds 3 --pretrain-steps 150 --steps 30 > gpurun_out/r3/cfg5_m$1_n$2.log 2>&1 || { tail -20 gpurun_out/r3/cfg5_m$1_n$2.log; exit 1; }
  grep -E "pretrain_steps|summary" gpurun_out/r3/cfg5_m$1_n$2.log
done
timeout -k 10 300 python bench.py --batch 100 --steps 200 --warmup 10 --no-baseline --no-prune --no-extras --teacher-steps 0 > gpurun_out/r3/b100.json 2> gpurun_out/r3/b100.err || { tail -30 gpurun_out/r3/b100.err; exit 3; }
cat gpurun_out/r3/b100.json

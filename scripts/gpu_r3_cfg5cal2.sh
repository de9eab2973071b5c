#!/bin/bash
# Config #5 calibration 2: easier settings (classes, modes, noise, pretrain steps), 1 seed each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3
for cfg in ${CFG5_LIST:-"20 4 2.0 300" "20 8 2.5 300" "100 2 1.5 300" "10 8 3.0 300"}; do
  set -- $cfg
  timeout -k 10 300 python -u experiments/prune_finetune.py --compare taylor,apoz,random --seeds 0 --classes $1 --modes $2 --noise $3 \
      --rounds 3 --pretrain-steps $4 --steps 30 > gpurun_out/r3/cfg5_c$1_m$2_n$3.log 2>&1 || { tail -20 gpurun_out/r3/cfg5_c$1_m$2_n$3.log; exit 1; }
  echo "== classes $1 modes $2 noise $3"
  grep -E "pretrain_steps" gpurun_out/r3/cfg5_c$1_m$2_n$3.log
  grep summary gpurun_out/r3/cfg5_c$1_m$2_n$3.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())['summary']
for m,rs in d.items(): print(m, [(r['after_prune_mean'], r['after_finetune_mean']) for r in rs])"
done

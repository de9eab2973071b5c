#!/bin/bash
# Config #5 at ImageNet shape (224 px): ResNet-50 iterative prune -> finetune, Taylor vs APoZ vs
# Random from one unsaturated teacher per seed (3 seeds), PrunableDDP, 3 rounds of 20%
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/cfg5_224
timeout -k 10 1000 python -u experiments/prune_finetune.py --compare taylor,apoz,random --seeds 0,1,2 --classes 20 --modes 8 \
    --noise 2.5 --teacher-target 0.85 --pretrain-steps 400 --check-every 20 --rounds 3 --steps 15 --val-batches 8 --res 224 \
    > gpurun_out/cfg5_224/cfg5.log 2>&1 || { tail -20 gpurun_out/cfg5_224/cfg5.log; exit 1; }
grep -E "pretrain_steps|summary" gpurun_out/cfg5_224/cfg5.log | cut -c1-1500

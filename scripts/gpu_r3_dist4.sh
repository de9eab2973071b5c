#!/bin/bash
# 4 self-launched ranks sharing the GPU over gloo: bench.py --gpus 4 with every extra (sharded
# ResNet / Shapley / generic path) and the default graph-replay pipeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/dist4
export TORCHPRUNER_DIST_BACKEND=gloo TORCHPRUNER_SHARE_GPU=1
timeout -k 10 900 python bench.py --gpus 4 --steps 3 --warmup 1 --batch 512 --no-prune --teacher-steps 50 --resnet-steps 2 --generic-steps 1 > gpurun_out/dist4/bench.json 2> gpurun_out/dist4/bench.err || { tail -40 gpurun_out/dist4/bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/dist4/bench.err | tail -8
cut -c1-900 gpurun_out/dist4/bench.json

#!/bin/bash
# B=100 / 256 with graph replay: pipeline depth 2 / 3 / 4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/depth
for b in 100 256; do
for d in 2 3 4 2 3 4; do
TORCHPRUNER_STREAMS_DEPTH=$d timeout -k 10 300 python bench.py --batch $b --steps 200 --warmup 20 --no-prune --no-extras --no-baseline --teacher-steps 0 > gpurun_out/depth/b${b}_d$d.json 2> gpurun_out/depth/b${b}_d$d.err || { tail -20 gpurun_out/depth/b${b}_d$d.err; exit 3; }
echo "B=$b depth $d: $(grep '\[bench\] 1 GPU' gpurun_out/depth/b${b}_d$d.err)"
done
done

#!/bin/bash
# B=100 extra after the B=2048 runs: graph replay at B=2048 (default) vs not (GRAPH_MAX_B=1024)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/interf
for m in 4096 1024; do
TORCHPRUNER_GRAPH_MAX_B=$m timeout -k 10 600 python -u bench.py --no-prune --no-baseline --generic-steps 1 > gpurun_out/interf/b_$m.json 2> gpurun_out/interf/b_$m.err || { tail -30 gpurun_out/interf/b_$m.err; exit 4; }
echo "GRAPH_MAX_B=$m"; grep -E "B=2048|B=100|bf16" gpurun_out/interf/b_$m.err
done

#!/bin/bash
# B=2048: eager 2 in flight (default) vs pipelined graph replay (TORCHPRUNER_GRAPH_MAX_B=2048) at depth 4 / 2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/bigb2
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-prune --no-extras --no-baseline --teacher-steps 0 --steps 40 --warmup 8 > gpurun_out/bigb2/$name.json 2> gpurun_out/bigb2/$name.err || { tail -20 gpurun_out/bigb2/$name.err; exit 3; }
  echo "$name: $(grep '\[bench\] 1 GPU' gpurun_out/bigb2/$name.err)"
}
for rep in 1 2; do
run default_$rep TORCHPRUNER_GRAPHS=auto
run pipe_graphs_d4_$rep TORCHPRUNER_GRAPH_MAX_B=2048
run pipe_graphs_d2_$rep TORCHPRUNER_GRAPH_MAX_B=2048 TORCHPRUNER_STREAMS_DEPTH=2
done

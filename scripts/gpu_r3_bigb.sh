#!/bin/bash
# large batches: eager depth 2 (default) vs graph replay depth 4 (B=1024 default, B=2048 forced)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/bigb
run() {  # name, env..., then bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-prune --no-extras --no-baseline --teacher-steps 0 --steps 40 --warmup 8 $BARGS > gpurun_out/bigb/$name.json 2> gpurun_out/bigb/$name.err || { tail -20 gpurun_out/bigb/$name.err; exit 3; }
  echo "$name: $(grep '\[bench\] 1 GPU' gpurun_out/bigb/$name.err)"
}
for rep in 1 2; do
BARGS="--batch 2048" run b2048_default_$rep TORCHPRUNER_GRAPHS=auto
BARGS="--batch 2048" run b2048_graphs_d4_$rep TORCHPRUNER_GRAPHS=all TORCHPRUNER_STREAMS_DEPTH=4
BARGS="--batch 2048" run b2048_graphs_d2_$rep TORCHPRUNER_GRAPHS=all TORCHPRUNER_STREAMS_DEPTH=2
BARGS="--batch 2048" run b2048_eager_d3_$rep TORCHPRUNER_GRAPHS=0 TORCHPRUNER_STREAMS_DEPTH=3
BARGS="--batch 1024" run b1024_default_$rep TORCHPRUNER_GRAPHS=auto
done

#!/bin/bash
# depth heuristic check: B=512 / 1024 default vs forced depth
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/midb
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graphs_gpu.py > gpurun_out/midb/tests.log 2>&1 || { tail -40 gpurun_out/midb/tests.log; exit 1; }
tail -1 gpurun_out/midb/tests.log
run() {
  local name=$1 b=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --batch $b --no-prune --no-extras --no-baseline --teacher-steps 0 --steps 60 --warmup 12 > gpurun_out/midb/$name.json 2> gpurun_out/midb/$name.err || { tail -20 gpurun_out/midb/$name.err; exit 3; }
  echo "$name: $(grep '\[bench\] 1 GPU' gpurun_out/midb/$name.err)"
}
for rep in 1 2; do
run b512_default_$rep 512 TORCHPRUNER_GRAPHS=auto
run b512_d2_$rep 512 TORCHPRUNER_STREAMS_DEPTH=2
run b1024_default_$rep 1024 TORCHPRUNER_GRAPHS=auto
run b1024_d4_$rep 1024 TORCHPRUNER_STREAMS_DEPTH=4
run b1024_d3_$rep 1024 TORCHPRUNER_STREAMS_DEPTH=3
done

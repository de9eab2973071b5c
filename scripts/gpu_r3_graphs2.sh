#!/bin/bash
# default pipeline depth 4 with graph replay: graph/pipeline GPU tests, B=100/256/2048 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/graphs2
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graphs_gpu.py > gpurun_out/graphs2/tests.log 2>&1 || { tail -40 gpurun_out/graphs2/tests.log; exit 1; }
tail -2 gpurun_out/graphs2/tests.log
for b in 100 100 256; do
timeout -k 10 300 python bench.py --batch $b --steps 200 --warmup 20 --no-prune --no-extras --no-baseline --teacher-steps 0 > gpurun_out/graphs2/b$b.json 2> gpurun_out/graphs2/b$b.err || { tail -20 gpurun_out/graphs2/b$b.err; exit 3; }
grep "\[bench\] 1 GPU" gpurun_out/graphs2/b$b.err
done

#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/last
timeout -k 10 400 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_graphs_gpu.py tests/test_conv_gpu.py tests/test_mlp_engine_gpu.py > gpurun_out/last/tests.log 2>&1 || { tail -40 gpurun_out/last/tests.log; exit 1; }
tail -1 gpurun_out/last/tests.log
timeout -k 10 300 python bench.py --batch 100 --steps 200 --warmup 20 --no-prune --no-extras --no-baseline --teacher-steps 0 > gpurun_out/last/b100.json 2> gpurun_out/last/b100.err || { tail -20 gpurun_out/last/b100.err; exit 3; }
grep '\[bench\] 1 GPU' gpurun_out/last/b100.err

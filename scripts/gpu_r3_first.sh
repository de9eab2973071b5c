#!/bin/bash
# round 3, first GPU pass: the new launcher / DP / MLP-shape tests, then the full 1-GPU bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_bench_gpu.py tests/test_dist_gpu.py tests/test_mlp_engine_gpu.py > gpurun_out/r3/t1.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r3/bench1.json 2> gpurun_out/r3/bench1.err

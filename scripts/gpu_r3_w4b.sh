#!/bin/bash
# F(4x4) iteration: numerics + per-layer timing vs F(2x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wino4_gpu.py \
    > gpurun_out/r3/w4_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/wino4_bench.py --batch 2048 > gpurun_out/r3/w4_bench.log 2>&1

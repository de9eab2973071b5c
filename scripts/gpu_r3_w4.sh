#!/bin/bash
# round 3: F(4x4) kernel numerics + per-layer timing vs F(2x2), then the launcher / DP tests and the bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wino4_gpu.py \
    > gpurun_out/r3/w4_tests.log 2>&1
rc=$?
if [ $rc -eq 0 ]; then
  timeout -k 10 300 python -u scripts/wino4_bench.py --batch 2048 > gpurun_out/r3/w4_bench.log 2>&1 || exit $?
fi
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 420 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_bench_gpu.py tests/test_dist_gpu.py tests/test_mlp_engine_gpu.py > gpurun_out/r3/t1.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r3/bench1.json 2> gpurun_out/r3/bench1.err

#!/bin/bash
# bf16 opt-in path: GPU tests, then the default bench (which reports the bf16 extra)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bf16_gpu.py > gpurun_out/r3/bf16_tests.log 2>&1 || { tail -40 gpurun_out/r3/bf16_tests.log; exit 1; }
tail -3 gpurun_out/r3/bf16_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3/bench_bf16.json 2> gpurun_out/r3/bench_bf16.err || { tail -30 gpurun_out/r3/bench_bf16.err; exit 2; }
grep "\[bench\]" gpurun_out/r3/bench_bf16.err

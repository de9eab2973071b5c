#!/bin/bash
# Full GPU test suite, then the driver's default bench (N=1, with extras); logs under gpurun_out/r3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3
timeout -k 10 900 python -u -m pytest --maxfail=25 -v --timeout 180 --timeout-method thread -m gpu tests/ > gpurun_out/r3/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r3/gpu_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3/bench_full.json 2> gpurun_out/r3/bench_full.err || { tail -30 gpurun_out/r3/bench_full.err; exit 2; }
cat gpurun_out/r3/bench_full.json

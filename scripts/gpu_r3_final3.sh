#!/bin/bash
# round-end style validation: full GPU suite, smoke(), default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/final3
timeout -k 10 900 python -u -m pytest --maxfail=25 -v --timeout 180 --timeout-method thread -m gpu tests/ > gpurun_out/final3/gpu_tests.log 2>&1 || { tail -40 gpurun_out/final3/gpu_tests.log; exit 1; }
tail -1 gpurun_out/final3/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final3/smoke.log 2>&1 || { tail -20 gpurun_out/final3/smoke.log; exit 2; }
tail -1 gpurun_out/final3/smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/final3/bench.json 2> gpurun_out/final3/bench.err || { tail -30 gpurun_out/final3/bench.err; exit 3; }
grep -v amdgpu.ids gpurun_out/final3/bench.err

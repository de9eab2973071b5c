#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/inval
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graphs_gpu.py > gpurun_out/inval/tests.log 2>&1 || { tail -40 gpurun_out/inval/tests.log; exit 1; }
tail -3 gpurun_out/inval/tests.log

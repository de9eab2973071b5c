#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/rnsens
timeout -k 10 500 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_resnet_bwd_gpu.py tests/test_resnet_engine_gpu.py tests/test_dist_gpu.py tests/test_pruned_engine_gpu.py > gpurun_out/rnsens/tests.log 2>&1 || { tail -40 gpurun_out/rnsens/tests.log; exit 1; }
tail -1 gpurun_out/rnsens/tests.log

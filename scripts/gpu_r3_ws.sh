#!/bin/bash
# warp-specialised 1x1 GEMM: GPU tests, then the ResNet-50 per-shape roofline with the new cfgs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ws
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_ws_gpu.py > gpurun_out/ws/tests.log 2>&1 || { tail -40 gpurun_out/ws/tests.log; exit 1; }
tail -3 gpurun_out/ws/tests.log
timeout -k 10 400 python -u scripts/r50_conv_roofline.py --ws --verbose > gpurun_out/ws/roofline.txt 2>&1 || { tail -30 gpurun_out/ws/roofline.txt; exit 2; }
cat gpurun_out/ws/roofline.txt

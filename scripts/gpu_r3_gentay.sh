#!/bin/bash
# 1x1 dgrad Taylor partials (EPI_FWD_TAY): kernel tests, ResNet engine tests, timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/gentay
timeout -k 10 500 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_resnet_bwd_gpu.py tests/test_resnet_engine_gpu.py tests/test_dist_gpu.py > gpurun_out/gentay/tests.log 2>&1 || { tail -40 gpurun_out/gentay/tests.log; exit 1; }
tail -1 gpurun_out/gentay/tests.log
for rep in 1 2; do
timeout -k 10 300 python -u scripts/host_probe.py resnet-taylor --batch 256 > gpurun_out/gentay/tay_$rep.txt 2>&1 || { tail -20 gpurun_out/gentay/tay_$rep.txt; exit 2; }
grep "rep [12]" gpurun_out/gentay/tay_$rep.txt | cut -c1-100
done

#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/svg
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graphs_gpu.py > gpurun_out/svg/tests.log 2>&1 || { tail -40 gpurun_out/svg/tests.log; exit 1; }
tail -2 gpurun_out/svg/tests.log
for l in 0 6; do
timeout -k 10 200 python -u scripts/host_probe.py shapley --layer $l > gpurun_out/svg/shapley_$l.txt 2>&1 || { tail -20 gpurun_out/svg/shapley_$l.txt; exit 4; }
grep rep gpurun_out/svg/shapley_$l.txt | cut -c1-130
done
timeout -k 10 300 python -u -m torchpruner_amd.bench.shapley_vgg > gpurun_out/svg/bench.txt 2>&1 || { tail -20 gpurun_out/svg/bench.txt; exit 5; }
grep layer gpurun_out/svg/bench.txt

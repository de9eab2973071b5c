#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/apozg
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graphs_gpu.py > gpurun_out/apozg/tests.log 2>&1 || { tail -40 gpurun_out/apozg/tests.log; exit 1; }
tail -2 gpurun_out/apozg/tests.log
timeout -k 10 200 python -u scripts/host_probe.py apoz --batch 100 > gpurun_out/apozg/apoz.txt 2>&1 || { tail -20 gpurun_out/apozg/apoz.txt; exit 2; }
grep rep gpurun_out/apozg/apoz.txt | cut -c1-150
timeout -k 10 200 python -u scripts/host_probe.py taylor --batch 100 > gpurun_out/apozg/taylor.txt 2>&1 || { tail -20 gpurun_out/apozg/taylor.txt; exit 3; }
grep rep gpurun_out/apozg/taylor.txt | cut -c1-150
for l in 0 6; do
timeout -k 10 200 python -u scripts/host_probe.py shapley --layer $l > gpurun_out/apozg/shapley_$l.txt 2>&1 || { tail -20 gpurun_out/apozg/shapley_$l.txt; exit 4; }
grep rep gpurun_out/apozg/shapley_$l.txt | cut -c1-150
done
for d in 2 3; do
TORCHPRUNER_STREAMS_DEPTH=$d timeout -k 10 300 python -u scripts/host_probe.py resnet-taylor --batch 256 > gpurun_out/apozg/rn_tay_d$d.txt 2>&1 || { tail -20 gpurun_out/apozg/rn_tay_d$d.txt; exit 5; }
echo "depth $d"; grep rep gpurun_out/apozg/rn_tay_d$d.txt | cut -c1-120
TORCHPRUNER_STREAMS_DEPTH=$d timeout -k 10 300 python -u scripts/host_probe.py resnet-apoz --batch 256 > gpurun_out/apozg/rn_apoz_d$d.txt 2>&1 || { tail -20 gpurun_out/apozg/rn_apoz_d$d.txt; exit 6; }
grep rep gpurun_out/apozg/rn_apoz_d$d.txt | cut -c1-120
done

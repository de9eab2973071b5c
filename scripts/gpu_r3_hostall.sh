#!/bin/bash
# host-boundness of the other attribution paths (Shapley layers 0/6/12, APoZ B=100, ResNet B=256)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/hostall
for l in 0 6 12; do
timeout -k 10 200 python -u scripts/host_probe.py shapley --layer $l > gpurun_out/hostall/shapley_$l.txt 2>&1 || { tail -20 gpurun_out/hostall/shapley_$l.txt; exit 1; }
grep rep gpurun_out/hostall/shapley_$l.txt
done
timeout -k 10 200 python -u scripts/host_probe.py apoz --batch 100 > gpurun_out/hostall/apoz.txt 2>&1 || { tail -20 gpurun_out/hostall/apoz.txt; exit 2; }
grep rep gpurun_out/hostall/apoz.txt
timeout -k 10 300 python -u scripts/host_probe.py resnet-apoz --batch 256 > gpurun_out/hostall/rn_apoz.txt 2>&1 || { tail -20 gpurun_out/hostall/rn_apoz.txt; exit 3; }
grep rep gpurun_out/hostall/rn_apoz.txt
timeout -k 10 300 python -u scripts/host_probe.py resnet-taylor --batch 256 > gpurun_out/hostall/rn_tay.txt 2>&1 || { tail -20 gpurun_out/hostall/rn_tay.txt; exit 4; }
grep rep gpurun_out/hostall/rn_tay.txt

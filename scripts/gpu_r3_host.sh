#!/bin/bash
# host-boundness probe of the B=100 fused-engine step (default 2 streams, depth 3, 1 stream)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/host
timeout -k 10 200 python -u scripts/b100_host_probe.py > gpurun_out/host/d2.txt 2>&1 || { tail -20 gpurun_out/host/d2.txt; exit 1; }
cat gpurun_out/host/d2.txt
TORCHPRUNER_STREAMS_DEPTH=3 timeout -k 10 200 python -u scripts/b100_host_probe.py > gpurun_out/host/d3.txt 2>&1 || { tail -20 gpurun_out/host/d3.txt; exit 1; }
cat gpurun_out/host/d3.txt
TORCHPRUNER_STREAMS=0 timeout -k 10 200 python -u scripts/b100_host_probe.py > gpurun_out/host/s1.txt 2>&1 || { tail -20 gpurun_out/host/s1.txt; exit 1; }
cat gpurun_out/host/s1.txt

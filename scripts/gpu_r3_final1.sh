#!/bin/bash
# default bench with every extra (incl. the B=100 figure), then the 4-rank shared-GPU rehearsal
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/final1
timeout -k 10 600 python -u bench.py > gpurun_out/final1/bench.json 2> gpurun_out/final1/bench.err || { tail -30 gpurun_out/final1/bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/final1/bench.err
bash scripts/gpu_r3_dist4.sh

#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/dgroof
timeout -k 10 400 python -u scripts/r50_dgrad_roofline.py --verbose > gpurun_out/dgroof/dgrad.txt 2>&1 || { tail -30 gpurun_out/dgroof/dgrad.txt; exit 1; }
cat gpurun_out/dgroof/dgrad.txt

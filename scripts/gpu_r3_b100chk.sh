#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/b100chk
for rep in 1 2; do
timeout -k 10 300 python bench.py --batch 100 --steps 200 --warmup 20 --no-prune --no-extras --no-baseline --teacher-steps 0 > gpurun_out/b100chk/b100_$rep.json 2> gpurun_out/b100chk/b100_$rep.err || { tail -20 gpurun_out/b100chk/b100_$rep.err; exit 3; }
echo "standalone B=100: $(grep '\[bench\] 1 GPU' gpurun_out/b100chk/b100_$rep.err)"
done
timeout -k 10 200 python -u scripts/b100_host_probe.py > gpurun_out/b100chk/probe.txt 2>&1 || { tail -20 gpurun_out/b100chk/probe.txt; exit 2; }
grep rep gpurun_out/b100chk/probe.txt

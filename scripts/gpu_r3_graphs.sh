#!/bin/bash
# per-slot graph replay in the stream pipeline: GPU tests, host probe, B=100 bench x2, headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/graphs
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_graphs_gpu.py tests/test_gemm_ws_gpu.py > gpurun_out/graphs/tests.log 2>&1 || { tail -40 gpurun_out/graphs/tests.log; exit 1; }
tail -2 gpurun_out/graphs/tests.log
timeout -k 10 200 python -u scripts/b100_host_probe.py > gpurun_out/graphs/probe.txt 2>&1 || { tail -20 gpurun_out/graphs/probe.txt; exit 2; }
cat gpurun_out/graphs/probe.txt
for i in 1 2; do
timeout -k 10 300 python bench.py --batch 100 --steps 200 --warmup 20 --no-prune --no-extras --no-baseline --teacher-steps 0 > gpurun_out/graphs/b100_$i.json 2> gpurun_out/graphs/b100_$i.err || { tail -20 gpurun_out/graphs/b100_$i.err; exit 3; }
grep "\[bench\] 1 GPU" gpurun_out/graphs/b100_$i.err
done
for b in 256 512; do
timeout -k 10 300 python bench.py --batch $b --steps 50 --warmup 10 --no-prune --no-extras --no-baseline --teacher-steps 0 > gpurun_out/graphs/b$b.json 2> gpurun_out/graphs/b$b.err || { tail -20 gpurun_out/graphs/b$b.err; exit 4; }
grep "\[bench\] 1 GPU" gpurun_out/graphs/b$b.err
done
timeout -k 10 300 python bench.py --no-prune --no-extras --no-baseline > gpurun_out/graphs/b2048.json 2> gpurun_out/graphs/b2048.err || { tail -20 gpurun_out/graphs/b2048.err; exit 5; }
grep "\[bench\] 1 GPU" gpurun_out/graphs/b2048.err

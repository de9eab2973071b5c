#!/bin/bash
# B=100 (the reference's attribution batch) step trace at HEAD + bench spread (default / depth 3)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/b100
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/b100/tr -o run --output-format csv -- python bench.py --batch 100 --steps 20 --warmup 5 --no-prune --no-extras --no-baseline --teacher-steps 0 > gpurun_out/b100/trace.log 2>&1 || { tail -30 gpurun_out/b100/trace.log; exit 1; }
python scripts/trace_step.py $(find gpurun_out/b100/tr -name "*kernel_trace.csv" | head -1) > gpurun_out/b100/step.txt
head -40 gpurun_out/b100/step.txt
python scripts/step_breakdown.py $(find gpurun_out/b100/tr -name "*kernel_trace.csv" | head -1) > gpurun_out/b100/breakdown.txt 2>&1 || true
for i in 1 2; do
timeout -k 10 300 python bench.py --batch 100 --steps 200 --warmup 20 --no-prune --no-extras --no-baseline --teacher-steps 0 > gpurun_out/b100/bench_$i.json 2> gpurun_out/b100/bench_$i.err || { tail -20 gpurun_out/b100/bench_$i.err; exit 2; }
grep "\[bench\] 1 GPU" gpurun_out/b100/bench_$i.err
done
TORCHPRUNER_STREAMS_DEPTH=3 timeout -k 10 300 python bench.py --batch 100 --steps 200 --warmup 20 --no-prune --no-extras --no-baseline --teacher-steps 0 > gpurun_out/b100/bench_d3.json 2> gpurun_out/b100/bench_d3.err || { tail -20 gpurun_out/b100/bench_d3.err; exit 3; }
grep "\[bench\] 1 GPU" gpurun_out/b100/bench_d3.err

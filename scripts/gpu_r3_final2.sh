#!/bin/bash
# graph-replay defaults (captured on a slot's first batch, B <= 4096, depth 4 only <= 2^18 px):
# graph tests, headline timing spread, then the full default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/final2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graphs_gpu.py tests/test_compute_dtype.py > gpurun_out/final2/tests.log 2>&1 || { tail -40 gpurun_out/final2/tests.log; exit 1; }
tail -1 gpurun_out/final2/tests.log
for rep in 1 2; do
for g in auto 0; do
TORCHPRUNER_GRAPHS=$g timeout -k 10 300 python bench.py --no-prune --no-extras --no-baseline --teacher-steps 0 > gpurun_out/final2/h_${g}_$rep.json 2> gpurun_out/final2/h_${g}_$rep.err || { tail -20 gpurun_out/final2/h_${g}_$rep.err; exit 3; }
echo "graphs=$g: $(grep '\[bench\] 1 GPU' gpurun_out/final2/h_${g}_$rep.err)"
done
done
timeout -k 10 600 python -u bench.py > gpurun_out/final2/bench.json 2> gpurun_out/final2/bench.err || { tail -30 gpurun_out/final2/bench.err; exit 4; }
grep -v amdgpu.ids gpurun_out/final2/bench.err

#!/bin/bash
# B=100 A/B: F(4x4) split-K candidates on / off, two runs each (the launch-bound step is noisy)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wino4_gpu.py > gpurun_out/r3/w4split_tests.log 2>&1 || { tail -15 gpurun_out/r3/w4split_tests.log; exit 1; }
tail -1 gpurun_out/r3/w4split_tests.log
for r in 1 2; do
  for sp in 1 0; do
    TORCHPRUNER_W4_SPLITS=$sp timeout -k 10 200 python bench.py --batch 100 --steps 300 --warmup 20 --no-baseline --no-prune --no-extras --teacher-steps 0 > gpurun_out/r3/b100_sp${sp}_$r.json 2>/dev/null || exit 2
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('splits', sys.argv[2], 'run', sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/r3/b100_sp${sp}_$r.json $sp $r
  done
done

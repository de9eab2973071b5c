#!/bin/bash
# F(4x4) variants: numerics and per-layer timing for each kernel mode (TP_W4_MODE)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3
rm -f gpurun_out/r3/w4_modes.log
for m in ${W4_MODES:-0 1}; do
  TP_W4_MODE=$m timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wino4_gpu.py \
      > gpurun_out/r3/w4_tests_m$m.log 2>&1 || exit $?
  echo "== TP_W4_MODE=$m" >> gpurun_out/r3/w4_modes.log
  TP_W4_MODE=$m timeout -k 10 200 python -u scripts/wino4_bench.py --batch 2048 --iters 5 >> gpurun_out/r3/w4_modes.log 2>&1 || exit $?
done

#!/bin/bash
# F(4x4) phase attribution: per-layer timing with phases switched off (TP_W4_DBG bits)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wino4_gpu.py \
    > gpurun_out/r3/w4_tests.log 2>&1 || exit $?
for d in ${W4_DBG_LIST:-0 3 16 19}; do
  echo "== TP_W4_DBG=$d" >> gpurun_out/r3/w4_dbg.log
  TP_W4_DBG=$d timeout -k 10 200 python -u scripts/wino4_bench.py --batch 2048 --iters 5 >> gpurun_out/r3/w4_dbg.log 2>&1 || exit $?
done

# Round-2 multi-rank check on the 1-GPU box: the gpu-marked DP engine test (2 and 3 ranks,
# gloo, shared GPU), the full GPU suite, then bench.py under torchrun at 2 and 4 ranks.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -x -v -s --timeout 250 --timeout-method thread > gpurun_out/dist_gpu_test.log 2>&1 || { tail -60 gpurun_out/dist_gpu_test.log; exit 1; }
grep -E "DIST_GPU_OK|max_rel_err|passed|failed" gpurun_out/dist_gpu_test.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash scripts/gpu_dist_rehearsal.sh

# RCCL single-rank collectives + multi-rank gloo DP engine tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/dist_tests.log 2>&1 || { tail -60 gpurun_out/dist_tests.log; exit 1; }
tail -6 gpurun_out/dist_tests.log

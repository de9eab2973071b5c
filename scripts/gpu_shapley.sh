set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_conv_gpu.py -x -q -k shapley -s > gpurun_out/shap_test.log 2>&1 || { grep -E "Error|assert|FAILED|Mismatch" gpurun_out/shap_test.log | tail -20; exit 1; }
grep -E "err=|passed|failed" gpurun_out/shap_test.log
timeout -k 10 400 python -m torchpruner_amd.bench.shapley_vgg --layers 0,3,6,9,12,14 --reference --json gpurun_out/shapley_1gpu.json > gpurun_out/shap_bench.log 2>&1 || { tail -20 gpurun_out/shap_bench.log; exit 1; }
grep "{" gpurun_out/shap_bench.log

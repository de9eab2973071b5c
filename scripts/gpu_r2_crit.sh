set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py -x -q -k "criterion or engine_taylor or engine_shapley" --timeout 200 --timeout-method thread > gpurun_out/crit_tests.log 2>&1 || { tail -60 gpurun_out/crit_tests.log; exit 1; }
tail -1 gpurun_out/crit_tests.log
timeout -k 10 400 python -u -m pytest tests/test_attributions.py tests/test_resnet_bwd_gpu.py tests/test_mlp_engine_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/crit_tests2.log 2>&1 || { tail -60 gpurun_out/crit_tests2.log; exit 1; }
tail -1 gpurun_out/crit_tests2.log

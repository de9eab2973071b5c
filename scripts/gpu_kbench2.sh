set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_conv_gpu.py -x -q -k "not engine" > gpurun_out/conv_gpu4.log 2>&1 || { grep -E "Error|assert|FAILED" gpurun_out/conv_gpu4.log | tail -20; exit 1; }
tail -1 gpurun_out/conv_gpu4.log
timeout -k 10 300 python -m torchpruner_amd.bench.conv_kernels --batch 256 --all-cfg > gpurun_out/kbench2.log 2>&1 || { tail -30 gpurun_out/kbench2.log; exit 1; }
cat gpurun_out/kbench2.log

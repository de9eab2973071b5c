set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_conv_gpu.py -q -x -k "wino" > gpurun_out/wino_tests.log 2>&1 || { tail -40 gpurun_out/wino_tests.log; exit 1; }
tail -2 gpurun_out/wino_tests.log
timeout -k 10 300 python -m torchpruner_amd.bench.conv_kernels --batch 512 --iters 10 --wino > gpurun_out/wino_kbench.log 2>&1 || { tail -30 gpurun_out/wino_kbench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/wino_kbench.log

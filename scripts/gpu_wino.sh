set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_conv_gpu.py -q -x -k "wino or conv_first or nan" > gpurun_out/wino_tests.log 2>&1 || { tail -40 gpurun_out/wino_tests.log; exit 1; }
tail -3 gpurun_out/wino_tests.log
timeout -k 10 300 python -m torchpruner_amd.bench.conv_kernels --batch 512 --iters 10 --wino > gpurun_out/wino_kbench.log 2>&1 || { tail -30 gpurun_out/wino_kbench.log; exit 1; }
cat gpurun_out/wino_kbench.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --train-steps 150 > gpurun_out/wino_bench.log 2>&1 || { tail -30 gpurun_out/wino_bench.log; exit 1; }
tail -5 gpurun_out/wino_bench.log

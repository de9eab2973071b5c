set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_conv_gpu.py tests/test_ops_gpu.py -q -x > gpurun_out/quick_tests.log 2>&1 || { tail -40 gpurun_out/quick_tests.log; exit 1; }
tail -1 gpurun_out/quick_tests.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_quick.log 2>&1 || { tail -30 gpurun_out/bench_quick.log; exit 1; }
grep "\[bench\]" gpurun_out/bench_quick.log

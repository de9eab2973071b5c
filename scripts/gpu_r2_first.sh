# first-layer packed-tap GEMM candidate: test + headline bench + B=100 bench + step trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k "first" > gpurun_out/first_tests.log 2>&1 || { tail -40 gpurun_out/first_tests.log; exit 1; }
tail -2 gpurun_out/first_tests.log
timeout -k 10 300 python -u bench.py --no-prune --no-baseline > gpurun_out/first_bench.log 2>&1 || { tail -30 gpurun_out/first_bench.log; exit 1; }
grep "\[bench\] 1 GPU" gpurun_out/first_bench.log
timeout -k 10 300 python -u bench.py --no-prune --no-baseline --batch 100 --steps 200 --warmup 20 > gpurun_out/first_b100.log 2>&1 || { tail -30 gpurun_out/first_b100.log; exit 1; }
grep "\[bench\] 1 GPU" gpurun_out/first_b100.log
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tr -o run --output-format csv -- python bench.py --steps 8 --warmup 2 --no-prune --no-baseline > gpurun_out/first_tr.log 2>&1 || { tail -30 gpurun_out/first_tr.log; exit 1; }
python scripts/trace_step.py $(find /tmp/tr -name "*kernel_trace.csv" | head -1) nchw_to_nhwc_pad > gpurun_out/first_step_b2048.txt
rm -rf /tmp/tr
head -4 gpurun_out/first_step_b2048.txt
tail -1 gpurun_out/first_step_b2048.txt

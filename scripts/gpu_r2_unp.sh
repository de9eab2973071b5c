# explicit-unpool staged dgrad candidate: tests + headline bench + step trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k "unpool or wino_dgrad" > gpurun_out/unp_tests.log 2>&1 || { tail -40 gpurun_out/unp_tests.log; exit 1; }
tail -2 gpurun_out/unp_tests.log
timeout -k 10 300 python -u bench.py --no-prune --no-baseline > gpurun_out/unp_bench.log 2>&1 || { tail -30 gpurun_out/unp_bench.log; exit 1; }
grep "\[bench\] 1 GPU" gpurun_out/unp_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tr -o run --output-format csv -- python bench.py --steps 8 --warmup 2 --no-prune --no-baseline > gpurun_out/unp_tr.log 2>&1 || { tail -30 gpurun_out/unp_tr.log; exit 1; }
python scripts/trace_step.py $(find /tmp/tr -name "*kernel_trace.csv" | head -1) nchw_to_nhwc_pad > gpurun_out/unp_step_b2048.txt
rm -rf /tmp/tr
tail -1 gpurun_out/unp_step_b2048.txt

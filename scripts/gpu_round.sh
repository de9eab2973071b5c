# Round check: GPU tests, smoke, 1-GPU bench, rocprof kernel stats of the bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 3 --baseline > gpurun_out/bench_full.log 2>&1 || { tail -30 gpurun_out/bench_full.log; exit 1; }
grep "\[bench\]" gpurun_out/bench_full.log; tail -1 gpurun_out/bench_full.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-prune --teacher-steps 0 > $R/gpurun_out/prof_bench.log 2>&1 || { tail -30 $R/gpurun_out/prof_bench.log; exit 1; }
echo done

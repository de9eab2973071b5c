set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --baseline > gpurun_out/bench1.log 2>&1 || { tail -30 gpurun_out/bench1.log; exit 1; }
tail -5 gpurun_out/bench1.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-prune > gpurun_out/prof1.log 2>&1 || { tail -30 gpurun_out/prof1.log; exit 1; }
find gpurun_out/prof1 -name "*stats*" | head

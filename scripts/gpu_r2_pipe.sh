# two-stream small-batch pipeline: bit-identity test + B=100 / B=256 / B=2048 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graphs_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pipe_tests.log 2>&1 || { tail -40 gpurun_out/pipe_tests.log; exit 1; }
tail -6 gpurun_out/pipe_tests.log
for B in 100 256; do
  timeout -k 10 300 python -u bench.py --no-prune --no-baseline --batch $B --steps 200 --warmup 20 > gpurun_out/pipe_b$B.log 2>&1 || { tail -30 gpurun_out/pipe_b$B.log; exit 1; }
  grep "\[bench\] 1 GPU" gpurun_out/pipe_b$B.log
  TORCHPRUNER_STREAMS=0 timeout -k 10 300 python -u bench.py --no-prune --no-baseline --batch $B --steps 200 --warmup 20 > gpurun_out/pipe0_b$B.log 2>&1 || { tail -30 gpurun_out/pipe0_b$B.log; exit 1; }
  grep "\[bench\] 1 GPU" gpurun_out/pipe0_b$B.log
done
timeout -k 10 300 python -u bench.py --no-prune --no-baseline > gpurun_out/pipe_b2048.log 2>&1 || { tail -30 gpurun_out/pipe_b2048.log; exit 1; }
grep "\[bench\] 1 GPU" gpurun_out/pipe_b2048.log

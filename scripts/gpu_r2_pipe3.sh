# two-stream pipeline at large batches (threshold lifted)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for B in 1024 2048; do
  TORCHPRUNER_STREAMS_MAX_PIXELS=1000000000 timeout -k 10 300 python -u bench.py --no-prune --no-baseline --batch $B --steps 40 --warmup 5 > gpurun_out/pipeL_b$B.log 2>&1 || { tail -30 gpurun_out/pipeL_b$B.log; exit 1; }
  echo "streams=1 $(grep '\[bench\] 1 GPU' gpurun_out/pipeL_b$B.log)"
  TORCHPRUNER_STREAMS=0 timeout -k 10 300 python -u bench.py --no-prune --no-baseline --batch $B --steps 40 --warmup 5 > gpurun_out/pipeL0_b$B.log 2>&1 || { tail -30 gpurun_out/pipeL0_b$B.log; exit 1; }
  echo "streams=0 $(grep '\[bench\] 1 GPU' gpurun_out/pipeL0_b$B.log)"
done

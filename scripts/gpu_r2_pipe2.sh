# two-stream pipeline threshold: B=256 / 512 / 1024 with and without
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for B in 256 512 1024; do
  for S in 1 0; do
    TORCHPRUNER_STREAMS=$S timeout -k 10 300 python -u bench.py --no-prune --no-baseline --batch $B --steps 60 --warmup 10 > gpurun_out/pipe${S}_b$B.log 2>&1 || { tail -30 gpurun_out/pipe${S}_b$B.log; exit 1; }
    echo "streams=$S $(grep '\[bench\] 1 GPU' gpurun_out/pipe${S}_b$B.log)"
  done
done

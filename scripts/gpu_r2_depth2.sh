# run-to-run spread of the pipelined B=100 headline: depth 2 / 3 / 4, three runs each
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for D in 2 3 4; do
  for r in 1 2 3; do
    TORCHPRUNER_STREAMS_DEPTH=$D timeout -k 10 200 python -u bench.py --no-prune --no-baseline --batch 100 --steps 200 --warmup 20 --teacher-steps 0 > gpurun_out/dd${D}_$r.log 2>&1 || { tail -30 gpurun_out/dd${D}_$r.log; exit 1; }
    echo "depth=$D run $r $(grep '\[bench\] 1 GPU' gpurun_out/dd${D}_$r.log)"
  done
done

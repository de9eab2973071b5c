# Calibrate the iterative prune protocol (torchpruner_amd/bench/prune_quality.py): Taylor vs
# Random top-1 after really pruning 50% of every VGG16 conv, 3 seeds per config.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
Q="python -u -m torchpruner_amd.bench.prune_quality"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 240 $Q "$@" > gpurun_out/q_$n.jsonl 2> gpurun_out/q_$n.err || { tail -30 gpurun_out/q_$n.err; return 1; }
  python scripts/quality_summary.py < gpurun_out/q_$n.jsonl
}
run H --seeds 0 1 2 --teacher-steps 1000 --recal-batches 0 --ft-steps 10 --final-ft-steps 40 &&
run I --seeds 0 1 2 --teacher-steps 300 --recal-batches 0 --ft-steps 10 --final-ft-steps 40 &&
run J --seeds 0 1 2 --teacher-steps 1000 --recal-batches 0 --increments 4 --ft-steps 5 --final-ft-steps 20 &&
run K --seeds 0 1 2 --teacher-steps 1000 --recal-batches 8 --increments 4 --ft-steps 5 --final-ft-steps 20 &&
run L --seeds 0 1 2 --teacher-steps 1000 --recal-batches 0 --ft-steps 0 --final-ft-steps 0 &&
run M --seeds 0 1 2 --teacher-steps 300 --noise 2.5 --modes 32 --recal-batches 0 --increments 4 --ft-steps 5 --final-ft-steps 20 || exit 1

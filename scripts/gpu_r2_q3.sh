# Prune-quality sweep, 5 seeds: scoring-data size x finetune budget (current training numerics).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
Q="python -u -m torchpruner_amd.bench.prune_quality"
run() {  # name, args...
  local n=$1; shift
  echo "== $n: $*"
  timeout -k 10 300 $Q "$@" > gpurun_out/q_$n.jsonl 2> gpurun_out/q_$n.err || { tail -30 gpurun_out/q_$n.err; return 1; }
  python scripts/quality_summary.py < gpurun_out/q_$n.jsonl
}
run R5 --seeds 0 1 2 3 4 --score-imgs 8000 &&
run R6 --seeds 0 1 2 3 4 --score-imgs 4000 &&
run R7 --seeds 0 1 2 3 4 --score-imgs 4000 --ft-steps 3 --final-ft-steps 10 &&
run R8 --seeds 0 1 2 3 4 --score-imgs 8000 --noise 3.0 || exit 1

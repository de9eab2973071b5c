# Prune-quality sweep, 5 seeds: teacher training length / weight decay (dead-channel structure).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
Q="python -u -m torchpruner_amd.bench.prune_quality"
run() {  # name, args...
  local n=$1; shift
  echo "== $n: $*"
  timeout -k 10 400 $Q "$@" > gpurun_out/q_$n.jsonl 2> gpurun_out/q_$n.err || { tail -30 gpurun_out/q_$n.err; return 1; }
  python scripts/quality_summary.py < gpurun_out/q_$n.jsonl
}
run T2 --seeds 0 1 2 3 4 --score-imgs 4000 --teacher-wd 0.005 &&
run T3 --seeds 0 1 2 3 4 --score-imgs 4000 --teacher-wd 0.002 --teacher-steps 3000 &&
run T1 --seeds 0 1 2 3 4 --score-imgs 4000 --teacher-steps 4000 || exit 1

# GPU suite after the native Linear change + prune-quality sweep under the current training numerics.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
Q="python -u -m torchpruner_amd.bench.prune_quality"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 $Q "$@" > gpurun_out/q_$n.jsonl 2> gpurun_out/q_$n.err || { tail -30 gpurun_out/q_$n.err; return 1; }
  python scripts/quality_summary.py < gpurun_out/q_$n.jsonl
}
run R1 --seeds 0 1 2 &&
run R2 --seeds 0 1 2 --score-imgs 4000 &&
run R3 --seeds 0 1 2 --increments 8 --ft-steps 3 &&
run R4 --seeds 0 1 2 --ft-steps 2 --final-ft-steps 10 || exit 1

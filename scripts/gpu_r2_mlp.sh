# MLP chains on the fused engine (tests, nbUNT timing, kernel trace) + quality sweep round 3.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_mlp_engine_gpu.py tests/test_resnet_engine_gpu.py tests/test_resnet_bwd_gpu.py tests/test_dist_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/mlp_tests.log 2>&1 || { tail -60 gpurun_out/mlp_tests.log; exit 1; }
tail -2 gpurun_out/mlp_tests.log
for d in mnist cifar10; do
  timeout -k 10 200 python experiments/prune_untrained.py --dataset $d > gpurun_out/unt_$d.log 2>&1 || { tail -30 gpurun_out/unt_$d.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/unt_$d.log | tail -1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_unt -o run --output-format csv -- python3 $R/experiments/prune_untrained.py --dataset mnist > $R/gpurun_out/prof_unt.log 2>&1 || { tail -30 $R/gpurun_out/prof_unt.log; exit 1; }
cd $R
python scripts/kernel_stats_summary.py $(find gpurun_out/prof_unt -name "*kernel_stats.csv" | head -1) 20
Q="python -u -m torchpruner_amd.bench.prune_quality"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 240 $Q "$@" > gpurun_out/q_$n.jsonl 2> gpurun_out/q_$n.err || { tail -30 gpurun_out/q_$n.err; return 1; }
  python scripts/quality_summary.py < gpurun_out/q_$n.jsonl
}
run N --seeds 0 1 2 --noise 2.5 --modes 32 --teacher-steps 1500 --recal-batches 0 --increments 4 --ft-steps 5 --final-ft-steps 20 &&
run O --seeds 0 1 2 --noise 3.5 --modes 32 --teacher-steps 2000 --recal-batches 0 --increments 4 --ft-steps 5 --final-ft-steps 20 &&
run P --seeds 0 1 2 --teacher-steps 1000 --recal-batches 0 --increments 4 --ft-steps 2 --final-ft-steps 10 || exit 1

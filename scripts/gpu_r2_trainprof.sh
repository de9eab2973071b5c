# Full GPU suite (generic path now on native convs), native ResNet-50 training step profile
# (kernel stats), roctx marker trace of the headline step.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
cd /tmp && export TMPDIR=/tmp
FMTS=native N=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o run --output-format csv -- python3 $R/scripts/r50_train_probe.py > $R/gpurun_out/prof_train.log 2>&1 || { tail -30 $R/gpurun_out/prof_train.log; exit 1; }
grep "img/s" $R/gpurun_out/prof_train.log
TORCHPRUNER_TRACE=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d $R/gpurun_out/prof_marker -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 2 --no-baseline --no-prune --teacher-steps 0 > $R/gpurun_out/prof_marker.log 2>&1 || { tail -30 $R/gpurun_out/prof_marker.log; exit 1; }
cd $R
python scripts/kernel_stats_summary.py gpurun_out/prof_train/run_kernel_stats.csv 45
ls gpurun_out/prof_marker

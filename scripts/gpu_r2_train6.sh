set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
FMTS=native N=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train6 -o run --output-format csv -- python3 $R/scripts/r50_train_probe.py > $R/gpurun_out/prof_train6.log 2>&1 || { tail -30 $R/gpurun_out/prof_train6.log; exit 1; }
cd $R
python scripts/train_step_breakdown.py gpurun_out/prof_train6/run_kernel_trace.csv > gpurun_out/train6_breakdown.txt
cat gpurun_out/train6_breakdown.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/train_tests.log 2>&1 || { tail -60 gpurun_out/train_tests.log; exit 1; }
tail -1 gpurun_out/train_tests.log
FMTS=native N=10 timeout -k 10 300 python scripts/r50_train_probe.py > gpurun_out/train_probe.log 2>&1 || { tail -30 gpurun_out/train_probe.log; exit 1; }
grep "img/s" gpurun_out/train_probe.log
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
FMTS=native N=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train8 -o run --output-format csv -- python3 $R/scripts/r50_train_probe.py > $R/gpurun_out/prof_train8.log 2>&1 || { tail -30 $R/gpurun_out/prof_train8.log; exit 1; }
cd $R
python scripts/train_step_breakdown.py gpurun_out/prof_train8/run_kernel_trace.csv > gpurun_out/train8_breakdown.txt
head -30 gpurun_out/train8_breakdown.txt

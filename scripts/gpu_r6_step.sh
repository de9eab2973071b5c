# round-6 GPU step: full GPU suite, then a kernel trace of the pruned (round-1) ResNet-50 training step
mkdir -p gpurun_out/prof_pruned
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/gpu_suite.log 2>&1
rc=$?; echo EXIT $rc >> gpurun_out/gpu_suite.log; tail -8 gpurun_out/gpu_suite.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pruned -o r1 -- python scripts/probes/pruned_train_probe.py --rounds 1 --steps 5 > gpurun_out/prof_pruned/probe.log 2>&1
rc=$?; grep pruned_train gpurun_out/prof_pruned/probe.log; exit $rc

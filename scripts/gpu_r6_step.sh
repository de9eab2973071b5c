# round-6 GPU step: pruned-width tests, the pruned training probe, kernel trace of the round-1 step
mkdir -p gpurun_out/prof_pruned2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_pruned_widths_gpu.py tests/test_train_gpu.py > gpurun_out/t4.log 2>&1
rc=$?; tail -3 gpurun_out/t4.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u scripts/probes/pruned_train_probe.py > gpurun_out/probe2.log 2>&1
rc=$?; grep pruned_train gpurun_out/probe2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pruned2 -o r1 -- python scripts/probes/pruned_train_probe.py --rounds 1 --steps 5 > gpurun_out/prof_pruned2/probe.log 2>&1

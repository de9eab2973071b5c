# round-6 GPU step: pruned-width block test, then the teacher-robustness probe (wgrad combine order A/B)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_pruned_widths_gpu.py -k bottlenecks > gpurun_out/t3.log 2>&1
rc=$?; tail -3 gpurun_out/t3.log
[ $rc -le 1 ] || exit $rc
R="lr=0.05 lr=0.02 lr=0.02,noise=3.0,modes=64"
timeout -k 10 400 python -u scripts/probes/teacher_robustness.py --seeds 0 1 2 --recipes $R > gpurun_out/teach_default.log 2>&1
rc=$?; grep recipe gpurun_out/teach_default.log; [ $rc -eq 0 ] || exit $rc
TP_WGRAD_COMBINE_LANES=1 timeout -k 10 400 python -u scripts/probes/teacher_robustness.py --seeds 0 1 2 --recipes $R > gpurun_out/teach_lanes1.log 2>&1
rc=$?; grep recipe gpurun_out/teach_lanes1.log; exit $rc

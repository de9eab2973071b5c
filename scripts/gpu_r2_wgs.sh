# wgrad on a side stream overlapping dgrad: training tests + ResNet-50 B=128 train step (on / off)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wgs_tests.log 2>&1 || { tail -40 gpurun_out/wgs_tests.log; exit 1; }
tail -2 gpurun_out/wgs_tests.log
for S in 1 0; do
  TORCHPRUNER_WGRAD_STREAM=$S FMTS=native timeout -k 10 300 python -u scripts/r50_train_probe.py > gpurun_out/wgs_train_$S.log 2>&1 || { tail -30 gpurun_out/wgs_train_$S.log; exit 1; }
  echo "wgrad_stream=$S $(grep 'ms/step' gpurun_out/wgs_train_$S.log)"
done

# X_SPAN (row-span staged Winograd input): kernel tests, ResNet engine tests, ResNet throughput.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_conv_gpu.py -k wino -x -q --timeout 200 --timeout-method thread > gpurun_out/span_tests.log 2>&1 || { tail -60 gpurun_out/span_tests.log; exit 1; }
tail -1 gpurun_out/span_tests.log
timeout -k 10 500 python -u -m pytest tests/test_resnet_engine_gpu.py tests/test_resnet_bwd_gpu.py tests/test_train_gpu.py tests/test_pruned_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/span_tests2.log 2>&1 || { tail -60 gpurun_out/span_tests2.log; exit 1; }
tail -1 gpurun_out/span_tests2.log
for m in apoz taylor; do
  timeout -k 10 300 python -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 8 --metric $m > gpurun_out/rn_$m.log 2>&1 || { tail -30 gpurun_out/rn_$m.log; exit 1; }
  grep "{" gpurun_out/rn_$m.log
done
FMTS=native N=10 timeout -k 10 300 python scripts/r50_train_probe.py > gpurun_out/train_probe.log 2>&1 || { tail -30 gpurun_out/train_probe.log; exit 1; }
grep "img/s" gpurun_out/train_probe.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-prune --no-baseline --teacher-steps 0 > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { tail -20 gpurun_out/bench_quick.err; exit 1; }
grep "\[bench\]" gpurun_out/bench_quick.err

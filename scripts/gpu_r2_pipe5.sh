# two-stream pipeline on the ResNet engine: bit-identity tests + ResNet-50 APoZ / Taylor throughput
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_resnet_engine_gpu.py tests/test_graphs_gpu.py -x -q --timeout 200 --timeout-method thread -k "pipeline or apoz_matches" > gpurun_out/pipe5_tests.log 2>&1 || { tail -40 gpurun_out/pipe5_tests.log; exit 1; }
tail -2 gpurun_out/pipe5_tests.log
for M in apoz taylor; do
  for S in 1 0; do
    TORCHPRUNER_STREAMS=$S timeout -k 10 300 python -u -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 10 --metric $M > gpurun_out/pipe5_${M}_$S.log 2>&1 || { tail -30 gpurun_out/pipe5_${M}_$S.log; exit 1; }
    echo "streams=$S $(tail -1 gpurun_out/pipe5_${M}_$S.log | cut -c1-130)"
  done
done

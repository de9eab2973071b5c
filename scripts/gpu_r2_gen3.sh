# GEN 3 round-robin dispatch: strided-dgrad tests, ResNet-50 Taylor + training throughput, Taylor step
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_resnet_bwd_gpu.py tests/test_train_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gen3_tests.log 2>&1 || { tail -40 gpurun_out/gen3_tests.log; exit 1; }
tail -2 gpurun_out/gen3_tests.log
timeout -k 10 300 python -u -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 10 --metric taylor > gpurun_out/gen3_tay.log 2>&1 || { tail -30 gpurun_out/gen3_tay.log; exit 1; }
tail -1 gpurun_out/gen3_tay.log | cut -c1-150
FMTS=native timeout -k 10 300 python -u scripts/r50_train_probe.py > gpurun_out/gen3_train.log 2>&1 || { tail -30 gpurun_out/gen3_train.log; exit 1; }
grep -v amdgpu.ids gpurun_out/gen3_train.log | tail -3
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/rt -o run --output-format csv -- python -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 3 --warmup 1 --metric taylor > gpurun_out/gen3_rt.log 2>&1 || { tail -30 gpurun_out/gen3_rt.log; exit 1; }
python scripts/step_breakdown.py $(find /tmp/rt -name "*kernel_trace.csv" | head -1) > gpurun_out/gen3_rn_tay_agg.txt
rm -rf /tmp/rt
head -12 gpurun_out/gen3_rn_tay_agg.txt

# vectorised NHWC channel reduction: op tests + ResNet-50 Taylor / Sensitivity bench + step breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread -k "channel_reduce or first_layer" > gpurun_out/cred_tests.log 2>&1 || { tail -40 gpurun_out/cred_tests.log; exit 1; }
tail -2 gpurun_out/cred_tests.log
timeout -k 10 300 python -u -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 10 --metric taylor > gpurun_out/cred_tay.log 2>&1 || { tail -30 gpurun_out/cred_tay.log; exit 1; }
tail -1 gpurun_out/cred_tay.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/rt -o run --output-format csv -- python -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 3 --warmup 1 --metric taylor > gpurun_out/cred_rt.log 2>&1 || { tail -30 gpurun_out/cred_rt.log; exit 1; }
python scripts/step_breakdown.py $(find /tmp/rt -name "*kernel_trace.csv" | head -1) > gpurun_out/cred_rn_tay_agg.txt
rm -rf /tmp/rt
head -12 gpurun_out/cred_rn_tay_agg.txt

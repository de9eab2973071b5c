# ResNet-50 Taylor step, ordered kernel listing (which config serves each fwd / dgrad GEMM)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/rt -o run --output-format csv -- python -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 3 --warmup 1 --metric taylor > gpurun_out/rt.log 2>&1 || { tail -30 gpurun_out/rt.log; exit 1; }
python scripts/trace_step.py $(find /tmp/rt -name "*kernel_trace.csv" | head -1) nchw_to_nhwc_pad > gpurun_out/rn_tay_step.txt
rm -rf /tmp/rt
tail -2 gpurun_out/rn_tay_step.txt

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn_taylor2 -o run --output-format csv -- python3 -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 3 --warmup 1 --metric taylor > $R/gpurun_out/prof_rn_taylor2.log 2>&1 || { tail -30 $R/gpurun_out/prof_rn_taylor2.log; exit 1; }
cd $R
python scripts/step_breakdown.py gpurun_out/prof_rn_taylor2/run_kernel_trace.csv nchw_to_nhwc_pad 40 > gpurun_out/rn_taylor2_breakdown.txt 2>&1 || true
cat gpurun_out/rn_taylor2_breakdown.txt

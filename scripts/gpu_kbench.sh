set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m torchpruner_amd.bench.conv_kernels --batch 256 --all-cfg > gpurun_out/kbench.log 2>&1 || { tail -30 gpurun_out/kbench.log; exit 1; }
cat gpurun_out/kbench.log
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $GRAFT_REPO_ROOT/gpurun_out/pmc1 -o run --output-format csv -- python -m torchpruner_amd.bench.conv_kernels --batch 256 --iters 3 > gpurun_out/pmc1.log 2>&1 || { tail -20 gpurun_out/pmc1.log; exit 0; }

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof4 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-prune --teacher-steps 0 > gpurun_out/prof4.log 2>&1 || { tail -30 gpurun_out/prof4.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $GRAFT_REPO_ROOT/gpurun_out/pmc4 -o run --output-format csv -- python -m torchpruner_amd.bench.conv_kernels --batch 512 --iters 2 > gpurun_out/pmc4.log 2>&1 || { tail -20 gpurun_out/pmc4.log; exit 1; }
grep -E "TOTAL|L " gpurun_out/pmc4.log | tail -14

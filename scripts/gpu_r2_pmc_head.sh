# headline step PMC (B=2048, random-init weights: no teacher training under the profiler):
# MFMA utilisation and LDS instructions per kernel of the last step
set -o pipefail
cd /tmp && export TMPDIR=/tmp
export TORCHPRUNER_AUTOTUNE=0  # same kernel choices in every pass (heuristic picks)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmch
mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d $O/p1 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-prune --no-baseline --teacher-steps 0 > $R/gpurun_out/pmch_p1.log 2>&1 || { echo "pass 1 failed"; tail -5 $R/gpurun_out/pmch_p1.log; exit 1; }
python3 $R/scripts/pmc_last_step.py nchw_to_nhwc_pad $O/p1 > $R/gpurun_out/headline_pmc_b2048.txt
rm -rf $O
cat $R/gpurun_out/headline_pmc_b2048.txt

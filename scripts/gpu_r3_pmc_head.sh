# Headline step PMC (B=2048) WITH native-kernel teacher training under the profiler (round-2 runs
# aborted there with HSA_STATUS_ERROR_INVALID_PACKET_FORMAT), two counter passes, then B=100 bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
export TORCHPRUNER_AUTOTUNE=0  # same kernel choices in every pass (heuristic picks)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmch3
mkdir -p $O
TS=${PMC_TEACHER_STEPS:-300}
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d $O/p1 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-prune --no-baseline --no-extras --teacher-steps $TS > $R/gpurun_out/pmch3_p1.log 2>&1 || { echo "pass 1 failed"; tail -15 $R/gpurun_out/pmch3_p1.log; exit 1; }
python3 $R/scripts/pmc_last_step.py nchw_to_nhwc_pad $O/p1 > $R/gpurun_out/headline_pmc_r3_p1.txt
timeout -s KILL 240 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d $O/p2 -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-prune --no-baseline --no-extras --teacher-steps $TS > $R/gpurun_out/pmch3_p2.log 2>&1 || { echo "pass 2 failed"; tail -15 $R/gpurun_out/pmch3_p2.log; exit 2; }
python3 $R/scripts/pmc_last_step.py nchw_to_nhwc_pad $O/p2 > $R/gpurun_out/headline_pmc_r3_p2.txt
rm -rf $O
cat $R/gpurun_out/headline_pmc_r3_p1.txt
cd $R && mkdir -p gpurun_out/r3 && unset TORCHPRUNER_AUTOTUNE && timeout -k 10 300 python bench.py --batch 100 --steps 200 --warmup 10 --no-baseline --no-prune --no-extras --teacher-steps 0 > gpurun_out/r3/b100.json 2> gpurun_out/r3/b100.err || { tail -30 gpurun_out/r3/b100.err; exit 3; }
cat gpurun_out/r3/b100.json

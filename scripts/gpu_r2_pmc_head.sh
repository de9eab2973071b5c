# headline step PMC (B=2048): MFMA utilisation, LDS, HBM bytes per kernel of the last step
set -o pipefail
cd /tmp && export TMPDIR=/tmp
export TORCHPRUNER_AUTOTUNE=0  # same kernel choices in every pass (heuristic picks)
R=$GRAFT_REPO_ROOT
O=/tmp/pmch
mkdir -p $O $R/gpurun_out
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace -d $O/p$i -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-prune --no-baseline > $R/gpurun_out/pmch_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmch_p$i.log; exit 1; }
done
python3 $R/scripts/pmc_last_step.py nchw_to_nhwc_pad $O/p1 $O/p2 $O/p3 > $R/gpurun_out/headline_pmc_b2048.txt
rm -rf $O
cat $R/gpurun_out/headline_pmc_b2048.txt

# PMC counters of the ResNet-50 APoZ engine step (B=256): MFMA busy, HBM bytes, LDS conflicts,
# one counter group per rocprofv3 run (+ kernel trace for durations).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export PYTHONPATH=$R
O=$R/gpurun_out/pmc_rn
mkdir -p $O
CMD="python3 -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 2 --warmup 1"
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-trace -d $O/p$i -o run --output-format csv -- $CMD > $O/p$i.log 2>&1 || { echo "group $i ($grp) failed"; tail -5 $O/p$i.log; exit 1; }
done
cd $R
python scripts/pmc_last_step.py nchw_to_nhwc_pad gpurun_out/pmc_rn/p1 gpurun_out/pmc_rn/p2 gpurun_out/pmc_rn/p3 gpurun_out/pmc_rn/p4

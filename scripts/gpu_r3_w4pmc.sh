#!/bin/bash
# PMC passes over the F(4x4) vs F(2x2) forward kernels on one layer shape (one rocprofv3 run per group)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/w4pmc
mkdir -p $O
SHAPE=${W4_SHAPE:-8 256 256}
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM TA_BUSY_avr TA_BUSY_max"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d $O/p$i -o run --output-format csv -- python3 $R/scripts/wino4_probe.py $SHAPE > $O/p$i.log 2>&1 || { echo "group $i failed"; tail -5 $O/p$i.log; exit 1; }
  for f in $(find $O/p$i -name "*counter_collection.csv"); do
    python3 $R/scripts/pmc_summary.py $f wino > $R/gpurun_out/w4pmc_g$i.txt
  done
done
rm -rf $O

#!/bin/bash
# PMC passes (3 groups) over the F(4x4) vs F(2x2) forward kernels on one layer shape
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/w4pmc2
mkdir -p $O
SHAPE=${W4_SHAPE:-8 256 256}
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES" \
           "SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_INSTS_VALU" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d $O/p$i -o run --output-format csv -- python3 $R/scripts/wino4_probe.py $SHAPE > $O/p$i.log 2>&1 || { echo "group $i failed"; tail -5 $O/p$i.log; exit 1; }
  for f in $(find $O/p$i -name "*counter_collection.csv"); do
    python3 $R/scripts/pmc_summary.py $f wino > $R/gpurun_out/w4pmc2_g$i.txt
  done
done
rm -rf $O

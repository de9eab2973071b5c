set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gemm_pmc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" \
           "SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INST_CYCLES_VMEM_RD SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc -d $R/gpurun_out/gemm_pmc/p$i -o run --output-format csv -- python3 $R/scripts/gemm_pmc_probe.py > $R/gpurun_out/gemm_pmc/p$i.log 2>&1 || { tail -20 $R/gpurun_out/gemm_pmc/p$i.log; exit 1; }
done
echo ok

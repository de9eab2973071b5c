set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcw3
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- python3 $R/scripts/probes/wino_probe.py > $O/kt.log 2>&1 || { echo "kt failed"; tail -3 $O/kt.log; }
i=0
for grp in "SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" "TA_TA_BUSY_sum TA_BUSY_avr" "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY" "SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp -d $O/p$i -o run --output-format csv -- python3 $R/scripts/probes/wino_probe.py > $O/p$i.log 2>&1 || { echo "group $i ($grp) failed"; tail -3 $O/p$i.log; }
done
exit 0

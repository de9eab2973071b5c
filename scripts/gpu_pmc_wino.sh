set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcw2
mkdir -p $O
i=0
for grp in "TA_TA_BUSY_sum TA_BUSY_avr" "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC" "SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_WAVES SQ_ACTIVE_INST_LDS" "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp -d $O/p$i -o run --output-format csv -- python3 $R/scripts/wino_probe.py > $O/p$i.log 2>&1 || { echo "group $i ($grp) failed"; tail -3 $O/p$i.log; }
done
exit 0

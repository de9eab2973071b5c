set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcl2
mkdir -p $O
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES" "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TA_DATA_STALLED_BY_TC_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $grp -d $O/p$i -o run --output-format csv -- python3 $R/scripts/probes/wino4_layer_probe.py > $O/p$i.log 2>&1 || { echo "group $i ($grp) failed"; tail -3 $O/p$i.log; exit 1; }
done
echo ok

# PMC of one VGG layer (S=8, C=K=256, B=2048, forward) on the fp32 F(2x2), bf16 F(2x2) and fp32
# F(4x4) kernels: instruction mix, MFMA busy, LDS waits / bank conflicts (one pass per group).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcbf
mkdir -p $O
for kind in wino2bf wino2 wino4; do
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $grp -d $O/$kind$i -o run --output-format csv -- python3 $R/scripts/probes/wino4_layer_probe.py --kind $kind > $O/$kind$i.log 2>&1 || { echo "$kind group $i failed"; tail -3 $O/$kind$i.log; exit 1; }
  done
  echo "== $kind"; python3 $R/scripts/pmc_table.py "$O/$kind[12]/**/*counter_collection.csv"
done

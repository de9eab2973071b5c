# MFMA utilisation and instruction mix of the 32-pixel F(4x4) kernels (VGG16 layer 1: C=K=64,
# B=2048, forward with pooling and data gradient), one PMC pass per counter group.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc32
mkdir -p $O
for mode in "--pool" "--dgrad"; do
  tag=$(echo $mode | tr -d '-')
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES" "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $grp -d $O/$tag$i -o run --output-format csv -- python3 $R/scripts/probes/wino4_layer_probe.py --S 32 --C 64 --K 64 $mode > $O/$tag$i.log 2>&1 || { echo "$tag group $i failed"; tail -3 $O/$tag$i.log; exit 1; }
  done
  echo "== S=32 C=K=64 B=2048 $tag"; python3 $R/scripts/pmc_table.py "$O/$tag[12]/**/*counter_collection.csv"
done

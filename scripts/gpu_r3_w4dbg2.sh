#!/bin/bash
# MODE 2 phase costs on one layer: time + LDS bank-conflict / wait counters per TP_W4_DBG setting
# (1 no U DMA, 2 no X DMA, 4 no patch reads, 8 no U reads, 16 no epilogue; results are wrong when set)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/w4dbg2
mkdir -p $O
SHAPE=${W4_SHAPE:-8 256 256}
for d in ${W4_DBG_LIST:-0 3 4 8 12 15 16 31}; do
  TP_W4_DBG=$d timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS --kernel-trace -d $O/d$d -o run --output-format csv -- python3 $R/scripts/wino4_probe.py $SHAPE > $O/d$d.log 2>&1 || { echo "dbg $d failed"; tail -5 $O/d$d.log; exit 1; }
  echo "== TP_W4_DBG=$d" >> $R/gpurun_out/w4dbg2.txt
  for f in $(find $O/d$d -name "*counter_collection.csv"); do
    python3 $R/scripts/pmc_summary.py $f wino >> $R/gpurun_out/w4dbg2.txt
  done
done
rm -rf $O

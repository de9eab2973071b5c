# VALU per wave of the F(4x4) split-points forward under the TP_W4_DBG phase switches
# (1 no U DMA, 2 no X DMA, 16 no epilogue; results wrong, counts only): where the non-transform
# VALU of the chunk loop comes from.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/w4dbg
mkdir -p $O
i=0
for cfg in "8 256" "32 64"; do
  set -- $cfg
  for dbg in 0 1 2 3 19; do
    i=$((i+1))
    TP_W4_DBG=$dbg timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d $O/p$i -o run --output-format csv -- python3 $R/scripts/probes/wino4_layer_probe.py --S $1 --C $2 --K $2 --variant 3 --iters 2 > $O/p$i.log 2>&1 || { echo "pmc $i failed"; tail -3 $O/p$i.log; exit 1; }
    python3 - "$O/p$i" "S=$1 C=$2 fwd dbg=$dbg" <<'PY'
import csv, glob, sys, collections, statistics
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "wino4" in r["Kernel_Name"]: agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: statistics.mean(v) for k, v in agg.items()}
w = m.pop("SQ_WAVES")
print(f"{sys.argv[2]:24s} " + "  ".join(f"{k[8:]} {v / w:7.0f}" for k, v in sorted(m.items())))
PY
  done
done

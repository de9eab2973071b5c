# Cost of the F(4x4) split-points epilogue: per (S, C, direction) the kernel time and VALU count
# with the full kernel and with TP_W4_DBG=16 (epilogue skipped; results wrong — timing only).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/w4epi
mkdir -p $O
i=0
for cfg in "8 256" "4 512" "16 128" "32 64"; do
  set -- $cfg
  for dir in fwd dgrad; do
    extra=""; [ $dir = dgrad ] && extra="--dgrad"
    for dbg in 0 16; do
      i=$((i+1))
      TP_W4_DBG=$dbg timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/t$i -o run --output-format csv -- python3 $R/scripts/probes/wino4_layer_probe.py --S $1 --C $2 --K $2 --variant 3 --iters 6 $extra > $O/t$i.log 2>&1 || { echo "trace $i failed"; tail -3 $O/t$i.log; exit 1; }
      TP_W4_DBG=$dbg timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS -d $O/p$i -o run --output-format csv -- python3 $R/scripts/probes/wino4_layer_probe.py --S $1 --C $2 --K $2 --variant 3 --iters 2 $extra > $O/p$i.log 2>&1 || { echo "pmc $i failed"; tail -3 $O/p$i.log; exit 1; }
      python3 - "$O/t$i" "$O/p$i" "S=$1 C=$2 $dir dbg=$dbg" <<'PY'
import csv, glob, sys, collections, statistics
t = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(t)) if "wino4" in r["Kernel_Name"]]
f = glob.glob(sys.argv[2] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "wino4" in r["Kernel_Name"]: agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: statistics.mean(v) for k, v in agg.items()}
w = m.get("SQ_WAVES", 1)
print(f"{sys.argv[3]:28s} {statistics.median(d[1:]) / 1e3:8.1f} us  VALU/wave {m['SQ_INSTS_VALU'] / w:7.0f}  MFMA/wave {m['SQ_INSTS_MFMA'] / w:6.0f}  LDS/wave {m['SQ_INSTS_LDS'] / w:6.0f}")
PY
    done
  done
done

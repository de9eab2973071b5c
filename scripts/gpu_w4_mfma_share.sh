# MFMA share of the F(4x4) split-points kernel: kernel time with every other MFMA pair of the
# main loop skipped (TP_W4_DBG=32, timing only; results wrong) vs the full kernel, per layer.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/w4share
mkdir -p $O
i=0
for cfg in "8 256" "4 512" "16 128" "32 64"; do
  set -- $cfg
  for dir in fwd dgrad; do
    extra=""; [ $dir = dgrad ] && extra="--dgrad"
    for dbg in 0 32; do
      i=$((i+1))
      TP_W4_DBG=$dbg timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/t$i -o run --output-format csv -- python3 $R/scripts/probes/wino4_layer_probe.py --S $1 --C $2 --K $2 --variant 3 --iters 40 $extra > $O/t$i.log 2>&1 || { echo "trace $i failed"; tail -3 $O/t$i.log; exit 1; }
      python3 - "$O/t$i" "S=$1 C=$2 $dir dbg=$dbg" <<'PY'
import csv, glob, sys, statistics
t = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(t)) if "wino4" in r["Kernel_Name"]]
print(f"{sys.argv[2]:26s} median of last 20: {statistics.median(d[-20:]) / 1e3:8.1f} us  (first {d[0] / 1e3:.1f})")
PY
    done
  done
done

# PMC of the memory-bound short-K 1x1 implicit GEMM (ResNet-50 training, 64 -> 256 at 56 px,
# B=128): instruction mix, busy / wait cycles for two tile configs (scripts/probes/lowk_gemm_probe.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmclowk
mkdir -p $O
i=0
for cfg in 4 2; do
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_INSTS_SMEM"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp -d $O/p$i -o run --output-format csv -- python3 $R/scripts/probes/lowk_gemm_probe.py --one 128 56 64 256 $cfg 1 > $O/p$i.log 2>&1 || { echo "pass $i (cfg $cfg: $grp) failed"; tail -3 $O/p$i.log; exit 1; }
    echo "== cfg $cfg pass $i"
    python3 - "$O/p$i" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "conv_igemm" not in k: continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    print(k[:70], {c: round(v / n[(k, c)]) for c, v in sorted(d.items())})
PY
  done
done

# PMC of one F(4x4) layer, forward vs data gradient (split-points kernel, variant 3), at the
# given S / C=K (default 8 px, 256 channels): instruction mix and busy cycles per direction.
set -o pipefail
S=${1:-8}; C=${2:-256}
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcpair_s${S}
mkdir -p $O
i=0
for dir in fwd dgrad; do
  extra=""; [ $dir = dgrad ] && extra="--dgrad"
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_INSTS_SMEM"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $grp -d $O/p$i -o run --output-format csv -- python3 $R/scripts/probes/wino4_layer_probe.py --S $S --C $C --K $C --variant 3 $extra > $O/p$i.log 2>&1 || { echo "pass $i ($dir: $grp) failed"; tail -3 $O/p$i.log; exit 1; }
    echo "== $dir pass $i"
    python3 - "$O/p$i" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "wino4" not in k: continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    print(k[:60], {c: round(v / n[(k, c)]) for c, v in sorted(d.items())})
PY
  done
done

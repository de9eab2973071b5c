# Training-step autotuner decisions with every candidate's time (ResNet-50, B=128), plus the
# kernel list of the last step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/traintune
mkdir -p $O
TORCHPRUNER_TUNER_LOG=2 FMTS=native N=3 timeout -k 10 400 rocprofv3 --kernel-trace -d $O/t -o run --output-format csv -- python3 $R/scripts/r50_train_probe.py > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
f=$(find $O/t -name '*kernel_trace.csv' | head -1)
python3 $R/scripts/train_step_breakdown.py $f > $O/breakdown.txt
python3 $R/scripts/train_kernel_list.py $f "." > $O/list.txt
head -3 $O/breakdown.txt; tail -1 $O/list.txt

# wgrad FastDiv check + training step, ResNet-50 attribution throughput (APoZ / Taylor) and a
# kernel trace of the Taylor step.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/train_tests.log 2>&1 || { tail -60 gpurun_out/train_tests.log; exit 1; }
tail -1 gpurun_out/train_tests.log
FMTS=native N=10 timeout -k 10 300 python scripts/r50_train_probe.py > gpurun_out/train_probe.log 2>&1 || { tail -30 gpurun_out/train_probe.log; exit 1; }
grep "img/s" gpurun_out/train_probe.log
for m in apoz taylor; do
  timeout -k 10 300 python -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 8 --metric $m > gpurun_out/rn_$m.log 2>&1 || { tail -30 gpurun_out/rn_$m.log; exit 1; }
  grep "{" gpurun_out/rn_$m.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn_taylor -o run --output-format csv -- python3 -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 3 --warmup 1 --metric taylor > $R/gpurun_out/prof_rn_taylor.log 2>&1 || { tail -30 $R/gpurun_out/prof_rn_taylor.log; exit 1; }
cd $R
python scripts/kernel_stats_summary.py gpurun_out/prof_rn_taylor/run_kernel_stats.csv 30

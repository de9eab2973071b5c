# Current-state profiles: ResNet-50 APoZ / Taylor engine steps (B=256), headline step at B=100,
# training probe, and the full GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
FMTS=native N=10 timeout -k 10 300 python scripts/r50_train_probe.py > gpurun_out/train_probe.log 2>&1 || { tail -30 gpurun_out/train_probe.log; exit 1; }
grep "img/s" gpurun_out/train_probe.log
export PYTHONPATH=$R
timeout -k 10 300 python -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 8 --warmup 2 --metric apoz > gpurun_out/rn_apoz.log 2>&1 || { tail -30 gpurun_out/rn_apoz.log; exit 1; }
timeout -k 10 300 python -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 8 --warmup 2 --metric taylor > gpurun_out/rn_taylor.log 2>&1 || { tail -30 gpurun_out/rn_taylor.log; exit 1; }
tail -1 gpurun_out/rn_apoz.log; tail -1 gpurun_out/rn_taylor.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn_apoz2 -o run --output-format csv -- python3 -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 3 --warmup 1 --metric apoz > $R/gpurun_out/prof_rn_apoz2.log 2>&1 || { tail -30 $R/gpurun_out/prof_rn_apoz2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_b100 -o run --output-format csv -- python3 $R/bench.py --batch 100 --steps 50 --warmup 5 --no-baseline --no-prune --teacher-steps 0 > $R/gpurun_out/prof_b100.log 2>&1 || { tail -30 $R/gpurun_out/prof_b100.log; exit 1; }
cd $R
python scripts/step_breakdown.py gpurun_out/prof_rn_apoz2/run_kernel_trace.csv > gpurun_out/rn_apoz2_breakdown.txt 2>&1 || true
head -25 gpurun_out/rn_apoz2_breakdown.txt
timeout -k 10 300 python bench.py --batch 100 --steps 200 --warmup 10 --no-baseline --no-prune --teacher-steps 0 > gpurun_out/b100.json 2> gpurun_out/b100.err || { tail -30 gpurun_out/b100.err; exit 1; }
cat gpurun_out/b100.json | cut -c1-200
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
python scripts/step_breakdown.py gpurun_out/prof_b100/run_kernel_trace.csv nchw_to_nhwc_pad 70 > gpurun_out/b100_breakdown.txt 2>&1 || true
head -3 gpurun_out/b100_breakdown.txt

# Full state check: GPU suite, smoke, headline bench twice (reproducibility), B=100, ResNet benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_f.json 2> gpurun_out/bench_f.err || { tail -30 gpurun_out/bench_f.err; exit 1; }
cat gpurun_out/bench_f.json; grep "\[bench\]" gpurun_out/bench_f.err
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-baseline > gpurun_out/bench_g.json 2> gpurun_out/bench_g.err || { tail -30 gpurun_out/bench_g.err; exit 1; }
grep "\[bench\]" gpurun_out/bench_g.err
timeout -k 10 300 python bench.py --batch 100 --steps 200 --warmup 10 --no-baseline --no-prune --teacher-steps 0 > gpurun_out/b100.json 2> gpurun_out/b100.err || { tail -30 gpurun_out/b100.err; exit 1; }
grep "\[bench\] 1 GPU" gpurun_out/b100.err
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 8 --warmup 2 --metric apoz > gpurun_out/rn_apoz.log 2>&1 || { tail -30 gpurun_out/rn_apoz.log; exit 1; }
timeout -k 10 300 python -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 8 --warmup 2 --metric taylor > gpurun_out/rn_taylor.log 2>&1 || { tail -30 gpurun_out/rn_taylor.log; exit 1; }
tail -1 gpurun_out/rn_apoz.log | cut -c1-140; tail -1 gpurun_out/rn_taylor.log | cut -c1-140

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/train_tests.log 2>&1 || { tail -60 gpurun_out/train_tests.log; exit 1; }
tail -2 gpurun_out/train_tests.log
FMTS=native N=10 timeout -k 10 300 python scripts/r50_train_probe.py > gpurun_out/train_probe.log 2>&1 || { tail -30 gpurun_out/train_probe.log; exit 1; }
grep "img/s" gpurun_out/train_probe.log
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-baseline > gpurun_out/bench_d.json 2> gpurun_out/bench_d.err || { tail -30 gpurun_out/bench_d.err; exit 1; }
cat gpurun_out/bench_d.json; grep "\[bench\]" gpurun_out/bench_d.err

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py -x -q -k "wino" --timeout 200 --timeout-method thread > gpurun_out/odd_tests.log 2>&1 || { tail -60 gpurun_out/odd_tests.log; exit 1; }
tail -1 gpurun_out/odd_tests.log
timeout -k 10 300 python bench.py --batch 100 --steps 200 --warmup 10 --no-baseline --no-prune --teacher-steps 0 > gpurun_out/b100.json 2> gpurun_out/b100.err || { tail -30 gpurun_out/b100.err; exit 1; }
grep "\[bench\] 1 GPU" gpurun_out/b100.err
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-baseline --no-prune --teacher-steps 0 > gpurun_out/b2048.json 2> gpurun_out/b2048.err || { tail -30 gpurun_out/b2048.err; exit 1; }
grep "\[bench\] 1 GPU" gpurun_out/b2048.err
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 8 --warmup 2 --metric apoz > gpurun_out/rn_apoz.log 2>&1 || { tail -30 gpurun_out/rn_apoz.log; exit 1; }
timeout -k 10 300 python -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 8 --warmup 2 --metric taylor > gpurun_out/rn_taylor.log 2>&1 || { tail -30 gpurun_out/rn_taylor.log; exit 1; }
tail -1 gpurun_out/rn_apoz.log | cut -c1-140; tail -1 gpurun_out/rn_taylor.log | cut -c1-140
FMTS=native N=10 timeout -k 10 300 python scripts/r50_train_probe.py > gpurun_out/train_probe.log 2>&1 || { tail -30 gpurun_out/train_probe.log; exit 1; }
grep "img/s" gpurun_out/train_probe.log

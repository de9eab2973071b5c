# B=100 figures of the bench (coalesced / one launch per batch / host loaders) with the tuner log,
# plus the graph / pipeline GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_graphs_gpu.py tests/test_coalesce_gpu.py > gpurun_out/tg.log 2>&1 || { tail -30 gpurun_out/tg.log; exit 1; }
tail -1 gpurun_out/tg.log
TORCHPRUNER_TUNER_LOG=1 timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --teacher-steps 0 --no-prune --no-baseline --extras b100 > gpurun_out/b100.json 2> gpurun_out/b100.log || { tail -30 gpurun_out/b100.log; exit 1; }
grep "\[bench\]" gpurun_out/b100.log; grep "in flight" gpurun_out/b100.log | head -40

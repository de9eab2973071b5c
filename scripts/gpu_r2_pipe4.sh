# two-stream pipeline for all batch sizes: tests (graphs/pipeline, engine, dist) + headline + B=100 + APoZ
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_graphs_gpu.py tests/test_dist_gpu.py tests/test_pruned_engine_gpu.py tests/test_mlp_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pipe4_tests.log 2>&1 || { tail -40 gpurun_out/pipe4_tests.log; exit 1; }
tail -2 gpurun_out/pipe4_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/pipe4_bench.log 2>&1 || { tail -30 gpurun_out/pipe4_bench.log; exit 1; }
grep "\[bench\]" gpurun_out/pipe4_bench.log
tail -1 gpurun_out/pipe4_bench.log | cut -c1-400
timeout -k 10 300 python -u bench.py --no-prune --no-baseline --batch 100 --steps 200 --warmup 20 > gpurun_out/pipe4_b100.log 2>&1 || { tail -30 gpurun_out/pipe4_b100.log; exit 1; }
grep "\[bench\] 1 GPU" gpurun_out/pipe4_b100.log

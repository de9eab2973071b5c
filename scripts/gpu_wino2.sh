set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 10 300 python scripts/wino_engine_check.py > gpurun_out/wino_check.log 2>&1 || { tail -30 gpurun_out/wino_check.log; exit 1; }
cat gpurun_out/wino_check.log
timeout -k 10 600 python -m pytest tests/test_conv_gpu.py -q -x -k "engine" > gpurun_out/wino_eng_tests.log 2>&1 || { tail -40 gpurun_out/wino_eng_tests.log; exit 1; }
tail -3 gpurun_out/wino_eng_tests.log
TORCHPRUNER_WINOGRAD=0 timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/nowino_bench.log 2>&1 || { tail -30 gpurun_out/nowino_bench.log; exit 1; }
grep bench gpurun_out/nowino_bench.log

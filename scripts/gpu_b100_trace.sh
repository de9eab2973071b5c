# B=100 (the reference's attribution batch, nbVGG:193-196) step trace + default bench at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/b100t -o run --output-format csv -- python bench.py --batch 100 --steps 10 --warmup 3 --no-prune --teacher-steps 0 > gpurun_out/b100t.log 2>&1 || { tail -30 gpurun_out/b100t.log; exit 1; }
python scripts/trace_step.py $(find gpurun_out/b100t -name "*kernel_trace.csv" | head -1) > gpurun_out/b100t_step.txt
tail -3 gpurun_out/b100t_step.txt
timeout -k 10 400 python bench.py --batch 100 --steps 200 --warmup 20 --no-prune --teacher-steps 0 > gpurun_out/b100_bench.log 2>&1 || { tail -30 gpurun_out/b100_bench.log; exit 1; }
grep "\[bench\] 1 GPU" gpurun_out/b100_bench.log
timeout -k 10 600 python bench.py > gpurun_out/bench_head.log 2>&1 || { tail -30 gpurun_out/bench_head.log; exit 1; }
tail -1 gpurun_out/bench_head.log | cut -c1-300

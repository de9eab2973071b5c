# bench.py twice with the same seed (reproducibility of the accuracy half), the full GPU suite +
# smoke, and a roctx marker trace of the headline step (TORCHPRUNER_TRACE=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err || { tail -30 gpurun_out/bench_a.err; exit 1; }
cat gpurun_out/bench_a.json; grep "\[bench\]" gpurun_out/bench_a.err
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-baseline > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || { tail -30 gpurun_out/bench_b.err; exit 1; }
grep "\[bench\]" gpurun_out/bench_b.err
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
cd /tmp && export TMPDIR=/tmp
TORCHPRUNER_TRACE=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d $R/gpurun_out/prof_marker -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 2 --no-baseline --no-prune --teacher-steps 0 > $R/gpurun_out/prof_marker.log 2>&1 || { tail -30 $R/gpurun_out/prof_marker.log; exit 1; }
ls $R/gpurun_out/prof_marker/*/ 2>/dev/null | head; ls $R/gpurun_out/prof_marker | head

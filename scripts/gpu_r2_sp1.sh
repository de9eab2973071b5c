# split-K = 1 candidates (no partial-slab combine launch) at small batch
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-prune --no-baseline --batch 100 --steps 200 --warmup 20 > gpurun_out/sp1_b100.log 2>&1 || { tail -30 gpurun_out/sp1_b100.log; exit 1; }
grep "\[bench\] 1 GPU" gpurun_out/sp1_b100.log
timeout -k 10 300 python -u bench.py --no-prune --no-baseline > gpurun_out/sp1_bench.log 2>&1 || { tail -30 gpurun_out/sp1_bench.log; exit 1; }
grep "\[bench\] 1 GPU" gpurun_out/sp1_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tr -o run --output-format csv -- python bench.py --batch 100 --steps 8 --warmup 2 --no-prune --no-baseline > gpurun_out/sp1_tr.log 2>&1 || { tail -30 gpurun_out/sp1_tr.log; exit 1; }
python scripts/trace_step.py $(find /tmp/tr -name "*kernel_trace.csv" | head -1) nchw_to_nhwc_pad > gpurun_out/sp1_step_b100.txt
rm -rf /tmp/tr
tail -1 gpurun_out/sp1_step_b100.txt
timeout -k 10 300 python -u scripts/run_overhead.py > gpurun_out/run_overhead.log 2>&1 || { tail -30 gpurun_out/run_overhead.log; exit 1; }
head -40 gpurun_out/run_overhead.log | grep -v amdgpu.ids

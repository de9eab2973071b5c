# B=100 one-launch-per-batch diagnosis: kernel trace of the bench's B=100 path without coalescing
# (kernel busy vs wall per batch, per-kernel table of the last batches), plus the F(4x4) variants on
# engine-like operands.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/wino4_variant_bench.py --variants 3 0 --batch 2048 --real > gpurun_out/w4real.log 2>&1 || { tail -20 gpurun_out/w4real.log; exit 1; }
grep -v amdgpu.ids gpurun_out/w4real.log
cd /tmp && export TMPDIR=/tmp
TORCHPRUNER_COALESCE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/b100prof -o run --output-format csv -- python3 $R/bench.py --batch 100 --steps 200 --warmup 20 --no-extras --no-prune --no-baseline --teacher-steps 0 > $R/gpurun_out/b100prof.log 2>&1 || { tail -30 $R/gpurun_out/b100prof.log; exit 1; }
grep "\[bench\]" $R/gpurun_out/b100prof.log
f=$(find $R/gpurun_out/b100prof -name '*kernel_trace.csv' | head -1)
python3 $R/scripts/probes/trace_overlap.py $f 0.15 20 2>&1 | tail -25
python3 $R/scripts/kernel_stats_summary.py $(find $R/gpurun_out/b100prof -name '*kernel_stats.csv' | head -1) 30

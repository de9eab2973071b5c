set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests/test_conv_gpu.py -x -q -k engine -s > gpurun_out/conv_gpu3.log 2>&1 || { grep -E "err|Error|assert" gpurun_out/conv_gpu3.log | tail -30; exit 1; }
tail -2 gpurun_out/conv_gpu3.log
for B in 128 256 512; do
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --batch $B > gpurun_out/bench2_$B.log 2>&1 || { tail -30 gpurun_out/bench2_$B.log; exit 1; }
grep "\[bench\]" gpurun_out/bench2_$B.log
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-prune > gpurun_out/prof2.log 2>&1 || { tail -30 gpurun_out/prof2.log; exit 1; }

set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m torchpruner_amd.bench.conv_kernels --batch 256 --all-cfg > gpurun_out/kbench3.log 2>&1 || { tail -30 gpurun_out/kbench3.log; exit 1; }
grep -E "f[456]/" gpurun_out/kbench3.log
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu5.log 2>&1 || { grep -E "Error|assert|FAILED" gpurun_out/pytest_gpu5.log | tail -30; exit 1; }
tail -1 gpurun_out/pytest_gpu5.log
for B in 256 512; do
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --batch $B > gpurun_out/bench5_$B.log 2>&1 || { tail -30 gpurun_out/bench5_$B.log; exit 1; }
grep "\[bench\]" gpurun_out/bench5_$B.log
done

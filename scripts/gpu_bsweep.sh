set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for B in 256 1024 2048; do
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --batch $B --no-prune --teacher-steps 0 > gpurun_out/bsweep_$B.log 2>&1 || { tail -30 gpurun_out/bsweep_$B.log; exit 1; }
grep "\[bench\] 1 GPU" gpurun_out/bsweep_$B.log
done

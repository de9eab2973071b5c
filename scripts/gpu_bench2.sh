set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_rep$i.log 2>&1 || { tail -30 gpurun_out/bench_rep$i.log; exit 1; }
grep "\[bench\]" gpurun_out/bench_rep$i.log
done

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for f in 0 1 0 1; do
TP_WINO_FOLD=$f timeout -k 10 300 python bench.py --batch 100 --steps 200 --warmup 10 --no-baseline --no-prune --teacher-steps 0 > gpurun_out/b100_$f.json 2> gpurun_out/b100_$f.err || { tail -30 gpurun_out/b100_$f.err; exit 1; }
echo "fold=$f $(grep '\[bench\] 1 GPU' gpurun_out/b100_$f.err)"
TP_WINO_FOLD=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-baseline --no-prune --teacher-steps 0 > gpurun_out/b2048_$f.json 2> gpurun_out/b2048_$f.err || { tail -30 gpurun_out/b2048_$f.err; exit 1; }
echo "fold=$f $(grep '\[bench\] 1 GPU' gpurun_out/b2048_$f.err)"
done
timeout -k 10 200 python scripts/wino_data_dependence.py > gpurun_out/wino_data.txt 2>&1 || { tail -20 gpurun_out/wino_data.txt; exit 1; }
cat gpurun_out/wino_data.txt

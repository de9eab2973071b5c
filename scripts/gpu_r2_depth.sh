# batches in flight: 2 vs 3 (VGG16 Taylor B=100 / 2048, ResNet-50 APoZ B=256)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for D in 3 2; do
  TORCHPRUNER_STREAMS_DEPTH=$D timeout -k 10 300 python -u bench.py --no-prune --no-baseline --batch 100 --steps 200 --warmup 20 > gpurun_out/depth${D}_b100.log 2>&1 || { tail -30 gpurun_out/depth${D}_b100.log; exit 1; }
  echo "depth=$D $(grep '\[bench\] 1 GPU' gpurun_out/depth${D}_b100.log)"
  TORCHPRUNER_STREAMS_DEPTH=$D timeout -k 10 300 python -u bench.py --no-prune --no-baseline --steps 40 --warmup 5 > gpurun_out/depth${D}_b2048.log 2>&1 || { tail -30 gpurun_out/depth${D}_b2048.log; exit 1; }
  echo "depth=$D $(grep '\[bench\] 1 GPU' gpurun_out/depth${D}_b2048.log)"
  TORCHPRUNER_STREAMS_DEPTH=$D timeout -k 10 300 python -u -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 10 > gpurun_out/depth${D}_rn.log 2>&1 || { tail -30 gpurun_out/depth${D}_rn.log; exit 1; }
  echo "depth=$D $(tail -1 gpurun_out/depth${D}_rn.log | cut -c1-120)"
done

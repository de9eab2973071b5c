# two-stream pipeline on ResNet-50 B=256 (size threshold lifted) vs one stream
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for M in apoz taylor; do
  for S in 1000000000 0; do
    TORCHPRUNER_STREAMS_MAX_PIXELS=$S timeout -k 10 300 python -u -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 10 --metric $M > gpurun_out/pipe6_${M}_$S.log 2>&1 || { tail -30 gpurun_out/pipe6_${M}_$S.log; exit 1; }
    echo "max_pixels=$S $(tail -1 gpurun_out/pipe6_${M}_$S.log | cut -c1-130)"
  done
done

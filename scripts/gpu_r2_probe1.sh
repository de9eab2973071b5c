# dgrad-vs-forward Winograd gap probe + current ResNet-50 APoZ/Taylor numbers
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u scripts/wino_data_dependence.py > gpurun_out/wino_dd.log 2>&1 || { tail -30 gpurun_out/wino_dd.log; exit 1; }
cat gpurun_out/wino_dd.log | grep -v amdgpu.ids
timeout -k 10 300 python -u -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 10 > gpurun_out/rn_apoz.log 2>&1 || { tail -30 gpurun_out/rn_apoz.log; exit 1; }
tail -1 gpurun_out/rn_apoz.log | cut -c1-400
timeout -k 10 300 python -u -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 10 --metric taylor > gpurun_out/rn_tay.log 2>&1 || { tail -30 gpurun_out/rn_tay.log; exit 1; }
tail -1 gpurun_out/rn_tay.log | cut -c1-400

set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -q -x > gpurun_out/ops5.log 2>&1 || { grep -E "Error|assert|FAILED" gpurun_out/ops5.log | tail -20; exit 1; }
tail -1 gpurun_out/ops5.log
timeout -k 10 300 python scripts/r50_probe.py > gpurun_out/r50_probe2.log 2>&1 || { tail -20 gpurun_out/r50_probe2.log; exit 1; }
grep -v amdgpu gpurun_out/r50_probe2.log
timeout -k 10 300 python -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 10 > gpurun_out/r50_apoz2.log 2>&1 || { tail -20 gpurun_out/r50_apoz2.log; exit 1; }
grep "{" gpurun_out/r50_apoz2.log
timeout -k 10 400 python experiments/prune_finetune.py --rounds 3 --steps 20 --batch 128 > gpurun_out/prune_ft2.log 2>&1 || { tail -20 gpurun_out/prune_ft2.log; exit 1; }
grep "{" gpurun_out/prune_ft2.log

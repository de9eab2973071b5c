set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m torchpruner_amd.bench.resnet50_apoz --batch 128 --steps 5 > gpurun_out/r50_apoz.log 2>&1 || { tail -20 gpurun_out/r50_apoz.log; exit 1; }
grep "{" gpurun_out/r50_apoz.log
timeout -k 10 400 python experiments/prune_finetune.py --rounds 2 --steps 5 --batch 64 > gpurun_out/prune_ft.log 2>&1 || { tail -20 gpurun_out/prune_ft.log; exit 1; }
grep "{" gpurun_out/prune_ft.log
timeout -k 10 300 python experiments/prune_untrained.py --dataset mnist > gpurun_out/unt_mnist.log 2>&1 || { tail -20 gpurun_out/unt_mnist.log; exit 1; }
timeout -k 10 300 python experiments/prune_untrained.py --dataset cifar10 > gpurun_out/unt_cifar.log 2>&1 || { tail -20 gpurun_out/unt_cifar.log; exit 1; }
grep "{" gpurun_out/unt_mnist.log gpurun_out/unt_cifar.log
timeout -k 10 300 python -m pytest tests/test_ablation.py -q > gpurun_out/abl.log 2>&1 || { tail -20 gpurun_out/abl.log; exit 1; }
tail -1 gpurun_out/abl.log

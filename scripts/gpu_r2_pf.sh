set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u experiments/prune_finetune.py --rounds 3 --frac 0.2 --steps 30 --batch 64 --pretrain-steps 80 > gpurun_out/pf1.log 2>&1 || { tail -40 gpurun_out/pf1.log; exit 1; }
tail -12 gpurun_out/pf1.log

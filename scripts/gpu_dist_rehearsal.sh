set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TORCHPRUNER_DIST_BACKEND=gloo TORCHPRUNER_SHARE_GPU=1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 1 --teacher-steps 50 --finetune-steps 0 > gpurun_out/dist2.log 2>&1 || { tail -40 gpurun_out/dist2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/dist2.log | tail -6
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 4 --warmup 1 --no-prune --teacher-steps 0 > gpurun_out/dist4.log 2>&1 || { tail -40 gpurun_out/dist4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/dist4.log | tail -3

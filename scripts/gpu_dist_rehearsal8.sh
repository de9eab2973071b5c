# 8-rank readiness rehearsal on the 1-GPU box: bench.py --gpus 8 self-spawns 8 ranks that share
# the MI355X over gloo (TORCHPRUNER_SHARE_GPU=1), every phase and extra at reduced sizes; the JSON
# carries phase_wall_s (teacher / headline / each extra / accuracy) for the wall-time projection.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TORCHPRUNER_DIST_BACKEND=gloo TORCHPRUNER_SHARE_GPU=1
timeout -k 10 1000 python -u bench.py --gpus 8 --steps 2 --warmup 1 --batch 128 --teacher-steps 50 \
  --baseline-batches 1 --quality-seeds 1 --generic-steps 1 --resnet-steps 1 --resnet-batch 16 \
  --finetune-steps 1 --finetune-batch 8 --finetune-res 64 --q5-res 64 --q5-max-steps 25 \
  > gpurun_out/dist8.json 2> gpurun_out/dist8.log || { tail -40 gpurun_out/dist8.log; exit 1; }
grep "\[bench\]" gpurun_out/dist8.log
python3 -c "import json; d=json.loads(open('gpurun_out/dist8.json').read().strip().splitlines()[-1]); print('n_gpus', d['n_gpus'], 'world_seen', d['world_size_seen'], 'backend', d['dist_backend']); print('phase_wall_s', d['phase_wall_s'])"

set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn -o run --output-format csv -- python3 -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 4 --warmup 1 --channels-last 0 > $R/gpurun_out/prof_rn.log 2>&1 || { tail -30 $R/gpurun_out/prof_rn.log; exit 1; }

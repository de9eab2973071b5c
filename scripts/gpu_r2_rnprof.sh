set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn_taylor -o run --output-format csv -- python3 -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 3 --warmup 1 --metric taylor > $R/gpurun_out/prof_rn_taylor.log 2>&1 || { tail -30 $R/gpurun_out/prof_rn_taylor.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn_apoz -o run --output-format csv -- python3 -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 3 --warmup 1 --metric apoz > $R/gpurun_out/prof_rn_apoz.log 2>&1 || { tail -30 $R/gpurun_out/prof_rn_apoz.log; exit 1; }
cd $R
python scripts/kernel_stats_summary.py gpurun_out/prof_rn_taylor/run_kernel_stats.csv 30
python scripts/kernel_stats_summary.py gpurun_out/prof_rn_apoz/run_kernel_stats.csv 20

set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/prof7 -o probe --output-format csv -- python3 $R/scripts/wino_probe.py > $R/gpurun_out/prof7p.log 2>&1 || { tail -30 $R/gpurun_out/prof7p.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof7 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-prune --train-steps 0 > $R/gpurun_out/prof7.log 2>&1 || { tail -30 $R/gpurun_out/prof7.log; exit 1; }

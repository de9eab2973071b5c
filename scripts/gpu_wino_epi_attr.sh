# Needs an experiment build: TORCHPRUNER_HIPFLAGS=-DTP_WINO_DEBUG python -m torchpruner_amd._build --force
# (the switches are compiled out of normal builds).
# Attribute Winograd bwd epilogue time: TP_WINO_DBG 8 = skip phase 2 (global traffic), 16 = skip
# phase 1 (output transform + LDS park); heuristic kernel choice so every run launches the same configs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp TORCHPRUNER_AUTOTUNE=0
for d in 0 8 16 24; do
  TP_WINO_DBG=$d timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/epi_$d -o run --output-format csv -- python bench.py --steps 4 --warmup 2 --no-prune --teacher-steps 0 > gpurun_out/epi_$d.log 2>&1 || { tail -20 gpurun_out/epi_$d.log; exit 1; }
done
echo done

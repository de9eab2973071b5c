#!/usr/bin/env bash
# One parametrised GPU-box runner (replaces the round 1-5 one-off gpu_*.sh wrappers):
#
#   gpurun -- 'bash scripts/gpu.sh TASK [ARGS...]'      (several tasks: 'bash scripts/gpu.sh a && bash scripts/gpu.sh b')
#
# tasks
#   tests [pytest -k expr]  GPU suite (one process, per-test timeout), then smoke()
#   bench [bench args]      the driver's bench line (default: --steps 20 --warmup 5) -> gpurun_out/bench.json
#   headline-prof           headline step: tuner log + kernel trace with one / two batches in flight
#   train-prof [rounds]     ResNet-50 training step (dense / pruned rounds) + kernel trace of the last round
#   resnet-prof             ResNet-50 APoZ / Taylor engine step kernel traces (B=256)
#   pmc-wino4 S C [dgrad]   two PMC passes of one F(4x4) layer (instruction mix, wait cycles)
#   pmc-lowk CFG            two PMC passes of the 64 -> 256 @ 56 px 1x1 training GEMM, tile config CFG
#   dist N                  N ranks self-launched on this one GPU over gloo, every bench phase at reduced sizes
#   teacher [recipes]       the accuracy protocol's teacher under both wgrad combine orders
#   ddp-overlap [args]      DDP bucket ready times inside the native ResNet-50 backward (1 rank, RCCL)
#   b100                    B=100 (the reference's attribution batch): bench extra + tuner log
# Every GPU step runs under its own timeout; a failing step ends the script (no retries).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p "$O"
export TMPDIR=/tmp
task=${1:-tests}
shift || true

step() {  # step NAME SECONDS CMD...: run, log to gpurun_out/NAME.log, stop on failure
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "[gpu.sh] step $name failed (rc $rc)"
    tail -30 "$O/$name.log"
    exit $rc
  fi
}

case $task in
  tests)
    if [ $# -gt 0 ]; then
      step gpu_tests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "$*"
    else
      step gpu_tests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
    fi
    tail -2 "$O/gpu_tests.log"
    step smoke 300 python __graft_entry__.py smoke
    tail -1 "$O/smoke.log"
    ;;
  bench)
    args=${*:-"--steps 20 --warmup 5"}
    timeout -k 10 900 python -u bench.py $args > "$O/bench.json" 2> "$O/bench.err" || { tail -30 "$O/bench.err"; exit 1; }
    grep "\[bench\]" "$O/bench.err"
    ;;
  headline-prof)
    TORCHPRUNER_TUNER_LOG=1 step hb 300 python -u bench.py --steps 20 --warmup 3 --no-extras --no-prune --no-baseline --teacher-steps 0
    grep "\[bench\]\|\[tuner\]" "$O/hb.log" | sort -u | head -60
    cd /tmp
    for s in 0 1; do
      TORCHPRUNER_STREAMS=$s timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/hprof$s" -o run --output-format csv -- \
        python3 "$R/bench.py" --steps 6 --warmup 2 --no-extras --no-prune --no-baseline --teacher-steps 0 > "$O/hprof$s.log" 2>&1 \
        || { tail -30 "$O/hprof$s.log"; exit 1; }
      echo "== streams=$s"; python3 "$R/scripts/step_breakdown.py" "$(find "$O/hprof$s" -name '*kernel_trace.csv' | head -1)"
    done
    ;;
  train-prof)
    rounds=${1:-0,1,2}
    step train_probe 400 python -u scripts/probes/pruned_train_probe.py --rounds "$rounds"
    grep pruned_train "$O/train_probe.log"
    last=${rounds##*,}
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/train_prof" -o r$last -- \
      python3 scripts/probes/pruned_train_probe.py --rounds "$last" --steps 5 > "$O/train_prof.log" 2>&1 || { tail -20 "$O/train_prof.log"; exit 1; }
    python3 scripts/rocpd_step.py "$O/train_prof/r${last}_results.db" 40
    ;;
  resnet-prof)
    cd /tmp
    for metric in apoz taylor; do
      PYTHONPATH=$R TORCHPRUNER_STREAMS=0 timeout -k 10 300 rocprofv3 --kernel-trace -d "$O/prof_rn/$metric" -o run --output-format csv -- \
        python3 -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 3 --warmup 1 --metric $metric > "$O/prof_rn_$metric.log" 2>&1 \
        || { tail -20 "$O/prof_rn_$metric.log"; exit 1; }
      echo "== $metric"; python3 "$R/scripts/step_breakdown.py" "$(find "$O/prof_rn/$metric" -name '*kernel_trace.csv' | head -1)" "nchw_to_nhwc_pad"
    done
    ;;
  pmc-wino4)
    S=${1:-8}; C=${2:-256}; extra=${3:+--dgrad}
    i=0
    for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES" \
               "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_INSTS_SMEM"; do
      i=$((i+1))
      timeout -s KILL 90 rocprofv3 --pmc $grp -d "$O/pmcw4_$i" -o run --output-format csv -- \
        python3 scripts/probes/wino4_layer_probe.py --S "$S" --C "$C" --K "$C" --variant 3 $extra > "$O/pmcw4_$i.log" 2>&1 \
        || { echo "pass $i failed"; tail -3 "$O/pmcw4_$i.log"; exit 1; }
    done
    python3 scripts/pmc_table.py "$O/pmcw4_[12]/**/*counter_collection.csv"
    ;;
  pmc-lowk)
    cfg=${1:-66}
    i=0
    for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES" \
               "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_INSTS_SMEM"; do
      i=$((i+1))
      timeout -s KILL 90 rocprofv3 --pmc $grp -d "$O/pmclowk_$i" -o run --output-format csv -- \
        python3 scripts/probes/lowk_gemm_probe.py --one 128 56 64 256 "$cfg" 1 > "$O/pmclowk_$i.log" 2>&1 \
        || { echo "pass $i failed"; tail -3 "$O/pmclowk_$i.log"; exit 1; }
    done
    python3 scripts/pmc_table.py "$O/pmclowk_[12]/**/*counter_collection.csv"
    ;;
  dist)
    N=${1:-4}
    TORCHPRUNER_DIST_BACKEND=gloo TORCHPRUNER_SHARE_GPU=1 step dist$N 1000 python -u bench.py --gpus "$N" --steps 2 --warmup 1 \
      --batch 128 --teacher-steps 50 --baseline-batches 1 --quality-seeds 1 --generic-steps 1 --resnet-steps 1 --resnet-batch 16 \
      --finetune-steps 1 --finetune-batch 8 --finetune-res 64 --q5-res 64 --q5-max-steps 25
    grep "\[bench\]" "$O/dist$N.log"
    ;;
  teacher)
    recipes=${*:-"lr=0.05"}
    step teach_default 600 python -u scripts/probes/teacher_robustness.py --seeds 0 1 2 --recipes $recipes
    TP_WGRAD_COMBINE_LANES=1 step teach_lanes1 600 python -u scripts/probes/teacher_robustness.py --seeds 0 1 2 --recipes $recipes
    grep -h recipe "$O/teach_default.log" "$O/teach_lanes1.log"
    ;;
  ddp-overlap)
    step ddp_overlap 400 python -u scripts/probes/ddp_overlap_probe.py "$@"
    grep ddp_overlap "$O/ddp_overlap.log"
    ;;
  b100)
    TORCHPRUNER_TUNER_LOG=1 step b100 400 python -u bench.py --steps 2 --warmup 1 --teacher-steps 0 --no-prune --no-baseline --extras b100
    grep "\[bench\]" "$O/b100.log"
    ;;
  *)
    echo "unknown task $task"; exit 2
    ;;
esac

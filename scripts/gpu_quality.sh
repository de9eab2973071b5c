set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "3.0 0 150" "3.0 1 150" "4.0 0 150" "4.0 1 150" "4.0 0 300" "5.0 0 300" "5.0 1 300" "6.0 0 400"; do
  set -- $cfg
  NOISE=$1 TSEED=$2 TEACHER_STEPS=$3 timeout -k 10 300 python scripts/quality_check.py > gpurun_out/q_$1_$2_$3.log 2>&1 || { tail -30 gpurun_out/q_$1_$2_$3.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/q_$1_$2_$3.log | grep -v "^direct\|^hook\|per-layer"
done

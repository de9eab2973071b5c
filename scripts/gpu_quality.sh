set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "2.0 4 0 300" "2.0 4 1 300" "3.0 4 0 300" "2.0 8 0 300" "2.0 8 1 300" "3.0 8 0 400" "1.5 16 0 400" "1.5 16 1 400"; do
  set -- $cfg
  NOISE=$1 MODES=$2 TSEED=$3 TEACHER_STEPS=$4 timeout -k 10 300 python scripts/quality_check.py > gpurun_out/qm_$1_$2_$3.log 2>&1 || { tail -30 gpurun_out/qm_$1_$2_$3.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/qm_$1_$2_$3.log | grep -v "^direct\|^hook"
done

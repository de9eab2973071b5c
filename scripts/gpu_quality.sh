set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "2.0 1" "2.0 2" "8.0 0" "8.0 1" "16.0 0" "16.0 1" "24.0 0"; do
  set -- $cfg
  NOISE=$1 TSEED=$2 timeout -k 10 300 python scripts/quality_check.py > gpurun_out/q_$1_$2.log 2>&1 || { tail -30 gpurun_out/q_$1_$2.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/q_$1_$2.log | grep -v "^direct\|^hook"
done

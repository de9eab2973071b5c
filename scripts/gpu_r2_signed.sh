set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python scripts/signed_taylor_probe.py 2>&1 | grep -v amdgpu.ids
TORCHPRUNER_AUTOTUNE=0 timeout -k 10 200 python scripts/signed_taylor_probe.py 2>&1 | grep -v amdgpu.ids

# Shapley prefix-delta GEMM: equivalence tests, nbUNT (MLP) timing, VGG deep-layer Shapley bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mlp_engine_gpu.py tests/test_pruned_engine_gpu.py tests/test_conv_gpu.py -k "shapley or mlp" -x -q --timeout 200 --timeout-method thread > gpurun_out/delta_tests.log 2>&1 || { tail -60 gpurun_out/delta_tests.log; exit 1; }
tail -2 gpurun_out/delta_tests.log
for d in mnist cifar10; do
  timeout -k 10 200 python experiments/prune_untrained.py --dataset $d > gpurun_out/unt_$d.log 2>&1 || { tail -30 gpurun_out/unt_$d.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/unt_$d.log | tail -1
done
TORCHPRUNER_PREFIX_DELTA=0 timeout -k 10 200 python experiments/prune_untrained.py --dataset mnist > gpurun_out/unt_mnist_copies.log 2>&1 || { tail -30 gpurun_out/unt_mnist_copies.log; exit 1; }
grep -v amdgpu.ids gpurun_out/unt_mnist_copies.log | tail -1
timeout -k 10 300 python -m torchpruner_amd.bench.shapley_vgg --layers 11,12,13,14 --json gpurun_out/shapley_deep_delta.json > gpurun_out/shap_delta.log 2>&1 || { tail -20 gpurun_out/shap_delta.log; exit 1; }
TORCHPRUNER_PREFIX_DELTA=0 timeout -k 10 300 python -m torchpruner_amd.bench.shapley_vgg --layers 11,12,13,14 --json gpurun_out/shapley_deep_copies.json > gpurun_out/shap_copies.log 2>&1 || { tail -20 gpurun_out/shap_copies.log; exit 1; }
python - <<'PY'
import json
for n in ("delta", "copies"):
    d = json.load(open(f"gpurun_out/shapley_deep_{n}.json"))
    print(n, [(l["layer"], l["units"], l["seconds"]) for l in d["layers"]])
PY

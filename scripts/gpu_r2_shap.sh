# Shapley (config #4 shape: B=100, S=5) GPU occupancy: wall vs kernel-busy time per layer run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m torchpruner_amd.bench.shapley_vgg --layers 0,6,12 > gpurun_out/shap.log 2>&1 || { tail -30 gpurun_out/shap.log; exit 1; }
grep -v amdgpu.ids gpurun_out/shap.log | tail -6
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/sh -o run --output-format csv -- python -m torchpruner_amd.bench.shapley_vgg --layers 6 > gpurun_out/shap_tr.log 2>&1 || { tail -30 gpurun_out/shap_tr.log; exit 1; }
python - <<'PY' $(find /tmp/sh -name "*kernel_trace.csv" | head -1)
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[len(rows) // 2:]  # second half: steady state
t0 = int(rows[0]["Start_Timestamp"]); t1 = max(int(r["End_Timestamp"]) for r in rows)
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
print(f"layer 6, second half of the kernels: wall {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us ({busy / (t1 - t0):.0%}), {len(rows)} launches")
PY
rm -rf /tmp/sh

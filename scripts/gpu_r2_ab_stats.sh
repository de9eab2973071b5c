set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 1 0 1 0; do
TORCHPRUNER_BN_EPI_STATS=$v FMTS=native N=20 timeout -k 10 300 python scripts/r50_train_probe.py > gpurun_out/train_probe_$v.log 2>&1 || { tail -30 gpurun_out/train_probe_$v.log; exit 1; }
echo "stats=$v $(grep 'img/s' gpurun_out/train_probe_$v.log)"
done

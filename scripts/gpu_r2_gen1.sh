set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_resnet_bwd_gpu.py tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gen1_tests.log 2>&1 || { tail -60 gpurun_out/gen1_tests.log; exit 1; }
tail -1 gpurun_out/gen1_tests.log
timeout -k 10 300 python -u scripts/r50_conv_roofline.py > gpurun_out/r50_roofline3.txt 2>&1 || { tail -30 gpurun_out/r50_roofline3.txt; exit 1; }
cat gpurun_out/r50_roofline3.txt
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -m torchpruner_amd.bench.resnet50_apoz --batch 256 --steps 8 --warmup 2 --metric apoz > gpurun_out/rn_apoz.log 2>&1 || { tail -30 gpurun_out/rn_apoz.log; exit 1; }
tail -1 gpurun_out/rn_apoz.log | cut -c1-140
FMTS=native N=10 timeout -k 10 300 python scripts/r50_train_probe.py > gpurun_out/train_probe.log 2>&1 || { tail -30 gpurun_out/train_probe.log; exit 1; }
grep "img/s" gpurun_out/train_probe.log
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/gemm_pmc2 -o run --output-format csv -- python3 $R/scripts/gemm_pmc_probe.py > $R/gpurun_out/gemm_pmc2.log 2>&1 || { tail -20 $R/gpurun_out/gemm_pmc2.log; exit 1; }
echo pmc-ok

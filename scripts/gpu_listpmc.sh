cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/pmc_list.txt 2>&1
grep -oE "^[[:space:]]*(TA_|TCP_|TD_|SQ_INSTS|SQ_INST_|SQ_LDS|SQ_WAIT|SQ_BUSY|SQ_ACTIVE|SQC_|TCC_HIT|TCC_MISS|TCC_EA0_RDREQ|SQ_VALU|GRBM)[A-Za-z0-9_]*" $GRAFT_REPO_ROOT/gpurun_out/pmc_list.txt | sort -u | tr -d ' ' | tr '\n' ' ' | head -c 6000

cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ic
timeout -k 10 120 rocprofv3 -L > gpurun_out/ic/avail.txt 2>&1 || true
grep -iE "ICACHE|SQC_|IFETCH|INST_LEVEL|SQ_WAIT_INST|SQ_INSTS_" gpurun_out/ic/avail.txt | head -80 > gpurun_out/ic/avail_sel.txt || true
echo listed

#!/bin/bash
# Texture-unit / LDS FIFO pressure of the MLP kernels (two --pmc passes, counters only).
# usage: tools/pmc_ta.sh OUTDIR [bench args...]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; shift
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-integrator --no-alt $*"
mkdir -p $OUT
i=0
for pass in "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CU_CYCLES SQ_INST_LEVEL_VMEM" \
            "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE"; do
  timeout -s KILL 120 rocprofv3 --pmc $pass -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  i=$((i+1))
done
python3 tools/pmc_diag_summary.py $OUT

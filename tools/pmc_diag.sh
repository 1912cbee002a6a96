#!/bin/bash
# Per-kernel SQ counter passes (one rocprofv3 run per pass, --pmc only: never with runtime/sys traces).
# usage: tools/pmc_diag.sh OUTDIR [bench args...]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; shift
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-integrator --no-alt $*"
mkdir -p $OUT
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
            "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" \
            "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" \
            "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  timeout -k 10 240 rocprofv3 --pmc $pass -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1
  i=$((i+1))
done
python3 tools/pmc_diag_summary.py $OUT

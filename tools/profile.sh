#!/bin/bash
# rocprofv3 evidence for the bench: kernel trace + stats, then separate PMC passes (FETCH_SIZE,
# WRITE_SIZE, GRBM_GUI_ACTIVE) — counters never combined with runtime/sys tracing, and FETCH_SIZE /
# WRITE_SIZE never in the same pass.   usage: tools/profile.sh OUTDIR [extra bench args]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/prof}; shift || true
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-integrator --no-alt $*"
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_fetch.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_write.log 2>&1
timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES -d $OUT/pmc_clk -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc_clk.log 2>&1
echo done

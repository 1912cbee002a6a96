#!/bin/bash
# Round-2 rocprofv3 evidence, one tag per run:
#   per precision mode: kernel trace + stats, then separate --pmc passes
#     FETCH_SIZE | WRITE_SIZE | SQ_VALU_MFMA_BUSY_CYCLES + SQ_BUSY_CYCLES + GRBM_GUI_ACTIVE
#     [| SQ_LDS_IDX_ACTIVE + SQ_LDS_BANK_CONFLICT + GRBM_GUI_ACTIVE with LDS=1]
#   integrator-only 2^20 x 128 batch: trace, FETCH_SIZE, WRITE_SIZE
# counters never combined with runtime/sys traces; every pass under its own time limit.
# usage: tools/profile_r02.sh TAG [precisions...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r02}; shift
PRECS=${*:-f32 split f16x2}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-integrator --no-alt --no-config4 --no-config5"
run() {  # name, then the rocprofv3 options
  local name=$1; shift
  echo "$(date +%T) $name" >> $OUT/progress.log
  timeout -k 10 240 rocprofv3 "$@" -- python3 "${CMD[@]}" > $OUT/$name.log 2>&1 || { echo "FAILED $name rc=$?"; tail -20 $OUT/$name.log; exit 1; }
}
for p in $PRECS; do
  CMD=(bench.py $ARGS --precision $p)
  run ${p}_trace --kernel-trace --stats -d $OUT/$p/trace -o run --output-format csv
  run ${p}_fetch --pmc FETCH_SIZE -d $OUT/$p/pmc_fetch -o run --output-format csv
  run ${p}_write --pmc WRITE_SIZE -d $OUT/$p/pmc_write -o run --output-format csv
  run ${p}_mfma --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/$p/pmc_clk -o run --output-format csv
done
# roctx phase ranges beside the kernel trace (marker domain; no counters in this pass)
CMD=(bench.py $ARGS --precision f32)
run roctx_f32 --marker-trace --kernel-trace -d $OUT/roctx -o run --output-format csv
CMD=(tools/integrator_only.py)
run integ_trace --kernel-trace --stats -d $OUT/integrator/trace -o run --output-format csv
run integ_fetch --pmc FETCH_SIZE -d $OUT/integrator/pmc_fetch -o run --output-format csv
run integ_write --pmc WRITE_SIZE -d $OUT/integrator/pmc_write -o run --output-format csv
# LDS-array occupancy (LDS=1): the forwards' A-fragment reads against the 256 B/clk/CU array; last,
# so an unsupported counter cannot cost the passes above
if [ -n "$LDS" ]; then
  for p in $PRECS; do
    CMD=(bench.py $ARGS --precision $p)
    run ${p}_lds --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $OUT/$p/pmc_lds -o run --output-format csv
  done
fi
echo done >> $OUT/progress.log
echo done

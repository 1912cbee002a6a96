#!/bin/bash
# SQ issue/wait counters for the F16 config-2 step (separate --pmc passes, each its own run).
# usage: tools/sq_pass.sh TAG [NOF_LIB]
TAG=${1:-sq}
[ -n "$2" ] && export NOF_LIB=$2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
CMD="python3 bench.py --no-cpu-baseline --no-integrator --no-alt --no-config4 --no-config5 --precision f16 --steps 10 --warmup 2"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/counters_$TAG.txt 2>&1 || true
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/${TAG}_p$i -o p -- $CMD > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
done
echo done

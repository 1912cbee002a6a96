#!/bin/bash
# Side-output write accounting: for the product library and the default-policy
# store variant (python tools/diag/variant.py nont store_default -> build_diag/nont), per precision mode,
# a kernel trace and separate FETCH_SIZE / WRITE_SIZE passes.  Summaries: tools/pmc_summary.py
# gpurun_out/abw_<variant>/<prec> <tag>.   usage: PRECS="f32 f16split" tools/ab_write.sh
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
ARGS="--steps 5 --warmup 2 --no-cpu-baseline --no-integrator --no-alt --no-config4 --no-config5"
for v in nont -; do
  lib=$PWD/nerf-or-nothing_amd/lib/libnof.so; tag=nt
  [ "$v" != "-" ] && { lib=$PWD/build_diag/$v/nerf-or-nothing_amd/lib/libnof.so; tag=$v; }
  for p in ${PRECS:-f32 f16split}; do
    OUT=gpurun_out/abw_$tag/$p
    mkdir -p $OUT
    for pass in "trace --kernel-trace --stats" "pmc_fetch --pmc FETCH_SIZE" "pmc_write --pmc WRITE_SIZE"; do
      set -- $pass; name=$1; shift
      echo "$(date +%T) $tag $p $name"
      NOF_LIB=$lib timeout -k 10 240 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- python3 bench.py $ARGS --precision $p > $OUT/$name.log 2>&1 || { echo "FAILED $tag $p $name"; tail -20 $OUT/$name.log; exit 1; }
    done
  done
done
echo done

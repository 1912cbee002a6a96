#!/bin/bash
# A/B timing of several builds in one box session: for each v in VARIANTS ("-" = lib/libnof.so) the patched-tree
# build build_diag/<v> (tools/diag/variant.py) or else lib/libnof_<v>.so,
# alternating, REPS rounds.  usage: VARIANTS="base -" PRECS="f16" REPS=2 tools/ab_multi.sh
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for v in ${VARIANTS:-base -}; do
    lib=nerf-or-nothing_amd/lib/libnof.so
    [ "$v" != "-" ] && lib=nerf-or-nothing_amd/lib/libnof_$v.so
    [ "$v" != "-" ] && [ -f build_diag/$v/nerf-or-nothing_amd/lib/libnof.so ] && lib=build_diag/$v/nerf-or-nothing_amd/lib/libnof.so
    for p in ${PRECS:-f16}; do
      NOF_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-integrator --no-alt --no-config4 --no-config5 --precision $p > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$v $p', d['value'], d['ms_per_step'], {k:v['avg_launch_ms'] for k,v in d['kernels'].items() if k in ('mlp_fwd','mlp_bwd','wgrad','wgrad_reduce')})"
    done
  done
done

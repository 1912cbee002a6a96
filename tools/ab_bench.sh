#!/bin/bash
# A/B timing of two builds in one box session: lib/libnof_${A}.so vs lib/libnof.so, alternating
# usage: A=old PRECS="f32 f16x2" REPS=2 tools/ab_bench.sh
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for lib in nerf-or-nothing_amd/lib/libnof_${A:-old}.so nerf-or-nothing_amd/lib/libnof.so; do
    for p in ${PRECS:-f32 f16x2}; do
      NOF_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-integrator --no-alt --no-config4 --no-config5 --precision $p > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
      python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$(basename $lib) $p', d['value'], d['ms_per_step'], {k:v['avg_launch_ms'] for k,v in d['kernels'].items() if k in ('mlp_fwd','mlp_bwd','wgrad')})"
    done
  done
done

#!/bin/bash
# Timing of diagnostic library builds (build_diag/VARIANT from tools/diag/variant.py, or lib/libnof_VARIANT.so;
# "" = product) for one precision.
# usage: PREC=f32 tools/diag_lib.sh VARIANT...   (results of diagnostic builds are garbage)
mkdir -p gpurun_out
for v in "" "$@"; do
  lib=nerf-or-nothing_amd/lib/libnof${v:+_$v}.so
  [ -n "$v" ] && [ -f build_diag/$v/nerf-or-nothing_amd/lib/libnof.so ] && lib=build_diag/$v/nerf-or-nothing_amd/lib/libnof.so
  NOF_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-integrator --no-alt --steps 20 --warmup 3 --precision ${PREC:-f32} > gpurun_out/dl_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/dl_$v.json')); k=d['kernels']; print('${v:-full}', {n:round(x['avg_launch_ms'],4) for n,x in k.items() if n.startswith(('mlp','wgrad'))})"
done

#!/bin/bash
# MLP-kernel overhead split: the full kernels vs diagnostic builds (timing only; results are garbage).
# usage: tools/diag_fwd.sh VARIANT...   (lib/libnof_VARIANT.so built by make VARIANT=.. DIAG=..; "" = product)
mkdir -p gpurun_out
for v in "" "$@"; do
  for p in f32 split; do
    lib=nerf-or-nothing_amd/lib/libnof${v:+_$v}.so
    NOF_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-integrator --no-alt --steps 20 --warmup 3 --precision $p > gpurun_out/df_$v$p.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/df_$v$p.json')); k=d['kernels']; print('${v:-full} $p', {n:round(x['avg_launch_ms'],4) for n,x in k.items() if n.startswith(('mlp','wgrad'))})"
  done
done

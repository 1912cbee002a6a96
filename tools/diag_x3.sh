#!/bin/bash
mkdir -p gpurun_out
for v in "" nosplit nomfma; do
  lib=nerf-or-nothing_amd/lib/libnof${v:+_$v}.so
  NOF_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-integrator --no-alt --steps 20 --warmup 3 --precision split > gpurun_out/dx_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/dx_$v.json')); k=d['kernels']; print('$v', d['ms_per_step'], {n:round(x['avg_launch_ms'],4) for n,x in k.items()})"
done

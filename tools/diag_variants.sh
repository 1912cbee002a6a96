set -e
mkdir -p gpurun_out
for v in "" nostore noipe both; do
  lib=nerf-or-nothing_amd/lib/libnof${v:+_$v}.so
  NOF_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --no-integrator --steps 30 --warmup 5 > gpurun_out/diag_$v.json 2>/dev/null
  python -c "import json,sys; d=json.load(open('gpurun_out/diag_$v.json')); k=d['kernels']; print('$v', d['ms_per_step'], {n:round(x['avg_launch_ms'],4) for n,x in k.items()})"
done

for r in 512 1024 2048 4096; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-integrator --no-alt --no-config4 --no-config5 --precision f16 --rays $r --steps 30 > gpurun_out/sw.json 2>gpurun_out/sw.err || { tail gpurun_out/sw.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sw.json')); print('$r', d['value'], d['ms_per_step'], {k:v['avg_launch_ms'] for k,v in d['kernels'].items()})"
done

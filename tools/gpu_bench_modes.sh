mkdir -p gpurun_out
for rep in 1 2; do for p in f16 f16x2 f16split; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-integrator --no-alt --no-config4 --no-config5 --precision $p > gpurun_out/b_$p.json 2>gpurun_out/b_$p.err || { tail gpurun_out/b_$p.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b_$p.json')); print('$p', d['value'], d['ms_per_step'], d['roofline']['frac'], {k:v['avg_launch_ms'] for k,v in d['kernels'].items() if k in ('mlp_fwd','mlp_bwd','wgrad')})"
done; done

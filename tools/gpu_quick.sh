mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
for p in ${PRECS:-f32}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-integrator --no-alt --precision $p > gpurun_out/b_$p.json 2>gpurun_out/b_$p.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/b_$p.json')); print('$p', d['value'], d['ms_per_step'], d['roofline']['frac'], {k:v['avg_launch_ms'] for k,v in d['kernels'].items()})"
done

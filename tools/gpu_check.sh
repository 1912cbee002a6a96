#!/bin/bash
# GPU tests + short benches of both precision modes (one gpurun call).
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1
rc=$?
tail -15 gpurun_out/t.log
[ $rc -ne 0 ] && exit $rc
for p in f32 split; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-integrator --no-alt --precision $p > gpurun_out/b_$p.json 2>gpurun_out/b_$p.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/b_$p.json')); print('$p', d['value'], d['ms_per_step'], d['roofline']['frac'], {k:v['avg_launch_ms'] for k,v in d['kernels'].items()})"
done

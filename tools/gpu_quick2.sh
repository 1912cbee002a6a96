#!/bin/bash
# parity of the MLP kernels (all modes) + short benches of the named precision modes
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_fullsize.py tests/test_gpu_numeric.py -x -q --timeout 150 --timeout-method thread > gpurun_out/tq.log 2>&1 || { tail -30 gpurun_out/tq.log; exit 1; }
tail -2 gpurun_out/tq.log
for p in ${PRECS:-f32 f16x2}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-integrator --no-alt --no-config4 --no-config5 --precision $p > gpurun_out/b_$p.json 2>gpurun_out/b_$p.err || { tail gpurun_out/b_$p.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b_$p.json')); print('$p', d['value'], d['ms_per_step'], d['roofline']['frac'], {k:v['avg_launch_ms'] for k,v in d['kernels'].items()})"
done

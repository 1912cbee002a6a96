#!/bin/bash
# smoke (the driver's order: build + smoke through __main__) + the default bench line, one gpurun call.
# usage: tools/gpu_bench.sh TAG [bench args...]
TAG=${1:-run}; shift
mkdir -p gpurun_out
timeout -k 10 180 python -u __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 420 python bench.py "$@" > gpurun_out/b_$TAG.json 2>gpurun_out/b_$TAG.err || { tail -20 gpurun_out/b_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b_$TAG.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('config4_1gpu', {}).get('value'), [(x['precision'], x['value'], x['roofline']['frac']) for x in d.get('alt_precision', [])], d.get('cpu_baseline', {}).get('value'), d.get('roofline_integrator', {}).get('frac'))"

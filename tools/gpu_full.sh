#!/bin/bash
# Full GPU suite + the default bench line (what the driver runs at round end), one gpurun call.
# usage: tools/gpu_full.sh TAG
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
rc=$?; tail -8 gpurun_out/t_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/b_$TAG.json 2>gpurun_out/b_$TAG.err || { tail -20 gpurun_out/b_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b_$TAG.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('config4_1gpu', {}).get('value'), [(x['precision'], x['value'], x['roofline']['frac']) for x in d.get('alt_precision', [])], d['cpu_baseline']['value'], d['roofline_integrator']['frac'])"

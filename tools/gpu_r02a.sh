#!/bin/bash
# round 2: new GPU tests (accumulation, buckets, DP failure paths, bench modes) + a default bench line
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_accum_dp.py tests/test_gpu_bench_dp.py -x -v -s --timeout 150 --timeout-method thread > gpurun_out/t2.log 2>&1
rc=$?; tail -25 gpurun_out/t2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-integrator > gpurun_out/b_default.json 2>gpurun_out/b_default.err || { tail -20 gpurun_out/b_default.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b_default.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('config4_1gpu'), [(x['precision'], x['value']) for x in d.get('alt_precision', [])])"

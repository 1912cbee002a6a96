#!/bin/bash
# F16-mode iteration on the box: the semantics probe, the F16 parity tests (step, edges, determinism),
# then a short bench of the F16 mode.  usage: tools/gpu_f16.sh [extra pytest -k filter]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 60 ./tools/probe/h32_probe | tee gpurun_out/h32_probe.txt || exit 1
K=${1:-"(step_parity and 4]) or deterministic[4] or masked_rays[4]"}
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_step.py tests/test_gpu_edges.py -k "$K" > gpurun_out/f16_tests.log 2>&1
rc=$?; tail -30 gpurun_out/f16_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline --no-integrator --no-alt --no-config4 --no-config5 --precision f16 > gpurun_out/b_f16.json 2>gpurun_out/b_f16.err || { tail gpurun_out/b_f16.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/b_f16.json')); print('f16', d['value'], d['ms_per_step'], d['roofline'], {k:v['avg_launch_ms'] for k,v in d['kernels'].items()})"

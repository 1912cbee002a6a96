cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for p in f32 f16; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04i/$p -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-integrator --no-alt --no-config4 --no-config5 --precision $p > gpurun_out/prof_r04i_$p.log 2>&1 || exit 1
done
echo done

#!/bin/bash
# Per-kernel average durations of two library builds under rocprofv3 --kernel-trace --stats (one F16
# bench run each): usage VARIANTS="base -" tools/ab_kernel_trace.sh [kernel-name regex]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/abk
for v in ${VARIANTS:-base -}; do
  lib=nerf-or-nothing_amd/lib/libnof.so
  [ "$v" != "-" ] && lib=build_diag/$v/nerf-or-nothing_amd/lib/libnof.so
  d=gpurun_out/abk/${v/-/product}
  NOF_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-integrator --no-alt --no-config4 --no-config5 --precision ${PREC:-f16} > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  f=$(find $d -name "run_kernel_stats.csv" | head -1)
  echo "== $v"
  python3 - "$f" "${1:-.}" <<'PY'
import csv, re, sys
for r in list(csv.reader(open(sys.argv[1])))[1:]:
    if re.search(sys.argv[2], r[0], re.I):
        print(f"  {r[0][:60]:60s} calls {r[1]:>5s} avg_us {float(r[3]) / 1e3:9.2f}")
PY
done

#!/bin/bash
# A/B of the any-shape path (tools/generic_steps.py, configs[0]) over build variants: VARIANTS="- name ..."
for rep in $(seq ${REPS:-2}); do
  for v in ${VARIANTS:-"-"}; do
    lib=nerf-or-nothing_amd/lib/libnof.so
    [ "$v" != "-" ] && lib=build_diag/$v/nerf-or-nothing_amd/lib/libnof.so
    echo -n "$v "
    NOF_LIB=$PWD/$lib timeout -k 10 200 python tools/generic_steps.py --steps 20 2>/dev/null | tail -1 || exit 1
  done
done

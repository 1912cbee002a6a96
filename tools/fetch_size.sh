#!/bin/bash
# FETCH_SIZE per kernel (its own rocprofv3 pass; FETCH_SIZE and WRITE_SIZE cannot share a pass)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/fs; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/p -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-integrator --no-alt "$@" > $OUT/log 2>&1 || exit 1
python3 - <<'PY'
import csv, collections
a = collections.defaultdict(list)
for r in csv.DictReader(open("gpurun_out/fs/p/run_counter_collection.csv")):
    a[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]))
for k, v in sorted(a.items()):
    print(f"{k:40s} FETCH_SIZE {sum(v)/len(v)/1e6:.3f} GB/launch (KB units; x2 per the gfx950 correction)")
PY

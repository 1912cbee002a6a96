"""Per-(kernel, grid) launch counts and average durations of a rocprofv3 --kernel-trace CSV: the default
bench run mixes workloads (config 2, configs[2..4], the render and PSNR legs), so a kernel's overall
average in run_kernel_stats.csv is not the headline launch's; the grid separates them.

usage: trace_by_grid.py run_kernel_trace.csv [kernel-name regex] [out.json]
"""
import collections
import csv
import json
import re
import sys

src = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
g = collections.defaultdict(list)
for r in csv.DictReader(open(src)):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("nof::", "")
    if not pat.search(name):
        continue
    grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    g[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
out = {f"{k} grid {grid}": {"calls": len(v), "avg_ms": round(sum(v) / len(v), 4), "min_ms": round(min(v), 4)}
       for (k, grid), v in sorted(g.items())}
for k, v in out.items():
    print(k, v)
if len(sys.argv) > 3:
    json.dump(out, open(sys.argv[3], "w"), indent=1)

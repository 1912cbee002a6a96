"""One training step's dispatches from a rocprofv3 --kernel-trace CSV (the last complete step, between the
last two k_adam launches): per-dispatch microseconds and grid, plus totals per kernel name.
usage: python tools/trace_step.py gpurun_out/<dir>/t_kernel_trace.csv [--quiet]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
idx = [i for i, r in enumerate(rows) if "k_adam" in r["Kernel_Name"]]
s, e = idx[-2] + 1, idx[-1] + 1
tot = collections.Counter()
for r in rows[s:e]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    name = r["Kernel_Name"].split("(")[0]
    tot[name] += d
    if "--quiet" not in sys.argv:
        print(f"{d:8.1f} us  grid {r['Grid_Size_X']:>9}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']:<4} {name}")
span = (int(rows[e - 1]["End_Timestamp"]) - int(rows[s]["Start_Timestamp"])) / 1000
for k, v in tot.most_common():
    print(f"{v:9.1f} us  {k}")
print(f"sum {sum(tot.values()):.1f} us, span {span:.1f} us")

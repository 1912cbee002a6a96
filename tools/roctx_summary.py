"""Summarise a rocprofv3 --marker-trace run (run_marker_api_trace.csv) into per-range host times:
range, count, mean and max microseconds (profiles/<tag>_roctx_ranges.csv).

usage: python tools/roctx_summary.py gpurun_out/prof_TAG/roctx/run_marker_api_trace.csv profiles/TAG_roctx_ranges.csv
"""
import collections
import csv
import sys

src, dst = sys.argv[1], sys.argv[2]
d = collections.defaultdict(list)
for r in csv.DictReader(open(src)):
    d[r["Function"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
with open(dst, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["range", "count", "avg_host_us", "max_host_us"])
    for k in sorted(d):
        v = d[k]
        w.writerow([k, len(v), round(sum(v) / len(v), 1), round(max(v), 1)])
print(open(dst).read())

"""Per-shape counters of an any-shape-path profile (tools/_cmd_gpmc6.sh: a kernel trace, then FETCH_SIZE,
WRITE_SIZE and MFMA-busy passes of tools/generic_steps.py, each its own run): one row per (kernel, grid
size), since one kernel name covers several GEMM shapes.

traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 B (gfx950 correction, as tools/pmc_summary.py);
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs).

usage: pmc_by_shape.py SRC_DIR TAG  ->  profiles/TAG_pmc_by_shape.json, profiles/TAG_kernel_stats.csv
"""
import collections
import csv
import json
import os
import shutil
import sys

src, tag = sys.argv[1], sys.argv[2]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, "profiles")
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
short = lambda n: n.split("(")[0].replace("void ", "").replace("nof::", "")

dur = collections.defaultdict(list)
for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))):
    grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
    dur[(short(r["Kernel_Name"]), grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
ctr = collections.defaultdict(list)
for sub in ("pmc_fetch", "pmc_write", "pmc_clk"):
    p = os.path.join(src, sub, "run_counter_collection.csv")
    for r in csv.DictReader(open(p)):
        ctr[(short(r["Kernel_Name"]), int(r["Grid_Size"]), r["Counter_Name"])].append(float(r["Counter_Value"]))

mean = lambda v: sum(v) / len(v) if v else None
out = {}
for (k, grid), us in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    if not k.startswith("k_"):
        continue
    m = lambda c: mean(ctr.get((k, grid, c), []))
    fetch, write, grbm, mfma = m("FETCH_SIZE"), m("WRITE_SIZE"), m("GRBM_GUI_ACTIVE"), m("SQ_VALU_MFMA_BUSY_CYCLES")
    e = {"calls": len(us), "avg_us": round(mean(us), 1), "total_us": round(sum(us), 1)}
    if fetch is not None and write is not None:
        b = (2 * fetch + write) * 1024
        e["hbm_MB_per_launch"] = round(b / 1e6, 1)
        e["hbm_TBps"] = round(b / (mean(us) * 1e-6) / 1e12, 2)
    if grbm and mfma is not None:
        e["mfma_busy"] = round(mfma / (1024 * grbm / 8), 3)
    out[f"{k} grid {grid}"] = e
json.dump(out, open(os.path.join(dst, f"{tag}_pmc_by_shape.json"), "w"), indent=1)
for k, v in out.items():
    print(k, json.dumps(v))

"""Per-kernel SQ counter sums from rocprofv3 sqlite outputs (tools/sq_pass.sh): mean per dispatch.
usage: python tools/sq_summary.py gpurun_out/TAG_p1 gpurun_out/TAG_p2 ... [--kernels REGEX]"""
import collections
import glob
import re
import sqlite3
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
rx = re.compile(sys.argv[sys.argv.index("--kernels") + 1] if "--kernels" in sys.argv else r"h32|wgrad_s")
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in args:
    for db in glob.glob(d + "/*.db"):
        c = sqlite3.connect(db)
        for name, disp, cname, val in c.execute(
                "select kernel_name, dispatch_id, counter_name, sum(value) from counters_collection "
                "group by dispatch_id, counter_name"):
            if rx.search(name):
                acc[name][cname].append(val)
for k, cs in acc.items():
    print(k)
    m = {n: sum(v) / len(v) for n, v in cs.items()}
    for n in sorted(m):
        print(f"   {n:28s} {m[n]:16.4g}")
    w = m.get("SQ_WAVE_CYCLES")
    if w:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC"):
            if n in m:
                print(f"   {n:28s} / WAVE_CYCLES = {m[n] / w:.3f}")

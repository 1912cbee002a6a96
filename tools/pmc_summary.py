"""Summarise a tools/profile.sh run into profiles/<tag>_*.json/csv (committed evidence).

traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 B  — FETCH_SIZE (KB) reads half of a wide
coalesced streaming read on gfx950 (MI355X_MICROARCH.md, HBM section), WRITE_SIZE is exact for
16-B-per-lane stores; effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration.
"""
import csv, collections, json, os, shutil, sys

src, tag = sys.argv[1], sys.argv[2]
suffix = sys.argv[3] if len(sys.argv) > 3 else ""  # "_split" / "_f16x2" for the other precision modes
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(root, "profiles")
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
short = lambda n: n.split("(")[0].replace("void ", "").replace("nof::", "")
stats = {short(r["Name"]): r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv")))}
agg = collections.defaultdict(list)
for sub in ("pmc_fetch", "pmc_write", "pmc_clk"):
    p = os.path.join(src, sub, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    for r in csv.DictReader(open(p)):
        agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
out = {}
for k, s in stats.items():
    if not k.startswith("k_"):
        continue
    avg_ns = float(s["AverageNs"])
    m = lambda c: (sum(agg[(k, c)]) / len(agg[(k, c)])) if agg.get((k, c)) else None
    fetch, write, grbm = m("FETCH_SIZE"), m("WRITE_SIZE"), m("GRBM_GUI_ACTIVE")
    e = {"calls": int(s["Calls"]), "avg_ms": avg_ns / 1e6}
    if fetch is not None and write is not None:
        e["hbm_bytes_per_launch"] = (2 * fetch + write) * 1024
        e["hbm_GBps"] = e["hbm_bytes_per_launch"] / (avg_ns * 1e-9) / 1e9
    if grbm is not None:
        e["eff_clock_GHz"] = grbm / 8 / (avg_ns * 1e-9) / 1e9
    out[k] = e
json.dump(out, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
# traffic lookup used by bench.py (bench kernel-timer names; split-mode kernels keyed with "_split")
names = {"k_mlp_fwd16<true>": "mlp_fwd", "k_mlp_bwd16": "mlp_bwd", "k_wgrad": "wgrad",
         "k_mlp_fwd16<0, true>": "mlp_fwd", "k_mlp_bwd16<0>": "mlp_bwd",
         "k_mlp_fwd16<2, true>": "mlp_fwd_f16x2", "k_mlp_bwd16<2>": "mlp_bwd_f16x2",
         "k_mlp_fwd<true, true>": "mlp_fwd_split", "k_mlp_bwd<true>": "mlp_bwd_split", "k_wgrad_x3": "wgrad_split",
         "k_mlp_fwd<1, true>": "mlp_fwd_split", "k_mlp_bwd<1>": "mlp_bwd_split", "k_wgrad_x3<1>": "wgrad_split",
         "k_mlp_fwd<2, true>": "mlp_fwd_f16x2", "k_mlp_bwd<2>": "mlp_bwd_f16x2", "k_wgrad_h": "wgrad_f16x2",
         "k_render_fwd<2>": "render_fwd" + suffix, "k_render_bwd<2>": "render_bwd" + suffix}
tfile = os.path.join(dst, "pmc_traffic.json")
traffic = json.load(open(tfile)) if os.path.exists(tfile) else {}
traffic.update({names[k]: v.get("hbm_bytes_per_launch") for k, v in out.items() if k in names})
json.dump(traffic, open(tfile, "w"), indent=1, sort_keys=True)
for k, v in out.items():
    print(k, json.dumps(v))

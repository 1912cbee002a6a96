"""Summarise a tools/profile_r02.sh (or ab_write.sh) run into profiles/<tag>_*.json/csv (committed
evidence) and the lookups bench.py reads (profiles/pmc_traffic.json, profiles/pmc_mfma.json).

traffic per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 B  — FETCH_SIZE (KB) reads half of a wide
coalesced streaming read on gfx950 (MI355X_MICROARCH.md, HBM section), WRITE_SIZE is exact for
16-B-per-lane stores.
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x kernel cycles), kernel cycles =
GRBM_GUI_ACTIVE / 8 XCDs (rocprofv3 sums GRBM over the XCDs).
effective clock = GRBM_GUI_ACTIVE / 8 / kernel duration — reported only for dispatches of at least
0.3 ms: the quotient reads high on shorter ones (MI355X_MICROARCH.md, DVFS), and it is never above
the 2.4 GHz peak clock by construction (a larger quotient is dropped as unreliable).

usage: pmc_summary.py SRC_DIR TAG [SUFFIX]   (SRC_DIR holds trace/ and pmc_*/ subdirectories)
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

SIMDS = 1024          # 256 CUs x 4 SIMDs
XCDS = 8
PEAK_CLOCK_GHZ = 2.4
MIN_CLOCK_MS = 0.3

src, tag = sys.argv[1], sys.argv[2]
suffix = sys.argv[3] if len(sys.argv) > 3 else ""  # "_split" / "_f16x2" / "_integrator"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.environ.get("NOF_PROFILES_DIR") or os.path.join(root, "profiles")  # override: tests
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
short = lambda n: n.split("(")[0].replace("void ", "").replace("nof::", "")
stats = {short(r["Name"]): r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv")))}
agg = collections.defaultdict(list)
for p in glob.glob(os.path.join(src, "pmc_*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(p)):
        agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
out = {}
for k, s in stats.items():
    if not k.startswith("k_"):
        continue
    avg_ns = float(s["AverageNs"])
    m = lambda c: (sum(agg[(k, c)]) / len(agg[(k, c)])) if agg.get((k, c)) else None
    fetch, write, grbm, mfma = m("FETCH_SIZE"), m("WRITE_SIZE"), m("GRBM_GUI_ACTIVE"), m("SQ_VALU_MFMA_BUSY_CYCLES")
    lds, ldsc = m("SQ_LDS_IDX_ACTIVE"), m("SQ_LDS_BANK_CONFLICT")
    e = {"calls": int(s["Calls"]), "avg_ms": avg_ns / 1e6}
    if lds is not None:
        # LDS-array cycles summed over the CUs, against 256 CUs x the kernel's GPU cycles (GRBM_GUI_ACTIVE
        # / 8): the fraction of CU-cycles the LDS array is busy (1.0 = 256 B/clk/CU for ds_read_b128)
        e["lds_idx_active"] = lds
        e["lds_bank_conflict"] = ldsc
        if grbm:
            e["lds_busy"] = round(lds / (256 * grbm / XCDS), 4)
    if fetch is not None and write is not None:
        e["hbm_bytes_per_launch"] = (2 * fetch + write) * 1024
        e["hbm_GBps"] = e["hbm_bytes_per_launch"] / (avg_ns * 1e-9) / 1e9
    if grbm is not None:
        cycles = grbm / XCDS
        clk = cycles / (avg_ns * 1e-9) / 1e9
        if avg_ns * 1e-6 >= MIN_CLOCK_MS and clk <= PEAK_CLOCK_GHZ:
            e["eff_clock_GHz"] = round(clk, 3)
        else:
            e["eff_clock_GHz"] = None
            e["eff_clock_note"] = "dispatch < 0.3 ms: GRBM_GUI_ACTIVE quotient unreliable"
        if mfma is not None:
            e["mfma_busy_cycles"] = mfma
            e["mfma_busy"] = round(mfma / (SIMDS * cycles), 4)  # fraction of SIMD-cycles with an MFMA busy
    out[k] = e
json.dump(out, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
# lookups read by bench.py (bench kernel-timer names; other precision modes keyed with "_<mode>")
names = {"k_mlp_fwd16<0, true>": "mlp_fwd", "k_mlp_bwd16<0>": "mlp_bwd", "k_wgrad": "wgrad",
         "k_mlp_fwd16<2, true>": "mlp_fwd_f16x2", "k_mlp_bwd16<2>": "mlp_bwd_f16x2",
         "k_mlp_fwd_h32<true>": "mlp_fwd_f16", "k_mlp_bwd_h32": "mlp_bwd_f16", "k_wgrad_s": "wgrad_f16",
         "k_wgrad_h": "wgrad_f16x2",
         "k_mlp_fwd<1, true>": "mlp_fwd_split", "k_mlp_bwd<1>": "mlp_bwd_split", "k_wgrad_x3<1>": "wgrad_split",
         "k_mlp_fwd16<3, true>": "mlp_fwd_f16split", "k_mlp_bwd16<3>": "mlp_bwd_f16split",
         "k_wgrad_x3<2>": "wgrad_f16split",
         "k_render_fwd<2>": "render_fwd" + suffix, "k_render_bwd<2>": "render_bwd" + suffix}
for fname, key in (("pmc_traffic.json", "hbm_bytes_per_launch"), ("pmc_mfma.json", "mfma_busy")):
    f = os.path.join(dst, fname)
    table = json.load(open(f)) if os.path.exists(f) else {}
    table.update({names[k]: v[key] for k, v in out.items() if k in names and v.get(key) is not None})
    table["_source"] = f"profiles/{tag}_pmc.json (tools/pmc_summary.py)"
    json.dump(table, open(f, "w"), indent=1, sort_keys=True)
for k, v in out.items():
    print(k, json.dumps(v))

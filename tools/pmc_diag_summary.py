"""Summarise tools/pmc_diag.sh: per kernel, average per launch of each SQ counter."""
import collections, csv, glob, json, os, sys

src = sys.argv[1]
agg = collections.defaultdict(list)
for p in glob.glob(os.path.join(src, "p*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("nof::", "")
        agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
out = collections.defaultdict(dict)
for (k, c), v in agg.items():
    if k.startswith("k_mlp") or k.startswith("k_wgrad"):
        out[k][c] = sum(v) / len(v)
json.dump(out, open(os.path.join(src, "summary.json"), "w"), indent=1)
for k, d in sorted(out.items()):
    print(k)
    for c in sorted(d):
        print(f"   {c:28s} {d[c]:.4g}")

#!/bin/bash
# Diagnostic counter passes (instruction cache, waits, LDS) on the MLP kernels, one --pmc pass each.
# usage: tools/pmc_diag2.sh TAG [precisions...]   -> gpurun_out/diag2_TAG/<prec>/<pass>/run_counter_collection.csv
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-x}; shift
OUT=gpurun_out/diag2_$TAG
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-integrator --no-alt --no-config4 --no-config5"
for p in ${*:-f32 f16x2}; do
  for pass in "ic:SQC_ICACHE_REQ SQC_ICACHE_MISSES" "wait:SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU" "act:SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS"; do
    name=${pass%%:*}; ctr=${pass#*:}
    echo "$(date +%T) $p $name" >> $OUT/progress.log
    timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/$p/$name -o run --output-format csv -- python3 bench.py $ARGS --precision $p > $OUT/${p}_$name.log 2>&1 || { echo "FAILED $p $name"; tail -5 $OUT/${p}_$name.log; exit 1; }
  done
done
python3 - "$OUT" <<'PY'
import collections, csv, glob, os, sys
out = sys.argv[1]
for prec in sorted(os.listdir(out)):
    d = os.path.join(out, prec)
    if not os.path.isdir(d): continue
    agg = collections.defaultdict(list)
    for p in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("nof::", "")
            if "mlp" in k or "wgrad" in k:
                agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    print("==", prec)
    for (k, c), v in sorted(agg.items()):
        print(f"{k:34s} {c:28s} {sum(v)/len(v):16.4g}")
PY

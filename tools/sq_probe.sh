#!/bin/bash
# SQ / cache counter passes over one quick_perf run (GPU box, repo root).  tools/sq_probe.sh OUT SPP [env...]
OUT=$1; SPP=$2; shift 2
R=$(pwd)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_VALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_BRANCH" \
           "TCC_HIT TCC_MISS TCP_TCC_READ_REQ TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ_LATENCY"; do
  i=$((i+1))
  env "$@" timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $R/$OUT/p$i -o run -- python3 $R/tools/quick_perf.py -s $SPP --reps 1 > $R/$OUT/p$i.log 2>&1 || { tail -5 $R/$OUT/p$i.log; exit 1; }
done
cd $R
python3 - $OUT <<'PY'
import csv, collections, sys, glob
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    if "k_render" not in k and "k_wf" not in k and "k_splat" not in k: continue
    wc = d.get("SQ_WAVE_CYCLES", 0) or 1
    print(k)
    print("  " + " ".join("%s=%.4g" % (n, v) for n, v in sorted(d.items())))
    av = d.get("SQ_ACTIVE_INST_VALU", 0)
    if av: print("  valu_active/wave_cyc=%.3f lane_util=%.3f lds_active=%.3f vmem_active=%.3f wait_any=%.3f wait_inst=%.3f"
                 % (av / wc, d.get("SQ_THREAD_CYCLES_VALU", 0) / (av * 64), d.get("SQ_ACTIVE_INST_LDS", 0) / wc,
                    d.get("SQ_ACTIVE_INST_VMEM", 0) / wc, d.get("SQ_WAIT_ANY", 0) / wc, d.get("SQ_WAIT_INST_ANY", 0) / wc))
PY

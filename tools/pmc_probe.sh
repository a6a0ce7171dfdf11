#!/bin/bash
# PMC counter passes over one quick_perf render (GPU box, repo root), one rocprofv3 run per set:
#   tools/pmc_probe.sh OUT SPP "COUNTERS SET 1" "COUNTERS SET 2" ...   (env passes through)
OUT=$1; SPP=$2; shift 2
R=$(pwd)
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/$OUT/p$i -o run -- python3 $R/tools/quick_perf.py -s $SPP --reps 1 > $R/$OUT/p$i.log 2>&1 || { tail -5 $R/$OUT/p$i.log; exit 1; }
done
cd $R && python3 - $OUT <<'PY'
import csv, glob, collections, sys
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    if "k_render" in k or "k_splat" in k:
        print(k)
        print("   " + " ".join("%s=%.4g" % kv for kv in sorted(d.items())))
PY

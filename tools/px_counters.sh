#!/bin/bash
# SQ instruction counters of k_render for one pixel rectangle (GPU box, repo root):
#   tools/px_counters.sh OUT X Y W H SPP
OUT=$1; shift
R=$(pwd)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/$OUT/p$i -o run -- python3 $R/tools/one_pixel.py "$@" > $R/$OUT/p$i.log 2>&1 || { tail -5 $R/$OUT/p$i.log; exit 1; }
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
    if "k_render" not in k: continue
    print(k)
    print("  " + " ".join("%s=%.4g" % (n, v) for n, v in sorted(d.items())))
PY

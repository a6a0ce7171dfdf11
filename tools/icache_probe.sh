cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ic
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES --output-format csv -d $R/gpurun_out/ic/p1 -o run -- python3 $R/tools/quick_perf.py -s 16 --reps 1 > $R/gpurun_out/ic/p1.log 2>&1 || { tail -5 $R/gpurun_out/ic/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_WAIT_ANY --output-format csv -d $R/gpurun_out/ic/p2 -o run -- python3 $R/tools/quick_perf.py -s 16 --reps 1 > $R/gpurun_out/ic/p2.log 2>&1 || { tail -5 $R/gpurun_out/ic/p2.log; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("gpurun_out/ic/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    if "k_render" in k or "k_splat" in k:
        print(k, " ".join("%s=%.4g" % kv for kv in sorted(d.items())))
PY

#!/bin/bash
# Per-kernel LatinSquare times (rocprofv3 kernel stats) of prebuilt variants on the C5 bench step:
#   tools/latin_kt.sh OUT CONFIG name1 name2 ...   (abbuild/<name>/libnart_hip.so; "main" = in-tree)
OUT=$1; CFG=$2; shift 2
R=$(pwd); mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$R"
for name in "$@"; do
  lib=abbuild/$name/libnart_hip.so; [ "$name" == "main" ] && lib=nart_amd/lib/libnart_hip.so
  NART_HIP_LIB=$lib timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$name -o run -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }
  echo "== $name"; python3 - $OUT/$name <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "latin" in n or "splat" in n or "render" in n or "primary" in n:
            print("%-50s calls %4s avg_ms %9.3f total_ms %9.3f" % (n[:50], r["Calls"], float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
PY
done

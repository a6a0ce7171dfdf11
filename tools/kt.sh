#!/bin/bash
# Kernel-trace timing of both path-tracer variants at SPP (GPU box, repo root): tools/kt.sh OUT SPP
OUT=$1; SPP=$2
R=$(pwd)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  NART_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/v$v -o run -- python3 $R/tools/quick_perf.py -s $SPP --reps 2 > $R/$OUT/v$v.log 2>&1 || { tail -5 $R/$OUT/v$v.log; exit 1; }
  echo "== variant $v"; head -4 $R/$OUT/v$v/run_kernel_stats.csv | cut -d, -f1-4
done

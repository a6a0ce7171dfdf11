#!/bin/bash
# Kernel trace of one rank's shard at N=8 (GPU box, repo root)
OUT=${1:-gpurun_out/shprof}
R=$(pwd); mkdir -p $OUT; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT -o run -- python3 $R/tools/shard_perf.py --ns 8 --rank 0 --reps 1 > $R/$OUT/log 2>&1 || { tail -5 $R/$OUT/log; exit 1; }
cut -d, -f1-4 $R/$OUT/run_kernel_stats.csv | head -14

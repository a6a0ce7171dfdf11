#!/bin/bash
# C3 1/2 shard, same box: k_splat_col4 + sample-major (default) vs two-band skewed splat + pixel-major.
for rep in 1 2; do
  timeout -k 10 300 python tools/shard_perf.py --config c3 --ns 2 --reps 2 > gpurun_out/c3n2_col4_$rep.log 2>&1 || exit 1
  NART_SPLAT_MODE=4 NART_SKEW_BANDS=2 timeout -k 10 300 python tools/shard_perf.py --config c3 --ns 2 --reps 2 > gpurun_out/c3n2_skew_$rep.log 2>&1 || exit 1
  echo "rep $rep col4: $(grep -o '"wall_ms": [0-9.]*\|"kernel_ms": [0-9.]*\|"splat_ms": [0-9.]*' gpurun_out/c3n2_col4_$rep.log | tr '\n' ' ') | skew2: $(grep -o '"wall_ms": [0-9.]*\|"kernel_ms": [0-9.]*\|"splat_ms": [0-9.]*' gpurun_out/c3n2_skew_$rep.log | tr '\n' ' ')"
done

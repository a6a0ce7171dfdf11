#!/bin/bash
# C4 1/8 shards: sampled probe (default 8 per group) vs every pixel (NART_PROBE_SUB=64), twice.
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r05ah_c4_probe_ab.log
: > $L
for v in 64 8 64 8; do
  export NART_PROBE_SUB=$v
  echo "== sub $v" >> $L
  timeout -k 10 300 python -u tools/shard_perf.py --config c4 --ns 8 --reps 1 >> $L 2>&1 || exit 1
done

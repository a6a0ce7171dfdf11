#!/bin/bash
# C5 volume kernel A/B on the GPU box: state machine (default) vs per-sample lock step, N=1 and 1/8 shard.
for v in 1 0; do
  echo "== NART_VOL_SM=$v"
  NART_VOL_SM=$v timeout -k 10 300 python tools/shard_perf.py --config c5 --ns 1 8 --rank 0 --reps 1 2>&1 | grep '^{' || exit 1
done

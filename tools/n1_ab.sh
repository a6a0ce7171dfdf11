#!/bin/bash
# Full-frame C3 kernel time of prebuilt variants (GPU box): tools/n1_ab.sh name...
for name in "$@"; do
  NART_HIP_LIB=$PWD/abbuild/$name/libnart_hip.so timeout -k 10 300 python -u tools/shard_perf.py --ns 1 --reps 2 > gpurun_out/n1.log 2>&1 || { tail -20 gpurun_out/n1.log; exit 1; }
  echo "$name $(grep '^{' gpurun_out/n1.log)"
done

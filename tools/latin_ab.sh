#!/bin/bash
# C5 LatinSquare time per prebuilt variant (GPU box): tools/latin_ab.sh name...
for name in "$@" "$1"; do
  NART_HIP_LIB=$PWD/abbuild/$name/libnart_hip.so timeout -k 10 300 python -u tools/shard_perf.py --config c5 --ns 1 --reps 2 > gpurun_out/lat.log 2>&1 || { tail -20 gpurun_out/lat.log; exit 1; }
  echo "[$name] $(grep '^{' gpurun_out/lat.log | cut -c1-160)"
done

#!/bin/bash
# Volume kernel occupancy A/B (prebuilt abbuild variants): C5 frame kernel ms and 1/8 shard.
OUT=${1:-gpurun_out/volw}; shift
mkdir -p $OUT
for v in "$@"; do
  NART_HIP_LIB=abbuild/$v/libnart_hip.so timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_$v.log 2>&1 || { tail -5 $OUT/c5_$v.log; exit 1; }
  NART_HIP_LIB=abbuild/$v/libnart_hip.so timeout -k 10 300 python tools/shard_perf.py --config c5 --ns 8 --reps 1 > $OUT/shard_$v.log 2>&1 || { tail -5 $OUT/shard_$v.log; exit 1; }
  echo "$v frame $(tail -n1 $OUT/c5_$v.log | grep -o '"kernel_ms_per_step": [0-9.]*') shard8 $(grep -o '"kernel_ms": [0-9.]*' $OUT/shard_$v.log | tr '\n' ' ')"
done

#!/bin/bash
# A/B of the splat kernels: col4 (mode 3) vs the tile-column sweep (mode 5) at prefetch depths 4/8/16
for cfg in c3 c5; do
  NART_HIP_LIB=abbuild/sw8/libnart_hip.so NART_SPLAT_MODE=3 tools/gpu_step.sh sw_${cfg}_col4 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline || exit 1
  for v in sw4 sw8 sw16; do
    NART_HIP_LIB=abbuild/$v/libnart_hip.so NART_SPLAT_MODE=5 tools/gpu_step.sh sw_${cfg}_$v 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline || exit 1
  done
done

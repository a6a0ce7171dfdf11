#!/bin/bash
# A/B of the per-sample buffer layout: sample-major + k_splat_col4 vs pixel-major + the skewed
# splat schedule (groups of 10 tile columns; abbuild variants with 1/5/20), C3 and C5.
tools/gpu_step.sh lay_pytest 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "layout or pixel_major" || exit 1
for cfg in c3 c5; do
  tools/gpu_step.sh lay_${cfg}_sample 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline || exit 1
  NART_LAYOUT=pixel tools/gpu_step.sh lay_${cfg}_pixel10 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline || exit 1
  for v in skew1 skew5 skew20; do
    NART_LAYOUT=pixel NART_HIP_LIB=abbuild/$v/libnart_hip.so tools/gpu_step.sh lay_${cfg}_$v 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline || exit 1
  done
done

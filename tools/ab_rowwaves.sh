#!/bin/bash
# Splat lane map A/B: one wave per lane group across buckets (default) vs bucket-major lanes
tools/gpu_step.sh rw_pytest 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "splat or high_spp_frame or volume_integrator or pixel_major" || exit 1
for cfg in c3 c5; do
  tools/gpu_step.sh rw_${cfg}_on 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline || exit 1
  NART_SPLAT_ROWWAVES=0 tools/gpu_step.sh rw_${cfg}_off 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline || exit 1
done

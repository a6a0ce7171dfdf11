#!/bin/bash
# Pixels per lane in k_splat_col4 (abbuild variants), C3 256 spp and C5 (1024 spp) splat times.
for name in "$@"; do
  NART_HIP_LIB=abbuild/$name/libnart_hip.so timeout -k 10 300 python tools/quick_perf.py -s 256 --reps 2 | tail -1 | \
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name C3 splat_ms %.2f' % d['splat_ms'])" || exit 1
done

#!/bin/bash
# Splat: per-pixel lanes (mode 2) vs four pixels per lane (mode 3) with prefetch-depth variants.
for name in "$@"; do  # abbuild variants
  for m in 2 3; do
    NART_SPLAT_MODE=$m NART_HIP_LIB=abbuild/$name/libnart_hip.so timeout -k 10 300 python tools/quick_perf.py -s 256 --reps 2 | tail -1 | \
      python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name mode $m splat_ms %.2f' % d['splat_ms'])" || exit 1
  done
done

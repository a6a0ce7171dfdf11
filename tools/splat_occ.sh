#!/bin/bash
# Splat time vs occupancy (dynamic LDS padding limits resident blocks per CU), GPU box, repo root:
#   tools/splat_occ.sh SPP bytes1 bytes2 ...   (0 = no padding)
SPP=$1; shift
for b in "$@"; do
  NART_SPLAT_LDS=$b timeout -k 10 300 python tools/quick_perf.py -s $SPP --reps 2 | tail -1 | \
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lds $b kernel_ms %.2f splat_ms %.2f' % (d['kernel_ms'], d['splat_ms']))" || exit 1
done

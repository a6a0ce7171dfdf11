#!/bin/bash
# Splat arithmetic modes on the GPU box (NART_SPLAT_MODE 0 direct, 1 thresholds, 2 thresholds + pow2 bucket, 3 four pixels per lane).
SPP=${1:-256}
for m in 2 3; do
  NART_SPLAT_MODE=$m timeout -k 10 300 python tools/quick_perf.py -s $SPP --reps 2 | tail -1 | \
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print('mode $m kernel_ms %.2f splat_ms %.2f' % (d['kernel_ms'], d['splat_ms']))" || exit 1
done

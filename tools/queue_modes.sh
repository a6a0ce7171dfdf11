#!/bin/bash
# C3 full-frame scheduling A/B on the GPU box (quorum kernel): slot order vs refill queues.
run() { env "$@" timeout -k 10 300 python tools/quick_perf.py -s 256 --reps 2 | tail -1 | \
  python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$* kernel_ms %.2f' % d['kernel_ms'])"; }
run NART_X=0 || exit 1
run NART_QUEUE=1 || exit 1
run NART_QUEUE_K=8 || exit 1
run NART_QUEUE_K=32 || exit 1

#!/bin/bash
# Speculative pairs: costly pixels per first-round wave (NART_QUEUE_K) sweep on C3 shards (rank 0).
set -o pipefail
mkdir -p gpurun_out/pairs
for cfg in "1 4" "1 16" "1 32" "0 16" "0 32"; do
  set -- $cfg
  NART_RQ_PAIRS=$1 NART_QUEUE_K=$2 timeout -k 10 300 python -u tools/shard_perf.py --ns 4 8 --reps 2 --rank 0 > gpurun_out/pairs/k_$1_$2.log 2>&1 || { tail -20 gpurun_out/pairs/k_$1_$2.log; exit 1; }
  grep '^{' gpurun_out/pairs/k_$1_$2.log | python3 -c "
import json,sys
print('pairs=$1 k=$2', ' '.join('N%d:%.1f' % (d['n'], d['worst']['kernel_ms']) for d in map(json.loads, sys.stdin)))"
done

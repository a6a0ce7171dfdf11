#!/bin/bash
# Sweep the costly-pixels-per-wave factor of the queue scheduler (GPU box): tools/k_sweep.sh LIB K...
export NART_HIP_LIB=$PWD/abbuild/$1/libnart_hip.so; shift
for k in "$@"; do
  NART_QUEUE_K=$k timeout -k 10 300 python -u tools/shard_perf.py --ns 2 4 8 --reps 1 --rank 0 > gpurun_out/ks.log 2>&1 || { tail -20 gpurun_out/ks.log; exit 1; }
  grep '^{' gpurun_out/ks.log | python -c "
import json,sys
print('k=$k', ' '.join('N%d:%.1f' % (d['n'], d['worst']['kernel_ms']) for d in map(json.loads, sys.stdin)))"
done

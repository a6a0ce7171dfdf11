#!/bin/bash
# Per-rank shard kernel time of prebuilt variants (GPU box): tools/shard_ab.sh "2 4 8" name...
NS=$1; shift
for name in "$@"; do
  NART_HIP_LIB=$PWD/abbuild/$name/libnart_hip.so timeout -k 10 300 python -u tools/shard_perf.py --ns $NS --reps 1 --rank 0 > gpurun_out/sab.log 2>&1 || { tail -20 gpurun_out/sab.log; exit 1; }
  grep '^{' gpurun_out/sab.log | python -c "
import json,sys
print('$name', ' '.join('N%d:%.1f' % (d['n'], d['worst']['kernel_ms']) for d in map(json.loads, sys.stdin)))"
done

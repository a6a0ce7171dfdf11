#!/bin/bash
# A/B of prebuilt variants (GPU box): C3 and Cornell at 64 spp, plus the 1/8 C3 shard (rank 0).
#   tools/ab2.sh name1 name2 ...
set -o pipefail
for name in "$@"; do
  bash tools/ab_run.sh 64 $name || exit 1
  bash tools/ab_run.sh 64 --scene cornell $name || exit 1
  NART_HIP_LIB=$PWD/abbuild/$name/libnart_hip.so timeout -k 10 300 python -u tools/shard_perf.py --ns 8 4 --reps 2 --rank 0 > gpurun_out/ab2_$name.log 2>&1 || { tail -20 gpurun_out/ab2_$name.log; exit 1; }
  grep '^{' gpurun_out/ab2_$name.log | python3 -c "
import json,sys
print('$name shard', ' '.join('N%d:%.1f' % (d['n'], d['worst']['kernel_ms']) for d in map(json.loads, sys.stdin)))"
done

#!/bin/bash
# Full-frame C3 time under run-time switches (GPU box): tools/env_ab.sh "ENV=1 ENV2=0" "..." ...
for e in "$@"; do
  env $e timeout -k 10 300 python -u tools/shard_perf.py --ns 1 --reps 2 > gpurun_out/envab.log 2>&1 || { tail -20 gpurun_out/envab.log; exit 1; }
  echo "[$e] $(grep '^{' gpurun_out/envab.log)"
done

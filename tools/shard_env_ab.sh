#!/bin/bash
# C3 shard time of rank r at N (GPU box): tools/shard_env_ab.sh N "ENV=..." ...
N=$1; shift
for e in "$@"; do
  env $e timeout -k 10 300 python -u tools/shard_perf.py --ns $N --reps 2 > gpurun_out/senv.log 2>&1 || { tail -20 gpurun_out/senv.log; exit 1; }
  echo "[N=$N $e] $(grep '^{' gpurun_out/senv.log | cut -c1-140)"
done

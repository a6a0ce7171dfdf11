#!/bin/bash
# Quorum A/B on the other configs (GPU box): tools/quorum_cfg.sh lib1 lib2 ...
for name in "$@"; do
  for c in c4 c2; do
    echo "== $name $c"
    NART_HIP_LIB=abbuild/$name/libnart_hip.so timeout -k 10 300 python tools/shard_perf.py --config $c --ns $([ $c == c4 ] && echo 8 || echo 1) --rank 0 --reps 1 2>&1 | grep '^{' || exit 1
  done
done

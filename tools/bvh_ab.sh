#!/bin/bash
# BVH build-parameter sweep (GPU box, repo root): tools/bvh_ab.sh SPP "ENV=.. ENV=.." ...
SPP=$1; shift
for spec in "$@"; do
  echo "== $spec"
  env $spec timeout -k 10 300 python tools/quick_perf.py -s $SPP --reps 2 --counters | tail -2 | python -c "
import json,sys
l=[json.loads(x) for x in sys.stdin.read().split(chr(10)) if x.strip()]
a,b=l
print('kernel_ms %.2f  nodes/s %.2f tris/s %.2f' % (a['kernel_ms'], b['node_visits_per_sample'], b['tri_tests_per_sample']))" || exit 1
done

#!/bin/bash
# Priority lanes A/B on small C3 shards (GPU box, repo root): queue tests, then rank-0 shard
# kernel times with NART_RQ_PRIO=0/1 and a few costly-pixels-per-wave settings.
set -o pipefail
mkdir -p gpurun_out/prio
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "queue" -x -v --timeout 200 --timeout-method thread > gpurun_out/prio/pytest.log 2>&1 || { tail -30 gpurun_out/prio/pytest.log; exit 1; }
tail -2 gpurun_out/prio/pytest.log
for cfg in "0 8" "1 8" "1 16" "1 32" "1 4"; do
  set -- $cfg
  NART_RQ_PRIO=$1 NART_QUEUE_K=$2 timeout -k 10 300 python -u tools/shard_perf.py --ns 2 4 8 --reps 2 --rank 0 > gpurun_out/prio/s_$1_$2.log 2>&1 || { tail -20 gpurun_out/prio/s_$1_$2.log; exit 1; }
  grep '^{' gpurun_out/prio/s_$1_$2.log | python3 -c "
import json,sys
print('prio=$1 k=$2', ' '.join('N%d:%.1f/%.1f' % (d['n'], d['worst']['kernel_ms'], d['worst']['wall_ms']) for d in map(json.loads, sys.stdin)))"
done

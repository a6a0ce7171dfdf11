#!/bin/bash
# Speculative pairs (GPU box, repo root): queue parity tests, then rank-0 shard kernel times of
# C3 at N=2/4/8 with NART_RQ_PAIRS=0/1.
set -o pipefail
mkdir -p gpurun_out/pairs
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "queue" -x -v --timeout 300 --timeout-method thread > gpurun_out/pairs/pytest.log 2>&1 || { tail -30 gpurun_out/pairs/pytest.log; exit 1; }
tail -2 gpurun_out/pairs/pytest.log
for cfg in "0" "1"; do
  NART_RQ_PAIRS=$cfg timeout -k 10 300 python -u tools/shard_perf.py --ns 2 4 8 --reps 2 --rank 0 > gpurun_out/pairs/s_$cfg.log 2>&1 || { tail -20 gpurun_out/pairs/s_$cfg.log; exit 1; }
  grep '^{' gpurun_out/pairs/s_$cfg.log | python3 -c "
import json,sys
print('pairs=$cfg', ' '.join('N%d:%.1f/%.1f' % (d['n'], d['worst']['kernel_ms'], d['worst']['wall_ms']) for d in map(json.loads, sys.stdin)))"
done

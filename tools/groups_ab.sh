#!/bin/bash
# Wave-group refill A/B (GPU box): full GPU parity suite, then C3 256 spp and Cornell 64 spp
# kernel times with NART_RQ_GROUPS=0/1.
set -o pipefail
mkdir -p gpurun_out/groups
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/groups/pytest.log 2>&1 || { tail -30 gpurun_out/groups/pytest.log; exit 1; }
tail -2 gpurun_out/groups/pytest.log
for g in 0 1 0 1; do
  NART_RQ_GROUPS=$g timeout -k 10 300 python tools/quick_perf.py -s 256 --reps 2 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('groups=$g C3 kernel_ms %.2f splat_ms %.2f' % (d['kernel_ms'], d['splat_ms']))" || exit 1
  NART_RQ_GROUPS=$g timeout -k 10 300 python tools/quick_perf.py -s 64 --scene cornell --reps 2 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('groups=$g C2 kernel_ms %.2f' % (d['kernel_ms']))" || exit 1
done

#!/bin/bash
# round 5: k_splat_rows with grouped LUT reads + select accumulation (PF 4 default, PF 8 variant)
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05g_pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "splat"
step r05g_c5 300 python -u tools/shard_perf.py --config c5 --ns 4 8 --reps 2 --rank 0
NART_HIP_LIB=abbuild/rpf8/libnart_hip.so step r05g_c5_pf8 300 python -u tools/shard_perf.py --config c5 --ns 4 8 --reps 2 --rank 0
step r05g_c3 300 python -u tools/shard_perf.py --config c3 --ns 2 4 8 --reps 2 --rank 0
NART_HIP_LIB=abbuild/rpf8/libnart_hip.so step r05g_c3_pf8 300 python -u tools/shard_perf.py --config c3 --ns 2 4 8 --reps 2 --rank 0

for v in 8 24 64; do
  NART_RQ_PRIO_ONLY=$v step r05g_prio_only$v 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2
done
step r05g_prio_only0 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2
echo all-done2

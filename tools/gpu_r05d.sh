#!/bin/bash
# round 5: early traversal-phase exit for priority lanes (NART_RQ_EARLY) on the C3 1/8 shard;
# glassSphere at bounces 10 vs 32 (overflow-list build)
step() { tools/gpu_step.sh "$@" || exit 1; }
for e in 0 1 2 4 8; do
  NART_RQ_EARLY=$e step r05d_early$e 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2
done
step r05d_b10 300 python -u tools/quick_perf.py -s 256 --reps 2 --bounces 10
step r05d_b32 300 python -u tools/quick_perf.py -s 256 --reps 2 --bounces 32
echo all-done

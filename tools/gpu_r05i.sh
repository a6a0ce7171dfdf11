#!/bin/bash
# round 5: NART_RQ_HALF + NART_RQ_SETPRIO with 4 / 6 / 8 / 12 costly pixels per first-round wave
# (NART_QUEUE_K), C3 1/8 shard all ranks; base twice (run-to-run spread)
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05i_base1 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2
for k in 4 6 8 12; do
  NART_QUEUE_K=$k NART_RQ_HALF=1 NART_RQ_SETPRIO=1 step r05i_hs_k$k 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2
done
step r05i_base2 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2
NART_RQ_HALF=1 NART_RQ_SETPRIO=1 step r05i_hs_c3n4 300 python -u tools/shard_perf.py --config c3 --ns 4 --reps 2
step r05i_base_c3n4 300 python -u tools/shard_perf.py --config c3 --ns 4 --reps 2
echo all-done

#!/bin/bash
# round 5: scheduling of the costliest chains on the C3 1/8 shard (all ranks): costly pixels on
# one wave per SIMD (NART_RQ_HALF), raised issue priority (NART_RQ_SETPRIO), four lanes for each
# first-round wave's costliest pixel (NART_RQ_QUAD); parity of each first
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05h_pytest 300 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "speculative_pairs"
step r05h_base 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2
NART_RQ_QUAD=1 step r05h_quad 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2
NART_RQ_SETPRIO=1 step r05h_setprio 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2
NART_RQ_HALF=1 step r05h_half 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2
NART_RQ_HALF=1 NART_RQ_SETPRIO=1 step r05h_half_setprio 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2
NART_RQ_QUAD=1 NART_RQ_SETPRIO=1 step r05h_quad_setprio 300 python -u tools/shard_perf.py --config c3 --ns 8 --reps 2
echo all-done

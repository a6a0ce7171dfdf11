#!/bin/bash
# round 5: k_splat_rows (splat mode 5) parity + small-launch A/B against k_splat_col4
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05e_pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "splat or frame"
step r05e_c5_rows 300 python -u tools/shard_perf.py --config c5 --ns 2 4 8 --reps 2 --rank 0
NART_SPLAT_SMALL=col4 step r05e_c5_col4 300 python -u tools/shard_perf.py --config c5 --ns 2 4 8 --reps 2 --rank 0
step r05e_c3_rows 300 python -u tools/shard_perf.py --config c3 --ns 2 4 8 --reps 2 --rank 0
NART_SPLAT_SMALL=col4 step r05e_c3_col4 300 python -u tools/shard_perf.py --config c3 --ns 2 4 8 --reps 2 --rank 0
echo all-done

#!/bin/bash
# round 5: whole GPU suite after the kernel diet (IList overflow columns, retired variants), then
# the C3 bench and the C3 shard timings
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05c_pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step r05c_bench 300 python -u bench.py
step r05c_shard_c3 300 python -u tools/shard_perf.py --config c3 --ns 1 8 --reps 2
echo all-done

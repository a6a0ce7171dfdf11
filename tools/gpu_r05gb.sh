#!/bin/bash
# round 5 final sweep, part 2: the four bench lines (reading the r05ga summaries), the one-process
# multi-device mode at N=1, per-rank shard timings of C3 / C5 / C4 at 1/2/4/8 ranks
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05gb_bench 300 python -u bench.py
step r05gb_bench_c2 300 python -u bench.py --config c2
step r05gb_bench_c5 300 python -u bench.py --config c5
step r05gb_bench_c4 400 python -u bench.py --config c4 --steps 2
step r05gb_bench_oneproc 300 python -u bench.py --one-process --gpus 1 --no-cpu-baseline
step r05gb_shard_c3 300 python -u tools/shard_perf.py --config c3 --ns 1 2 4 8 --reps 2
step r05gb_shard_c5 300 python -u tools/shard_perf.py --config c5 --ns 1 2 4 8 --reps 2
step r05gb_shard_c4 500 python -u tools/shard_perf.py --config c4 --ns 1 2 4 8 --reps 1
echo all-done

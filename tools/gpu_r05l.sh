#!/bin/bash
# round 5 checkpoint (part 2): C4 bench line, per-rank shard timings of C3 / C5 / C4 at 1/2/4/8 ranks
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05l_bench_c4 400 python -u bench.py --config c4 --steps 2
step r05l_shard_c3 300 python -u tools/shard_perf.py --config c3 --ns 1 2 4 8 --reps 2
step r05l_shard_c5 300 python -u tools/shard_perf.py --config c5 --ns 1 2 4 8 --reps 2
step r05l_shard_c4 500 python -u tools/shard_perf.py --config c4 --ns 1 2 4 8 --reps 1
echo all-done

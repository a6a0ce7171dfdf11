#!/bin/bash
# round 5: rocprofv3 kernel statistics + FETCH_SIZE / WRITE_SIZE / SQ passes of the C3, C4 and C5
# bench commands (one step each), and the C3 2-rank shards again (rank-0 spread check)
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05m_prof_c3 600 bash tools/profile.sh gpurun_out/prof_r05m_c3
step r05m_prof_c5 600 bash tools/profile.sh gpurun_out/prof_r05m_c5 --config c5 --steps 1 --warmup 0 --no-cpu-baseline
step r05m_prof_c4 900 bash tools/profile.sh gpurun_out/prof_r05m_c4 --config c4 --steps 1 --warmup 0 --no-cpu-baseline
step r05m_shard_c3n2 300 python -u tools/shard_perf.py --config c3 --ns 2 --reps 3
echo all-done

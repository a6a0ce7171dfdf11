#!/bin/bash
# round 5: splat weight records (gtab, default build) vs the d2-cell LUT (abbuild/lut0)
step() { tools/gpu_step.sh "$@" || exit 1; }
step r05a_pytest_splat 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "splat or frame"
step r05a_shard_c5_gtab 300 python -u tools/shard_perf.py --config c5 --ns 1 8 --reps 2 --rank 0
NART_HIP_LIB=abbuild/lut0/libnart_hip.so step r05a_shard_c5_lut 300 python -u tools/shard_perf.py --config c5 --ns 1 8 --reps 2 --rank 0
step r05a_shard_c3_gtab 300 python -u tools/shard_perf.py --config c3 --ns 1 8 --reps 2 --rank 0
NART_HIP_LIB=abbuild/lut0/libnart_hip.so step r05a_shard_c3_lut 300 python -u tools/shard_perf.py --config c3 --ns 1 8 --reps 2 --rank 0
echo all-done

#!/bin/bash
# k_splat_skew: wave-uniform all-rows branch.  Splat parity, then C5/C3 A/B (full frames).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r05r_skew_uniform_ab.log
: > $L
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "splat or skew" > gpurun_out/r05r_pytest_splat.log 2>&1 \
 && for v in new base new base; do
      if [ $v = base ]; then export NART_HIP_LIB=abbuild/nouni/libnart_hip.so; else unset NART_HIP_LIB; fi
      echo "== $v" >> $L
      timeout -k 10 200 python -u tools/shard_perf.py --config c5 --ns 1 --reps 2 >> $L 2>&1 || exit 1
      timeout -k 10 200 python -u tools/shard_perf.py --config c3 --ns 1 --reps 2 >> $L 2>&1 || exit 1
    done

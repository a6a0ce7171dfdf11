#!/bin/bash
# Volume kernel next-sample prefetch: parity, then C5 A/B (full frame and the 1/8 shard's worst rank).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r05p_vol_prefetch_ab.log
: > $L
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "volume or vol" > gpurun_out/r05p_pytest_vol.log 2>&1 \
 && for v in new base new base; do
      if [ $v = base ]; then export NART_HIP_LIB=abbuild/nopf/libnart_hip.so; else unset NART_HIP_LIB; fi
      echo "== $v c5" >> $L
      timeout -k 10 200 python -u tools/shard_perf.py --config c5 --ns 1 8 --reps 2 >> $L 2>&1 || exit 1
    done

#!/bin/bash
# LatinSquare second-half three-stage replay: parity tests, then C5/C4/C3 A/B (shard_perf N=1).
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r05o_latin_half_ab.log
: > $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "latin" > gpurun_out/r05o_pytest_latin.log 2>&1 \
 && for cfg in c5 c4c3; do :; done \
 && for v in new base new base; do
      if [ $v = base ]; then export NART_HIP_LIB=abbuild/nohalf/libnart_hip.so; else unset NART_HIP_LIB; fi
      echo "== $v c5" >> $L
      timeout -k 10 200 python -u tools/shard_perf.py --config c5 --ns 1 --reps 2 >> $L 2>&1 || exit 1
    done \
 && for v in new base; do
      if [ $v = base ]; then export NART_HIP_LIB=abbuild/nohalf/libnart_hip.so; else unset NART_HIP_LIB; fi
      echo "== $v c3" >> $L
      timeout -k 10 200 python -u tools/shard_perf.py --config c3 --ns 1 --reps 2 >> $L 2>&1 || exit 1
    done

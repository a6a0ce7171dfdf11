#!/bin/bash
# Register top-of-stack in the traversal.  Parity suite, then C3 A/B (full + every 1/8 shard), C4.
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r05v_stack_top_ab.log
: > $L
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r05v_pytest_parity.log 2>&1 || exit 1
for v in new base new base; do
  if [ $v = base ]; then export NART_HIP_LIB=abbuild/nostk/libnart_hip.so; else unset NART_HIP_LIB; fi
  echo "== $v" >> $L
  timeout -k 10 300 python -u tools/shard_perf.py --config c3 --ns 1 8 --reps 2 >> $L 2>&1 || exit 1
  timeout -k 10 120 python -u tools/quick_perf.py --scene c4 -w 1920 -H 1080 -s 32 --reps 2 >> $L 2>&1 || exit 1
done

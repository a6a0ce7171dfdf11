#!/bin/bash
# Single-light EstimateDirect path in the environment-light build (NART_ONE_LIGHT_ENV).  Environment parity
# tests, then C4 per-kernel times (1080p/32) and the C4 4K/512 frame, new vs base.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_frames.py -k "env or c4 or texture" > gpurun_out/r05al_pytest.log 2>&1 || exit 1
L=$R/gpurun_out/r05al_c4.log
: > $L
for v in new base new base; do
  if [ $v = base ]; then export NART_HIP_LIB=$R/abbuild/no1l/libnart_hip.so; else unset NART_HIP_LIB; fi
  echo "== $v" >> $L
  timeout -k 10 300 python -u tools/shard_perf.py --config c4 --ns 1 8 --reps 1 >> $L 2>&1 || exit 1
done

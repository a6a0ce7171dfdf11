#!/bin/bash
# Single-light EstimateDirect path in the area-light builds too (variant all1l = NART_ONE_LIGHT_ALL=1).
# Parity (glass / Cornell scenes in the parity suite), then C3 / C2 whole frames and C3 1/8 shards.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
export NART_HIP_LIB=$R/abbuild/all1l/libnart_hip.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r05am_pytest.log 2>&1 || exit 1
L=$R/gpurun_out/r05am_one_light_all.log
: > $L
for v in new base new base; do
  if [ $v = base ]; then unset NART_HIP_LIB; else export NART_HIP_LIB=$R/abbuild/all1l/libnart_hip.so; fi
  echo "== $v" >> $L
  timeout -k 10 300 python -u tools/shard_perf.py --config c3 --ns 1 8 --reps 2 >> $L 2>&1 || exit 1
  timeout -k 10 300 python -u tools/shard_perf.py --config c2 --ns 1 --reps 2 >> $L 2>&1 || exit 1
done

#!/bin/bash
# Sampled cost probe for the wave-group order (NART_PROBE_SUB 8 vs 64 = every pixel): frame wall
# time of C3 / C2 / C4 whole frames, and the GPU parity suite.
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/r05ac_probe_sub_ab.log
: > $L
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_frames.py -k "not c4 and not c5" > gpurun_out/r05ac_pytest.log 2>&1 || exit 1
for v in 8 64 8 64; do
  export NART_PROBE_SUB=$v
  for c in c3 c2 c4; do
    echo "== sub $v $c" >> $L
    timeout -k 10 200 python -u tools/shard_perf.py --config $c --ns 1 --reps $([ $c = c4 ] && echo 1 || echo 3) >> $L 2>&1 || exit 1
  done
done

#!/bin/bash
# Speculative lane groups of 4: parity, chain latency, 1/8 C3 shard (GPU box).
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "queue" > gpurun_out/quad_pytest.log 2>&1 || { tail -30 gpurun_out/quad_pytest.log; exit 1; }
tail -1 gpurun_out/quad_pytest.log
timeout -k 10 200 python -u tools/pair_latency.py 256 > gpurun_out/quad_lat.log 2>&1 || { tail -20 gpurun_out/quad_lat.log; exit 1; }
grep rect gpurun_out/quad_lat.log
for v in main q4 main q4; do
  if [ $v == main ]; then L=$PWD/nart_amd/lib/libnart_hip.so; else L=$PWD/abbuild/$v/libnart_hip.so; fi
  NART_HIP_LIB=$L timeout -k 10 300 python -u tools/shard_perf.py --ns 8 --reps 2 > gpurun_out/quad.log 2>&1 || { tail -20 gpurun_out/quad.log; exit 1; }
  echo "[$v] $(grep '^{' gpurun_out/quad.log | cut -c1-150)"
done

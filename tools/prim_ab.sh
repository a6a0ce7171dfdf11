#!/bin/bash
# k_primary refill vs lock step: parity tests on the main build, then C3 full-frame times (GPU box).
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "glass or cornell or refill or environment or materials" > gpurun_out/prim_pytest.log 2>&1 || { tail -30 gpurun_out/prim_pytest.log; exit 1; }
tail -1 gpurun_out/prim_pytest.log
for v in main prim0 main prim0; do
  if [ $v == main ]; then L=$PWD/nart_amd/lib/libnart_hip.so; else L=$PWD/abbuild/$v/libnart_hip.so; fi
  NART_HIP_LIB=$L timeout -k 10 300 python -u tools/shard_perf.py --ns 1 --reps 2 > gpurun_out/prim.log 2>&1 || { tail -20 gpurun_out/prim.log; exit 1; }
  echo "[$v] $(grep '^{' gpurun_out/prim.log | cut -c1-150)"
done

#!/bin/bash
# Wave-aligned splat buckets: splat parity tests, then C3 / C5 splat times per setting (GPU box).
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "splat or c1 or glass_sphere_64" > gpurun_out/sal_pytest.log 2>&1 || { tail -30 gpurun_out/sal_pytest.log; exit 1; }
tail -1 gpurun_out/sal_pytest.log
for a in 1 0 1 0; do
  NART_SPLAT_ALIGN=$a timeout -k 10 300 python -u tools/shard_perf.py --ns 1 --reps 2 > gpurun_out/sal.log 2>&1 || { tail -20 gpurun_out/sal.log; exit 1; }
  echo "[c3 align=$a] $(grep '^{' gpurun_out/sal.log | cut -c1-150)"
done
for a in 1 0; do
  NART_SPLAT_ALIGN=$a timeout -k 10 300 python -u tools/shard_perf.py --config c5 --ns 1 --reps 1 > gpurun_out/sal.log 2>&1 || { tail -20 gpurun_out/sal.log; exit 1; }
  echo "[c5 align=$a] $(grep '^{' gpurun_out/sal.log | cut -c1-150)"
done

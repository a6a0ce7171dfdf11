timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "volume" > gpurun_out/vw_pytest.log 2>&1; tail -1 gpurun_out/vw_pytest.log
for r in 1000 0; do
  NART_VOL_W4_ROUNDS=$r timeout -k 10 300 python tools/shard_perf.py --config c5 --ns 1 2 4 8 --reps 1 > gpurun_out/vw_shard_$r.log 2>&1 || exit 1
  echo "w4_rounds=$r $(grep -o '"n": [0-9]*\|"kernel_ms": [0-9.]*' gpurun_out/vw_shard_$r.log | tr '\n' ' ')"
done

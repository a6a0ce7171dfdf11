#!/bin/bash
# Volume kernel slow-phase quorum A/B (NART_VOL_QUORUM): parity tests, C5 frame and 1/8 shard.
OUT=${1:-gpurun_out/volq}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "volume or skew" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for q in 0 8 16 32; do
  NART_VOL_QUORUM=$q timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c5_q$q.log 2>&1 || { tail -5 $OUT/c5_q$q.log; exit 1; }
  NART_VOL_QUORUM=$q timeout -k 10 300 python tools/shard_perf.py --config c5 --ns 8 4 --reps 1 > $OUT/shard_q$q.log 2>&1 || { tail -5 $OUT/shard_q$q.log; exit 1; }
  echo "q=$q frame $(tail -n1 $OUT/c5_q$q.log | grep -o '"kernel_ms_per_step": [0-9.]*') shards $(grep -o '"n": [0-9]*\|"kernel_ms": [0-9.]*' $OUT/shard_q$q.log | tr '\n' ' ')"
done

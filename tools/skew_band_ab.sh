#!/bin/bash
# k_splat_skew tile-row bands A/B (NART_SKEW_BANDS 1 / 2): parity, C5 / C3 frames, forced-skew shards.
OUT=${1:-gpurun_out/band}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "splat or skew or framebuffer" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for c in c5 c3; do for b in 1 2; do
  NART_SKEW_BANDS=$b timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > $OUT/${c}_b$b.log 2>&1 || { tail -5 $OUT/${c}_b$b.log; exit 1; }
  echo "$c bands=$b $(tail -n1 $OUT/${c}_b$b.log | grep -o '"splat_ms_per_step": [0-9.]*')"
done; done
for b in 1 2; do
  NART_SPLAT_MODE=4 NART_SKEW_BANDS=$b timeout -k 10 400 python tools/shard_perf.py --config c5 --ns 2 4 8 --reps 1 > $OUT/shard_c5_skew_b$b.log 2>&1 || exit 1
  echo "c5 forced skew bands=$b $(grep -o '"n": [0-9]*\|"splat_ms": [0-9.]*' $OUT/shard_c5_skew_b$b.log | tr '\n' ' ')"
done

#!/bin/bash
# Three-kernel LatinSquare (k_latin_draws/_perm/_emit) vs the single-kernel forms: parity + A/B.
OUT=${1:-gpurun_out/latin3}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "latin or high_spp or volume" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for c in c5 c3; do
  for m in -1 0 3; do
    NART_LATIN=$m timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > $OUT/${c}_m$m.log 2>&1 || { tail -5 $OUT/${c}_m$m.log; exit 1; }
    echo "$c NART_LATIN=$m $(tail -n1 $OUT/${c}_m$m.log | grep -o '"latin_ms_per_step": [0-9.]*\|"ms_per_step": [0-9.]*\|"bit_identical": [a-z]*' | tr '\n' ' ')"
  done
done
